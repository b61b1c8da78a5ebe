set -o pipefail
# usage (on the GPU box): TAG=r03a STEPS="tests smoke bench rays" bash tools/gpu_run.sh
TAG=${TAG:-r03}
mkdir -p gpurun_out
for s in ${STEPS:-tests smoke bench}; do
  case $s in
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1 ;;
    bench) timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit 1 ;;
    drv)   timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv_$TAG.json 2> gpurun_out/bench_drv_$TAG.log || exit 1 ;;
    rays)  timeout -k 10 300 python -u tools/dump_rays.py gpurun_out/rays_$TAG.npz > gpurun_out/rays_$TAG.log 2>&1 || exit 1 ;;
    binning) timeout -k 10 120 tools/calib/calib_binning 85000000 40975 5 > gpurun_out/binning_85M_$TAG.json && timeout -k 10 120 tools/calib/calib_binning 22500000 40975 5 > gpurun_out/binning_22M_$TAG.json || exit 1 ;;
  esac
  echo "step $s done"
done
