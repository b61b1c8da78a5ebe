set -o pipefail
# usage (on the GPU box): TAG=r02o bash tools/gpu_final.sh -> GPU tests + smoke, metric bench (with CPU baseline),
# per-config bench lines (1, 2, 3@16spp, 5), light-path variant line, rocprof trace + PMC passes
TAG=${TAG:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit 1
for c in 1 2 3 5; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/bench_cfg${c}_$TAG.json 2> gpurun_out/bench_cfg${c}_$TAG.log || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --bdpt 256,4 --steps 16 --warmup 8 > gpurun_out/bench_bdpt_$TAG.json 2> gpurun_out/bench_bdpt_$TAG.log || exit 1
bash tools/profile.sh $TAG trace fetch write sq
