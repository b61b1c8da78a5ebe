set -o pipefail
# usage (on the GPU box): TAG=r03h bash tools/gpu_configs_r3.sh -> smoke, metric bench (with CPU baseline),
# per-config bench lines (1, 2, 3@16spp, 5) and the light-path variant line
TAG=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.log || exit 1
echo "metric done"
for c in 1 2 3 5; do
  timeout -k 10 400 python -u bench.py --config $c --gui-steps 0 > gpurun_out/bench_cfg${c}_$TAG.json 2> gpurun_out/bench_cfg${c}_$TAG.log || exit 1
  echo "config $c done"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --gui-steps 0 --bdpt 256,4 --steps 16 --warmup 8 > gpurun_out/bench_bdpt_$TAG.json 2> gpurun_out/bench_bdpt_$TAG.log || exit 1
echo "bdpt done"
