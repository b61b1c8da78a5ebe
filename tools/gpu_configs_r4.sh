set -o pipefail
# usage (on the GPU box): TAG=r04i bash tools/gpu_configs_r4.sh -> per-config bench lines (1, 2, 3@16spp, 5) and the light-path variant line
TAG=${TAG:-r04}
O=${GRAFT_REPO_ROOT:-.}/gpurun_out/cfg_$TAG
mkdir -p $O
for c in 1 2 3 5; do
  timeout -k 10 400 python -u bench.py --config $c --gui-steps 0 > $O/bench_cfg${c}.json 2> $O/bench_cfg${c}.log || exit 1
  echo "config $c done"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --gui-steps 0 --bdpt 256,4 --steps 16 --warmup 8 > $O/bench_bdpt.json 2> $O/bench_bdpt.log || exit 1
echo "bdpt done"
