# round 4 (k): heavy-first pixel order (path_order 2): parity, then A/B against path_order 1
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04k
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "fused_frames or fused_full_size or params_are_validated" > $O/tests.log 2>&1
for i in 1 2; do
  for po in 1 2; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --path-order $po > $O/bench_po${po}_$i.json 2> $O/bench_po${po}_$i.err
  done
done
for po in 1 2; do
  timeout -k 10 300 python -u tools/scale_probe.py --nranks 1 8 --steps 20 --path-order $po > $O/scale_po$po.json 2> $O/scale_po$po.err
done
