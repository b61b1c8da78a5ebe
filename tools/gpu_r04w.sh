# round 4 (w): path_order 2 = heavy-first TILES (recorded per-pixel costs): parity, synchronous calls, fused bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04w
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "tile_order or fused_frames or fused_full_size or path_kernel or params_are_validated" > $O/tests.log 2>&1
for r in 1 2; do
  for po in 1 2; do
    timeout -k 10 150 python3 tools/sync_trace.py 8 0 2 $po > $O/st_po${po}_$r.json 2> $O/st_po${po}_$r.log
  done
done
for po in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --path-order $po > $O/bench_po$po.json 2> $O/bench_po$po.err
done
