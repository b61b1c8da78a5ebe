# round 4 (r): edge sizes incl. depth 20, empty-rank snapshots
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04r
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
  -k "edge_sizes or rank_without_tiles or tiny_and_degenerate" > $O/tests.log 2>&1
