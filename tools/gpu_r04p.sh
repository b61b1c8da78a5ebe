# round 4 (p): edge sizes (1x1, ragged 37x23, depth 1), ranks without tiles, local-group gather with empty ranks
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multigpu.py -x -v --timeout 200 --timeout-method thread \
  -k "edge_sizes or rank_without_tiles or empty_ranks" > $O/tests.log 2>&1
