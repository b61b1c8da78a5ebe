# round 4 (q): after the empty-rank gather fix -- every multi-GPU test (RCCL single rank, local groups, bench --gpus 2) and the edge cases
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04q
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_multigpu.py tests/test_gpu_parity.py -x -v --timeout 250 --timeout-method thread \
  -k "multigpu or edge_sizes or rank_without_tiles or fused_frames" > $O/tests.log 2>&1
