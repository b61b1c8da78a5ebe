# round 4: size-aware automatic path kernel -- path-kernel tests and the bench's synchronous legs
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ab
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "path_kernel or edge_sizes or config3_stated" > $O/tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.log
