set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_multigpu.py -x -v --timeout 250 --timeout-method thread > $O/multigpu_tests.log 2>&1
