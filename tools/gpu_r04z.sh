# round 4 (z): every GPU test and smoke after routing the remaining stream waits through the bounded waits
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04z
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
