set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04ac
cd $R
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/r04ac/smoke.log 2>&1
