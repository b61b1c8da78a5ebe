# round 4: final validation -- every GPU test, smoke, the driver's command, the default bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04al
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.log
