# round 4: validation with 512-thread k_shade blocks -- every GPU test, smoke, driver's command, default bench, configs 2 and 5
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ai
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.log
timeout -k 10 300 python3 bench.py --config 2 --no-cpu-baseline > $O/cfg2.json 2> $O/cfg2.log
timeout -k 10 400 python3 bench.py --config 5 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.log
