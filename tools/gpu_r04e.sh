set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04f
mkdir -p $O
cd $R
timeout -k 10 120 python3 tools/sync_trace.py 6 0 2 > $O/sync_pk0.json 2> $O/sync_pk0.log
timeout -k 10 120 env KHP_LIB=$R/variants/libkirk_pprof.so python3 tools/sync_trace.py 4 0 2 > $O/sync_pprof.json 2> $O/sync_pprof.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.log
timeout -k 5 90 env KHP_LIB=$R/variants/libkirk_commtrace.so python3 -u tools/comm_probe.py > $O/comm_probe.log 2>&1
