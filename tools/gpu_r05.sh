mkdir -p gpurun_out/r05a
timeout -k 10 300 python -u -m pytest tests/test_multigpu.py tests/test_output.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r05a/tests.log 2>&1 || exit 1
timeout -k 10 300 env KHP_LIB=variants/libkirk_prof.so python -u tools/path_drain_probe.py 3 path_kernel=2 > gpurun_out/r05a/drain.jsonl 2> gpurun_out/r05a/drain.log || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.log
