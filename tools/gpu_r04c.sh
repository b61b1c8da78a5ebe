set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04c
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "path_kernel or single_rank or errors" tests/test_multigpu.py -x -v --timeout 200 --timeout-method thread > $O/gpu_tests_new.log 2>&1
cd /tmp && export TMPDIR=/tmp
for v in "1 2" "2 2" "2 0"; do
  set -- $v
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_pk$1_wf$2 -o run -- python3 $R/tools/sync_trace.py 4 $1 $2 > $O/calls_pk$1_wf$2.json 2> $O/calls_pk$1_wf$2.log
done
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.log
