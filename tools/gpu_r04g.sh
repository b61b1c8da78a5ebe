set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04g
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "fused_frames or single_rank or path_kernel_frames" tests/test_multigpu.py -x -v --timeout 200 --timeout-method thread > $O/gpu_tests_comm.log 2>&1
for r in 1 2; do
  for v in base noheavy heavy300 heavy1000; do
    if [ $v = base ]; then L=""; else L=$R/variants/libkirk_$v.so; fi
    timeout -k 10 120 env ${L:+KHP_LIB=$L} python3 tools/sync_trace.py 6 0 2 > $O/pk_${v}_$r.json 2> $O/pk_${v}_$r.log
  done
done
timeout -k 5 90 env KHP_LIB=$R/variants/libkirk_commtrace.so python3 -u tools/comm_probe.py > $O/comm_probe.log 2>&1
