# round-5 GPU steps (usage on the box: bash tools/gpu_r05.sh <step> [tag])
set -o pipefail
T=${2:-r05}
mkdir -p gpurun_out/$T
case "$1" in
park)
  timeout -k 10 400 python -u -m pytest tests/test_output.py tests/test_multigpu.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/$T/tests_out.log 2>&1 || exit 1
  timeout -k 10 400 env KHP_LIB=variants/libkirk_pk24_16.so python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "path_kernel or edge_sizes or quirk_scenes" > gpurun_out/$T/tests_park.log 2>&1 || exit 1
  for r in 1 2; do
    for v in base pk24_16 pk16_8 pk32_0; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 200 python -u tools/sync_calls.py 8 >> gpurun_out/$T/sync_calls.jsonl 2>> gpurun_out/$T/sync_calls.log || exit 1
    done
  done
  timeout -k 10 300 env KHP_LIB=variants/libkirk_pk24_16prof.so python -u tools/path_drain_probe.py 2 path_kernel=2 > gpurun_out/$T/drain_pk24_16.jsonl 2> gpurun_out/$T/drain_pk.log
  ;;
dwide)
  ./tools/calib/logsum_bench > gpurun_out/$T/logsum_bench.txt 2>&1 || exit 1
  timeout -k 10 400 env KHP_LIB=variants/libkirk_dwide.so python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "path_kernel or edge_sizes or quirk_scenes" > gpurun_out/$T/tests_dwide.log 2>&1 || exit 1
  for r in 1 2; do
    for v in base dwide; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 200 python -u tools/sync_calls.py 8 >> gpurun_out/$T/sync_calls.jsonl 2>> gpurun_out/$T/sync_calls.log || exit 1
    done
  done
  timeout -k 10 300 env KHP_LIB=variants/libkirk_dwideprof.so python -u tools/path_drain_probe.py 2 > gpurun_out/$T/drain_dwide.jsonl 2> gpurun_out/$T/drain_dwide.log
  ;;
tmtrace)
  timeout -k 10 400 python -u -m pytest tests/test_output.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/$T/tests_out.log 2>&1 || exit 1
  env KHP_LIB=variants/libkirk_tmtrace.so timeout -k 10 200 python -u tools/sync_calls.py 2 > gpurun_out/$T/tmtrace.jsonl 2> gpurun_out/$T/tmtrace.log || exit 1
  ;;
esac
