# round 4: chunk staggering probe (env KHP_CHUNK_STAGGER = b): parity, then the driver's command and the default bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ad
mkdir -p $O
cd $R
export GPU_MAX_HW_QUEUES=8
KHP_CHUNK_STAGGER=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "driver_batch or fused_full_size or path_chunking or chunked_and_instrumented or fused_frames" > $O/tests.log 2>&1
for r in 1 2; do
  for st in -1 1 2 3; do
    KHP_CHUNK_STAGGER=$st timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 > $O/drv_st${st}_$r.json 2> $O/drv_st${st}_$r.log
  done
done
