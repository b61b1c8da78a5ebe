# round 4: k_shade block size probe (128 / 512 threads: 2x / 0.5x the block allocations) vs 256
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04ag
mkdir -p $O
cd $R
KHP_LIB=$R/variants/libkirk_sb128.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "frame_parity or fused_frames" > $O/tests_128.log 2>&1
KHP_LIB=$R/variants/libkirk_sb512.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "frame_parity or fused_frames" > $O/tests_512.log 2>&1
for r in 1 2; do
  for v in base sb128 sb512; do
    if [ $v = base ]; then L=""; else L=$R/variants/libkirk_$v.so; fi
    timeout -k 10 300 env ${L:+KHP_LIB=$L} python3 bench.py --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.log
  done
done
