# round 4: k_shade (512-thread blocks) held to 6 waves per SIMD (3 blocks per CU instead of 2) vs unconstrained
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04am
mkdir -p $O
cd $R
KHP_LIB=$R/variants/libkirk_sw6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "frame_parity or fused_frames" > $O/tests_sw6.log 2>&1
for r in 1 2 3; do
  for v in base sw6; do
    if [ $v = base ]; then L=""; else L=$R/variants/libkirk_$v.so; fi
    timeout -k 10 300 env ${L:+KHP_LIB=$L} python3 bench.py --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.log
    timeout -k 10 300 env ${L:+KHP_LIB=$L} python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 > $O/d_${v}_$r.json 2> $O/d_${v}_$r.log
  done
done
