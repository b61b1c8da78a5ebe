# round 4 (t): k_shade with wave-level queue allocation and one-wave blocks (variant shadewave) vs block_alloc4
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04t
mkdir -p $O
cd $R
KHP_LIB=$R/variants/libkirk_shadewave.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "frame_parity or fused_frames or driver_batch" > $O/tests_variant.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_base_$i.json 2> $O/bench_base_$i.err
  KHP_LIB=$R/variants/libkirk_shadewave.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_wave_$i.json 2> $O/bench_wave_$i.err
done
