# round 4 (n): four-way any-hit step for wide shadow rays: parity, then A/B against the KIRK-order step (variant any4off)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04n
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_any4_$i.json 2> $O/bench_any4_$i.err
  timeout -k 10 300 env KHP_LIB=$R/variants/libkirk_any4off.so python -u bench.py --no-cpu-baseline > $O/bench_off_$i.json 2> $O/bench_off_$i.err
done
timeout -k 10 200 python -u tools/scale_probe.py --nranks 8 --steps 20 > $O/scale_any4.json 2> $O/scale_any4.err
timeout -k 10 200 env KHP_LIB=$R/variants/libkirk_any4off.so python -u tools/scale_probe.py --nranks 8 --steps 20 > $O/scale_off.json 2> $O/scale_off.err
