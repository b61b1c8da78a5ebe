set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04h
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.log
for r in 1 2; do
  for v in base drain1 drain1r16; do
    if [ $v = base ]; then L=""; else L=$R/variants/libkirk_$v.so; fi
    timeout -k 10 120 env ${L:+KHP_LIB=$L} python3 tools/sync_trace.py 6 0 2 > $O/pk_${v}_$r.json 2> $O/pk_${v}_$r.log
  done
done
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.log
bash tools/profile.sh r04h trace fetch write
