# round 4 (x): k_path register-pressure probes -- no per-lane ray counters (nocount), counters in LDS (ldscount),
# LDS counters + the any-hit limit in h.t (lean), HEAD
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04x
mkdir -p $O
cd $R
KHP_LIB=$R/variants/libkirk_lean.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread \
  -k "path_kernel or edge_sizes or tiny_and_degenerate" > $O/tests_lean.log 2>&1
for r in 1 2; do
  for v in base nocount ldscount lean; do
    if [ $v = base ]; then L=""; else L=$R/variants/libkirk_$v.so; fi
    timeout -k 10 150 env ${L:+KHP_LIB=$L} python3 tools/sync_trace.py 8 0 2 > $O/st_${v}_$r.json 2> $O/st_${v}_$r.log
  done
done
