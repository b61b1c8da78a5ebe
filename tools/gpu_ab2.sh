set -o pipefail
# A/B of library variants: bench line + rank-0-of-8 frame time (scale probe) per variant
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc = 0 ] || exit 1
fi
for v in "$@"; do
  lib=$R/ba_pathtracing_fur_amd/lib/libkirk_hip${v:+_$v}.so
  [ "$v" = "base" ] && lib=$R/ba_pathtracing_fur_amd/lib/libkirk_hip.so
  KHP_LIB=$lib timeout -k 10 200 python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline 2>/dev/null > $R/gpurun_out/ab_$v.json || exit 1
  KHP_LIB=$lib timeout -k 10 200 python3 $R/tools/scale_probe.py --nranks 8 --ranks-max 2 --steps 3 2>/dev/null | grep -v scale_probe > $R/gpurun_out/abp_$v.json || exit 1
  python3 -c "
import json; d=json.load(open('$R/gpurun_out/ab_$v.json')); f=d['frame']; p=json.loads(open('$R/gpurun_out/abp_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], 'ms', d['ms_per_step'], 'ext', f['extend_ms'], 'sh', f['shadow_ms'], 'frac', d['roofline']['frac'], '| N8 rank ms', p['max_rank_ms'], 'proj', p['projected_msamples_s'])"
done
