set -o pipefail
# A/B on the GPU box: (TESTS=1: all GPU tests first), then per config "ENV=.. ENV=..|bench/probe args":
# bench line (N=1) + rank-0-of-8 frame time (scale probe).  CONFIGS is ';'-separated.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
  tail -2 gpurun_out/gpu_tests.log; [ $rc = 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_tests.log | head -20; exit 1; }
fi
IFS=';' read -ra CFG <<< "$CONFIGS"
i=0
for cfg in "${CFG[@]}"; do
  i=$((i+1))
  ev=${cfg%%|*}; args=""; [[ "$cfg" == *"|"* ]] && args=${cfg#*|}
  env $ev timeout -k 10 200 python3 $R/bench.py --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline $args 2>/dev/null > $R/gpurun_out/cfg_$i.json || exit 1
  pargs=""; [[ "$args" == *"--sync-steps"* ]] && pargs="--sync-steps"
  env $ev timeout -k 10 200 python3 $R/tools/scale_probe.py --nranks ${NR:-8} --ranks-max 2 --steps ${STEPS:-6} $pargs 2>/dev/null | grep -v scale_probe > $R/gpurun_out/cfgp_$i.json || exit 1
  python3 -c "
import json; d=json.load(open('$R/gpurun_out/cfg_$i.json')); f=d['frame']; p=json.loads(open('$R/gpurun_out/cfgp_$i.json').read().strip().splitlines()[-1])
print('$cfg |', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'avg', d['roofline']['avg_launch_ms'], '| N${NR:-8} rank ms', p['max_rank_ms'], 'proj', p['projected_msamples_s'])"
done
