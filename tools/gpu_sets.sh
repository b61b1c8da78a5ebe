set -o pipefail
# path-set A/B on the GPU box: parity tests, then bench + rank-0-of-8 probe per env combo (CONFIGS: ';'-separated env strings)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "path_sets or chunking or shards or progressive" > gpurun_out/gpu_sets_tests.log 2>&1 || { tail -30 gpurun_out/gpu_sets_tests.log; exit 1; }
tail -1 gpurun_out/gpu_sets_tests.log
IFS=';' read -ra CFG <<< "$CONFIGS"
i=0
for cfg in "${CFG[@]}"; do
  i=$((i+1))
  env $cfg timeout -k 10 200 python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline 2>/dev/null > $R/gpurun_out/set_$i.json || exit 1
  env $cfg timeout -k 10 200 python3 $R/tools/scale_probe.py --nranks 8 --ranks-max 2 --steps 3 2>/dev/null | grep -v scale_probe > $R/gpurun_out/setp_$i.json || exit 1
  python3 -c "
import json; d=json.load(open('$R/gpurun_out/set_$i.json')); f=d['frame']; p=json.loads(open('$R/gpurun_out/setp_$i.json').read().strip().splitlines()[-1])
print('$cfg |', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], '| N8 rank ms', p['max_rank_ms'], 'proj', p['projected_msamples_s'])"
done
