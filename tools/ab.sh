#!/bin/bash
# A/B tuning variants of libkirk_hip (built with `make variant`), same bench, sequential processes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
  lib=$R/ba_pathtracing_fur_amd/lib/libkirk_hip${v:+_$v}.so
  [ "$v" = "base" ] && lib=$R/ba_pathtracing_fur_amd/lib/libkirk_hip.so
  KHP_LIB=$lib timeout -k 10 300 python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline 2>/dev/null \
   | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['frame']; print('$v', d['value'], 'ext', f['extend_ms'], 'sh', f['shadow_ms'], 'shade', f['shade_ms'], 'spill/ray', f['stack_spills_per_ray'], 'pruned/ray', f.get('pruned_pops_per_ray'), f.get('shadow_pruned_pops_per_ray'), 'frac', d['roofline']['frac'])" || exit 1
done
