set -o pipefail
# usage (on the GPU box): TAG=x bash tools/gpu_ab_flag.sh "<common bench args>" "<args A>" "<args B>" ...
# each variant's bench runs ROUNDS times (default 2), alternated against drift
TAG=${TAG:-ab}; COMMON=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "$@"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --gui-steps 0 --sync-check-steps 0 $COMMON $v > gpurun_out/ab_${TAG}_${i}_$r.json 2> gpurun_out/ab_${TAG}_${i}_$r.log || exit 1
    i=$((i+1))
  done
done
python3 - "$TAG" "$#" <<'PY'
import json, sys, os
t, n = sys.argv[1], int(sys.argv[2])
for i in range(n):
    out = []
    for r in range(1, int(os.environ.get("ROUNDS", "2")) + 1):
        d = json.loads(open(f"gpurun_out/ab_{t}_{i}_{r}.json").read().strip().splitlines()[-1])
        iso = (d.get("isolated") or {}).get("k_extend", {})
        out.append((d["value"], d["frame"]["extend_ms"], iso.get("ms_per_frame")))
    print(i, out)
PY
