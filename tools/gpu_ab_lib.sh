set -o pipefail
# usage (on the GPU box): TAG=x bash tools/gpu_ab_lib.sh "<common bench args>" default variants/libkirk_a.so ...
# each library's bench runs ROUNDS times (default 2), alternated against drift; "default" = the product build
TAG=${TAG:-abl}; COMMON=$1; shift
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for v in "$@"; do
    if [ "$v" = default ]; then L=""; else L="$v"; fi
    KHP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --gui-steps 0 --sync-check-steps 0 --iso-steps 0 $COMMON > gpurun_out/ab_${TAG}_${i}_$r.json 2> gpurun_out/ab_${TAG}_${i}_$r.log || exit 1
    i=$((i+1))
  done
done
python3 - "$TAG" "$@" <<'PY'
import json, sys, os
t, libs = sys.argv[1], sys.argv[2:]
for i, l in enumerate(libs):
    out = []
    for r in range(1, int(os.environ.get("ROUNDS", "2")) + 1):
        d = json.loads(open(f"gpurun_out/ab_{t}_{i}_{r}.json").read().strip().splitlines()[-1])
        out.append((d["value"], d["frame"]["extend_ms"]))
    print(i, l, out)
PY
