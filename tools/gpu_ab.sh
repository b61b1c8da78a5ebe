set -o pipefail
# usage (on the GPU box): TAG=x bash tools/gpu_ab.sh "<bench args A>" "<bench args B>" [tests -k expr]
# runs the selected GPU tests, then bench A, B, A, B (alternated against drift)
TAG=${TAG:-ab}
mkdir -p gpurun_out
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$3" > gpurun_out/ab_tests_$TAG.log 2>&1 || exit 1
fi
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $1 > gpurun_out/ab_${TAG}_A$r.json 2> gpurun_out/ab_${TAG}_A$r.log || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $2 > gpurun_out/ab_${TAG}_B$r.json 2> gpurun_out/ab_${TAG}_B$r.log || exit 1
done
python - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
for k in ("A1", "B1", "A2", "B2"):
    d = json.loads(open(f"gpurun_out/ab_{t}_{k}.json").read().strip().splitlines()[-1])
    f = d["frame"]
    print(k, d["value"], "sync", (d.get("sync_steps") or {}).get("value"), "shade_ms", f["shade_ms"], "ext", f["extend_ms"], "dev", f["device_ms"])
PY
