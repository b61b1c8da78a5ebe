set -o pipefail
# usage (on the GPU box): TAG=x KNOB=--heavy-iters bash tools/gpu_knob_ab.sh v1 v2 ... -> bench.py (metric
# row) once per knob value in order, ROUNDS times over (alternated against drift), then a summary line per value.
TAG=${TAG:-knob}
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $KNOB $v $BENCH_ARGS > gpurun_out/knob_${TAG}_${v}_$r.json 2> gpurun_out/knob_${TAG}_${v}_$r.log || exit 1
  done
done
python - "$TAG" "$@" <<'PY'
import json, os, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    out = []
    for r in range(1, int(os.environ.get("ROUNDS", "2")) + 1):
        d = json.loads(open(f"gpurun_out/knob_{t}_{v}_{r}.json").read().strip().splitlines()[-1])
        out.append((d["value"], d["roofline"]["frac"], d["frame"]["extend_ms"]))
    print(v, out)
PY
