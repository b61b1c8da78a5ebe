set -o pipefail
# usage (on the GPU box): TAG=x TESTS=1 bash tools/gpu_abn.sh <variant|main> ... -> (GPU tests with the main lib,)
# then bench.py (metric row) once per listed library in order, twice over (alternated against drift).
# A variant is ba_pathtracing_fur_amd/lib/variants/<name>/libkirk_hip.so (tools/build_variant.sh).
TAG=${TAG:-abn}
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abn_tests_$TAG.log 2>&1 || exit 1
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    if [ "$v" = main ]; then L=""; else L=ba_pathtracing_fur_amd/lib/variants/$v/libkirk_hip.so; fi
    KHP_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/abn_${TAG}_${v}_$r.json 2> gpurun_out/abn_${TAG}_${v}_$r.log || exit 1
  done
done
ROUNDS=${ROUNDS:-2} python - "$TAG" "$@" <<'PY'
import json, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    out = []
    for r in range(1, int(__import__("os").environ.get("ROUNDS", "2")) + 1):
        d = json.loads(open(f"gpurun_out/abn_{t}_{v}_{r}.json").read().strip().splitlines()[-1])
        out.append((d["value"], d["roofline"]["frac"], d["frame"]["extend_ms"]))
    print(v, out)
PY
