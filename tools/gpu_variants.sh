set -o pipefail
# usage (on the GPU box): TAG=x bash tools/gpu_variants.sh "<bench args>" base v1 v2 ...   (base = the in-tree library)
# each variant's bench runs twice, interleaved, against drift
TAG=${TAG:-var}; ARGS=$1; shift
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L="KHP_LIB=ba_pathtracing_fur_amd/lib/variants/$v/libkirk_hip.so"; fi
    env $L timeout -k 10 300 python -u bench.py --no-cpu-baseline $ARGS > gpurun_out/v_${TAG}_${v}_$r.json 2> gpurun_out/v_${TAG}_${v}_$r.log || exit 1
  done
done
python - "$TAG" "$@" <<'PY'
import json, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    vals = []
    for r in (1, 2):
        d = json.loads(open(f"gpurun_out/v_{t}_{v}_{r}.json").read().strip().splitlines()[-1])
        vals.append((d["value"], d["frame"]["extend_ms"], (d.get("isolated") or {}).get("k_extend", {}).get("ms_per_frame")))
    print(v, vals)
PY
