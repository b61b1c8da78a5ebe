set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" > gpurun_out/fif_$tag.json 2> gpurun_out/fif_$tag.log || exit 1; }
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 64 --warmup 32 --sync-check-steps 0 --iso-steps 0"
for r in 1 2; do
run base_$r $B
run fg_f2_16_$r GPU_MAX_HW_QUEUES=8 KHP_LIB=ba_pathtracing_fur_amd/lib/variants/fg/libkirk_hip.so $B --frames-in-flight 2 --fuse 16
run fg_f2_32_$r GPU_MAX_HW_QUEUES=8 KHP_LIB=ba_pathtracing_fur_amd/lib/variants/fg/libkirk_hip.so $B --frames-in-flight 2 --fuse 32
run half_f2_32_$r GPU_MAX_HW_QUEUES=8 $B --frames-in-flight 2 --fuse 32
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/fif_*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["value"], d["frame"]["extend_ms"])
PY
