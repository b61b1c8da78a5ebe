# round-5 GPU steps (usage on the box: bash tools/gpu_r05.sh <step> [tag])
set -o pipefail
T=${2:-r05}
mkdir -p gpurun_out/$T
case "$1" in
park)
  timeout -k 10 400 python -u -m pytest tests/test_output.py tests/test_multigpu.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/$T/tests_out.log 2>&1 || exit 1
  timeout -k 10 400 env KHP_LIB=variants/libkirk_pk24_16.so python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "path_kernel or edge_sizes or quirk_scenes" > gpurun_out/$T/tests_park.log 2>&1 || exit 1
  for r in 1 2; do
    for v in base pk24_16 pk16_8 pk32_0; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 200 python -u tools/sync_calls.py 8 >> gpurun_out/$T/sync_calls.jsonl 2>> gpurun_out/$T/sync_calls.log || exit 1
    done
  done
  timeout -k 10 300 env KHP_LIB=variants/libkirk_pk24_16prof.so python -u tools/path_drain_probe.py 2 path_kernel=2 > gpurun_out/$T/drain_pk24_16.jsonl 2> gpurun_out/$T/drain_pk.log
  ;;
dwide)
  ./tools/calib/logsum_bench > gpurun_out/$T/logsum_bench.txt 2>&1 || exit 1
  timeout -k 10 400 env KHP_LIB=variants/libkirk_dwide.so python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "path_kernel or edge_sizes or quirk_scenes" > gpurun_out/$T/tests_dwide.log 2>&1 || exit 1
  for r in 1 2; do
    for v in base dwide; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 200 python -u tools/sync_calls.py 8 >> gpurun_out/$T/sync_calls.jsonl 2>> gpurun_out/$T/sync_calls.log || exit 1
    done
  done
  timeout -k 10 300 env KHP_LIB=variants/libkirk_dwideprof.so python -u tools/path_drain_probe.py 2 > gpurun_out/$T/drain_dwide.jsonl 2> gpurun_out/$T/drain_dwide.log
  ;;
tmtrace)
  timeout -k 10 400 python -u -m pytest tests/test_output.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/$T/tests_out.log 2>&1 || exit 1
  env KHP_LIB=variants/libkirk_tmtrace.so timeout -k 10 200 python -u tools/sync_calls.py 2 > gpurun_out/$T/tmtrace.jsonl 2> gpurun_out/$T/tmtrace.log || exit 1
  ;;
ab)   # in-tree library (A) against variants/libkirk_<base>.so (B), alternated; $3 = B's name; $4 = bench args
  B=${3:-base}
  for r in 1 2; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $4 > gpurun_out/$T/ab_A$r.json 2> gpurun_out/$T/ab_A$r.log || exit 1
    env KHP_LIB=variants/libkirk_$B.so timeout -k 10 300 python -u bench.py --no-cpu-baseline $4 > gpurun_out/$T/ab_B$r.json 2> gpurun_out/$T/ab_B$r.log || exit 1
  done
  python - $T <<'PY'
import json, sys
t = sys.argv[1]
for k in ("A1", "B1", "A2", "B2"):
    d = json.loads(open(f"gpurun_out/{t}/ab_{k}.json").read().strip().splitlines()[-1])
    f = d["frame"]
    print(k, d["value"], "sync", (d.get("sync_steps") or {}).get("value"), "gui", (d.get("gui_steps") or {}).get("value"),
          "ext", f["extend_ms"], "b0/b1", [b["extend_ms"] for b in f["per_bounce"]], "dev", f["device_ms"],
          "iso_ext", (d.get("isolated") or {}).get("k_extend", {}).get("ms_per_frame"),
          "iso_sh", (d.get("isolated") or {}).get("k_shadow", {}).get("ms_per_frame"), "tm", (d.get("output_stage") or {}).get("tonemap_rgba8_ms"))
PY
  ;;
vars)   # the in-tree library and variants/libkirk_<v>.so for v in $3 (space-separated), alternated twice; $4 = bench args
  for r in 1 2; do
    for v in base $3; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 300 python -u bench.py --no-cpu-baseline $4 > gpurun_out/$T/v_${v}_$r.json 2> gpurun_out/$T/v_${v}_$r.log || exit 1
    done
  done
  python - $T base $3 <<'PY'
import json, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    for r in (1, 2):
        d = json.loads(open(f"gpurun_out/{t}/v_{v}_{r}.json").read().strip().splitlines()[-1])
        f = d["frame"]
        print(v, r, d["value"], "sync", (d.get("sync_steps") or {}).get("value"), "ext", f["extend_ms"],
              "per_bounce", [b["extend_ms"] for b in f["per_bounce"]], "shade", f["shade_ms"], "dev", f["device_ms"])
PY
  ;;
parity)
  # a variant library (KHP_LIB) is not named libkirk_hip.so: skip the mapping check then
  D=""; [ -n "$KHP_LIB" ] && D="--deselect tests/test_gpu_parity.py::test_native_library_is_loaded"
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu $D > gpurun_out/$T/tests_parity.log 2>&1 || exit 1
  ;;
r05r)   # fused shadow stage parity + A/B, octant keys, rank probe
  env KHP_LIB=variants/libkirk_fsh.so bash tools/gpu_r05.sh parity $T || exit 1
  mv gpurun_out/$T/tests_parity.log gpurun_out/$T/tests_parity_fsh.log
  env KHP_LIB=variants/libkirk_fsh5.so bash tools/gpu_r05.sh parity $T || exit 1
  mv gpurun_out/$T/tests_parity.log gpurun_out/$T/tests_parity_fsh5.log
  bash tools/gpu_r05.sh vars $T "fsh fsh5 oct" > gpurun_out/$T/vars.txt || exit 1
  env KHP_LIB=variants/libkirk_oct.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --ray-sort-from 1 > gpurun_out/$T/oct_rs1.json 2> gpurun_out/$T/oct_rs1.log || exit 1
  timeout -k 10 300 python -u tools/rank_probe.py > gpurun_out/$T/rank_probe.json 2> gpurun_out/$T/rank_probe.log || exit 1
  env KHP_LIB=variants/libkirk_fsh.so timeout -k 10 300 python -u tools/rank_probe.py > gpurun_out/$T/rank_probe_fsh.json 2> gpurun_out/$T/rank_probe_fsh.log || exit 1
  ;;
coop)   # cooperative leaf step: parity, GUI/synchronous calls (k_path), bench A/B (k_extend/k_shadow), rank probe
  env KHP_LIB=variants/libkirk_coopP32.so bash tools/gpu_r05.sh parity $T || exit 1
  mv gpurun_out/$T/tests_parity.log gpurun_out/$T/tests_parity_coopP32.log
  env KHP_LIB=variants/libkirk_coopT32.so bash tools/gpu_r05.sh parity $T || exit 1
  mv gpurun_out/$T/tests_parity.log gpurun_out/$T/tests_parity_coopT32.log
  for r in 1 2; do
    for v in base coopP16 coopP32 coopP48; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 200 python -u tools/sync_calls.py 8 >> gpurun_out/$T/sync_calls.jsonl 2>> gpurun_out/$T/sync_calls.log || exit 1
    done
  done
  bash tools/gpu_r05.sh vars $T "coopT32" > gpurun_out/$T/vars.txt || exit 1
  env KHP_LIB=variants/libkirk_coopT32.so timeout -k 10 300 python -u tools/rank_probe.py > gpurun_out/$T/rank_probe_coopT32.json 2> gpurun_out/$T/rank_probe_coopT32.log || exit 1
  ;;
one)   # one variant $3: parity, bench A/B, rank probe
  env KHP_LIB=variants/libkirk_$3.so bash tools/gpu_r05.sh parity $T || exit 1
  bash tools/gpu_r05.sh vars $T "$3" > gpurun_out/$T/vars.txt || exit 1
  timeout -k 10 300 python -u tools/rank_probe.py > gpurun_out/$T/rank_probe_base.json 2> gpurun_out/$T/rank_probe_base.log || exit 1
  env KHP_LIB=variants/libkirk_$3.so timeout -k 10 300 python -u tools/rank_probe.py > gpurun_out/$T/rank_probe_$3.json 2> gpurun_out/$T/rank_probe_$3.log || exit 1
  ;;
args)   # the in-tree library without / with bench args $3, alternated twice; then parity
  for r in 1 2; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T/v_base_$r.json 2> gpurun_out/$T/v_base_$r.log || exit 1
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $3 > gpurun_out/$T/v_args_$r.json 2> gpurun_out/$T/v_args_$r.log || exit 1
  done
  python - $T base args <<'PY' > gpurun_out/$T/vars.txt
import json, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    for r in (1, 2):
        d = json.loads(open(f"gpurun_out/{t}/v_{v}_{r}.json").read().strip().splitlines()[-1])
        f = d["frame"]
        print(v, r, d["value"], "sync", (d.get("sync_steps") or {}).get("value"), "ext", f["extend_ms"],
              "per_bounce", [b["extend_ms"] for b in f["per_bounce"]], "shade", f["shade_ms"], "dev", f["device_ms"],
              "iso_ext", d["isolated"]["k_extend"]["ms_per_frame"], "iso_sh", d["isolated"]["k_shadow"]["ms_per_frame"])
PY
  bash tools/gpu_r05.sh parity $T || exit 1
  ;;
cfgs)   # the configs' bench lines, then the instruction-mix PMC passes at the driver's shape
  for c in 1 2 3 5; do
    timeout -k 10 400 python -u bench.py --config $c > gpurun_out/$T/cfg$c.json 2> gpurun_out/$T/cfg$c.log || exit 1
  done
  STEPS=20 bash tools/profile.sh $T mix mix2 || exit 1
  ;;
cfgsort)   # configs 1 and 2 with and without ray regrouping, alternated; claim-block variants on the metric row
  for r in 1 2; do
    for c in 1 2; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c > gpurun_out/$T/cfg${c}_rs2_$r.json 2> gpurun_out/$T/cfg${c}_rs2_$r.log || exit 1
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c --ray-sort-from 0 > gpurun_out/$T/cfg${c}_rs0_$r.json 2> gpurun_out/$T/cfg${c}_rs0_$r.log || exit 1
    done
  done
  bash tools/gpu_r05.sh vars $T "cb8 cb11" > gpurun_out/$T/vars.txt || exit 1
  ;;
autosort)   # parity, then the configs and the metric row with the library defaults
  bash tools/gpu_r05.sh parity $T || exit 1
  for c in 1 2 metric; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --config $c > gpurun_out/$T/cfg$c.json 2> gpurun_out/$T/cfg$c.log || exit 1
  done
  ;;
args2)   # in-tree defaults vs bench args $3 vs bench args $4, alternated twice
  for r in 1 2; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T/v_base_$r.json 2> gpurun_out/$T/v_base_$r.log || exit 1
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $3 > gpurun_out/$T/v_a_$r.json 2> gpurun_out/$T/v_a_$r.log || exit 1
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $4 > gpurun_out/$T/v_b_$r.json 2> gpurun_out/$T/v_b_$r.log || exit 1
  done
  python - $T base a b <<'PY' > gpurun_out/$T/vars.txt
import json, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    for r in (1, 2):
        d = json.loads(open(f"gpurun_out/{t}/v_{v}_{r}.json").read().strip().splitlines()[-1])
        f = d["frame"]
        print(v, r, d["value"], "sync", (d.get("sync_steps") or {}).get("value"), "ext", f["extend_ms"],
              "per_bounce", [b["extend_ms"] for b in f["per_bounce"]], "shade", f["shade_ms"], "dev", f["device_ms"])
PY
  ;;
drv)   # variant $3: parity, then the driver's command alternated with the in-tree library 3 times
  env KHP_LIB=variants/libkirk_$3.so bash tools/gpu_r05.sh parity $T || exit 1
  for r in 1 2 3; do
    for v in base $3; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/$T/d_${v}_$r.json 2> gpurun_out/$T/d_${v}_$r.log || exit 1
    done
  done
  python - $T base $3 <<'PY' > gpurun_out/$T/vars.txt
import json, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    for r in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/{t}/d_{v}_{r}.json").read().strip().splitlines()[-1])
        f = d["frame"]
        print(v, r, d["value"], "sync", (d.get("sync_steps") or {}).get("value"), "ext", [b["extend_ms"] for b in f["per_bounce"]],
              "sh", [b["shadow_ms"] for b in f["per_bounce"]], "dev", f["device_ms"])
PY
  ;;
drv2)   # variants $3 and $4 [and $5]: the driver's command alternated with the in-tree library 2 times each
  for r in 1 2; do
    for v in base $3 $4 $5; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/$T/d_${v}_$r.json 2> gpurun_out/$T/d_${v}_$r.log || exit 1
    done
  done
  python - $T base $3 $4 $5 <<'PY' > gpurun_out/$T/vars.txt
import json, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    for r in (1, 2):
        d = json.loads(open(f"gpurun_out/{t}/d_{v}_{r}.json").read().strip().splitlines()[-1])
        f = d["frame"]
        print(v, r, d["value"], "ext", [b["extend_ms"] for b in f["per_bounce"]], "lane", [b["lane_use"] for b in f["per_bounce"]], "dev", f["device_ms"])
PY
  ;;
drvp)   # variant $3: parity, then the driver's command and the default bench alternated with the in-tree library
  env KHP_LIB=variants/libkirk_$3.so bash tools/gpu_r05.sh parity $T || exit 1
  env KHP_LIB=variants/libkirk_$3.so timeout -k 10 400 python -u -m pytest tests/test_output.py tests/test_multigpu.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/$T/tests_other.log 2>&1 || exit 1
  for r in 1 2; do
    for v in base $3; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/$T/d_${v}_$r.json 2> gpurun_out/$T/d_${v}_$r.log || exit 1
      env $L timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T/v_${v}_$r.json 2> gpurun_out/$T/v_${v}_$r.log || exit 1
    done
  done
  python - $T base $3 <<'PY' > gpurun_out/$T/vars.txt
import json, sys
t = sys.argv[1]
for v in sys.argv[2:]:
    for k in ("d", "v"):
        for r in (1, 2):
            d = json.loads(open(f"gpurun_out/{t}/{k}_{v}_{r}.json").read().strip().splitlines()[-1])
            f = d["frame"]
            print(v, k, r, d["value"], "sync", (d.get("sync_steps") or {}).get("value"), "ext", [b["extend_ms"] for b in f["per_bounce"]], "dev", f["device_ms"])
PY
  ;;
full)   # every GPU test, then the driver's bench command and the default one
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$T/bench_driver.json 2> gpurun_out/$T/bench_driver.log || exit 1
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.log || exit 1
  ;;
esac
