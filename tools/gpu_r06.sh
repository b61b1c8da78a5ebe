#!/bin/bash
# round-6 GPU steps (usage on the box: bash tools/gpu_r06.sh <step> [tag])
set -o pipefail
T=${2:-r06}
mkdir -p gpurun_out/$T
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
case "$1" in
ra)   # render-ahead: its tests, the path-kernel parity tests, then the synchronous-call timings
  KHP_NO_BUILD=1 timeout -k 10 500 $PYT tests/test_render_ahead.py > gpurun_out/$T/tests_ra.log 2>&1 || exit 1
  KHP_NO_BUILD=1 timeout -k 10 400 $PYT tests/test_gpu_parity.py -k "path_kernel or edge_sizes or quirk or progressive or tiny or pathtracer_api" > gpurun_out/$T/tests_pk.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/sync_calls.py 8 > gpurun_out/$T/sync_calls.jsonl 2> gpurun_out/$T/sync_calls.log || exit 1
  ;;
sync)  # synchronous-call timings only ($3: extra env, e.g. KHP_LIB=variants/libkirk_x.so)
  env $3 timeout -k 10 300 python -u tools/sync_calls.py 8 >> gpurun_out/$T/sync_calls.jsonl 2>> gpurun_out/$T/sync_calls.log || exit 1
  ;;
probe)  # tools/ra_probe.py over the in-tree library and variants/libkirk_<v>.so for v in $3; $4: render_ahead list
  for v in base $3; do
    if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
    env $L timeout -k 10 300 python -u tools/ra_probe.py 12 1,8 ${4:-1,0} >> gpurun_out/$T/ra_probe.jsonl 2>> gpurun_out/$T/ra_probe.log || exit 1
  done
  ;;
drain)  # per-wave k_path timelines with render-ahead on and off (variants/libkirk_prof.so)
  for ra in 1 0; do
    KHP_LIB=variants/libkirk_prof.so timeout -k 10 300 python -u tools/path_drain_probe.py 3 path_kernel=2 render_ahead=$ra >> gpurun_out/$T/drain.jsonl 2>> gpurun_out/$T/drain.log || exit 1
  done
  ;;
leaf)   # leaf-record reuse inside a wave (variants/libkirk_leafreuse.so)
  KHP_LIB=variants/libkirk_leafreuse.so timeout -k 10 300 python -u tools/leaf_reuse.py 8 > gpurun_out/$T/leaf_reuse.json 2> gpurun_out/$T/leaf_reuse.log || exit 1
  ;;
full)   # the whole GPU suite, then the driver's bench command
  KHP_NO_BUILD=1 timeout -k 10 1000 $PYT tests > gpurun_out/$T/gpu_tests.log 2>&1 || exit 1
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$T/bench_driver_cmd.json 2> gpurun_out/$T/bench.log || exit 1
  ;;
bench)  # the driver's bench command only
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$T/bench_driver_cmd.json 2> gpurun_out/$T/bench.log || exit 1
  ;;
vars)   # the driver's bench shape (fused passes only), in-tree vs variants/libkirk_<v>.so for v in $3, alternated twice
  for r in 1 2; do
    for v in base $3; do
      if [ $v = base ]; then L=""; else L="KHP_LIB=variants/libkirk_$v.so"; fi
      env $L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 > gpurun_out/$T/v_${v}_$r.json 2> gpurun_out/$T/v_${v}_$r.log || exit 1
    done
  done
  python - $T base $3 <<'PY'
import json, sys
t = sys.argv[1]
for r in (1, 2):
    for v in sys.argv[2:]:
        d = json.loads(open(f"gpurun_out/{t}/v_{v}_{r}.json").read().strip().splitlines()[-1])
        rl = d["roofline"]
        print(r, v, d["value"], "frac", rl["frac"], "b-ms", [b["ms_per_frame"] for b in rl["per_bounce"]])
PY
  ;;
knobs)  # the driver's bench shape with bench.py flag sets $3.. (each a quoted string), alternated twice
  shift 2
  for r in 1 2; do
    i=0
    for k in "$@"; do
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 $k > gpurun_out/$T/k${i}_$r.json 2> gpurun_out/$T/k${i}_$r.log || exit 1
      d=$(python -c "import json,sys; d=json.loads(open('gpurun_out/$T/k${i}_$r.json').read().strip().splitlines()[-1]); rl=d['roofline']; print(d['value'], rl['frac'], [b['ms_per_frame'] for b in rl['per_bounce']])")
      echo "$r [$k] $d" | tee -a gpurun_out/$T/knobs.txt
      i=$((i+1))
    done
  done
  ;;
fuse)   # fused-batch rate of F consecutive 8-spp passes (tools/fuse_probe.py), twice
  for r in 1 2; do
    timeout -k 10 300 python -u tools/fuse_probe.py 6 ${3:-1,2,3,4} >> gpurun_out/$T/fuse_probe.jsonl 2>> gpurun_out/$T/fuse_probe.log || exit 1
  done
  ;;
fuse1)  # the GUI call's pass (1 spp): fused batches through the path kernel and the wavefront, and single calls
  timeout -k 10 200 python -u tools/fuse_probe.py 8 1 1 2 2 >> gpurun_out/$T/fuse1.jsonl 2>> gpurun_out/$T/fuse1.log || exit 1
  timeout -k 10 200 python -u tools/fuse_probe.py 8 1,2,3,4,6,8 1 2 0 >> gpurun_out/$T/fuse1.jsonl 2>> gpurun_out/$T/fuse1.log || exit 1
  timeout -k 10 200 python -u tools/fuse_probe.py 8 3,4,6,8 1 1 0 >> gpurun_out/$T/fuse1.jsonl 2>> gpurun_out/$T/fuse1.log || exit 1
  ;;
envab)  # the driver's bench shape with environment settings $3.. (each a quoted string, "-" = none), alternated twice
  shift 2
  for r in 1 2; do
    i=0
    for e in "$@"; do
      E=$e; [ "$E" = "-" ] && E=""
      env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 > gpurun_out/$T/e${i}_$r.json 2> gpurun_out/$T/e${i}_$r.log || exit 1
      d=$(python -c "import json,sys; d=json.loads(open('gpurun_out/$T/e${i}_$r.json').read().strip().splitlines()[-1]); rl=d['roofline']; fr=d['frame']; print(d['value'], rl['frac'], [b['ms_per_frame'] for b in rl['per_bounce']], fr['device_ms'], fr['shade_ms'])")
      echo "$r [$e] $d" | tee -a gpurun_out/$T/envab.txt
      i=$((i+1))
    done
  done
  ;;
guiab)  # bench's GUI and sync lines with environment settings $3.. ("-" = none), alternated twice
  shift 2
  for r in 1 2; do
    i=0
    for e in "$@"; do
      E=""; A=""
      for t in $e; do case $t in -) ;; *=*) E="$E $t" ;; *) A="$A $t" ;; esac; done
      env $E timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --iso-steps 0 $A > gpurun_out/$T/g${i}_$r.json 2> gpurun_out/$T/g${i}_$r.log || exit 1
      d=$(python -c "import json,sys; d=json.loads(open('gpurun_out/$T/g${i}_$r.json').read().strip().splitlines()[-1]); g=d['gui_steps']; s=d['sync_steps']; print('gui', g['value'], g['ms_per_call'], 'sync', s['value'], 'gui_calls', g['call_ms'])")
      echo "$r [$e] $d" | tee -a gpurun_out/$T/guiab.txt
      i=$((i+1))
    done
  done
  ;;
tiles)  # rank-of-N projection (tools/scale_probe.py, the driver's 20 passes) per tile size $3..
  shift 2
  for t in "$@"; do
    timeout -k 10 300 python -u tools/scale_probe.py --nranks 1 8 --steps 20 --tile $t > gpurun_out/$T/scale_tile$t.txt 2>&1 || exit 1
  done
  ;;
fif)    # rank-of-8 projection with two batches in flight (fuse 10) and 8 hardware queues, vs the default
  timeout -k 10 300 python -u tools/scale_probe.py --nranks 1 8 --steps 20 > gpurun_out/$T/scale_base.txt 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/scale_probe.py --nranks 1 8 --steps 20 --set frames_in_flight=2 fuse_frames=10 > gpurun_out/$T/scale_fif2.txt 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u tools/scale_probe.py --nranks 1 8 --steps 20 --set frames_in_flight=2 fuse_frames=5 > gpurun_out/$T/scale_fif2f5.txt 2>&1 || exit 1
  ;;
chunks)  # default 32 passes and the driver's 20 with the automatic chunk cap vs an explicit 2^27 (round 5's), alternated
  for r in 1 2; do
    for c in 0 134217728; do
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 --chunk-paths $c > gpurun_out/$T/c32_${c}_$r.json 2> gpurun_out/$T/c32_${c}_$r.log || exit 1
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --sync-check-steps 0 --gui-steps 0 --iso-steps 0 --chunk-paths $c > gpurun_out/$T/c20_${c}_$r.json 2> gpurun_out/$T/c20_${c}_$r.log || exit 1
      python -c "import json; f=lambda n: json.loads(open(n).read().strip().splitlines()[-1]); a=f('gpurun_out/$T/c32_${c}_$r.json'); b=f('gpurun_out/$T/c20_${c}_$r.json'); print($r, 'chunk_paths', $c, '32 passes', a['value'], a['frame']['extend_launches'] if 'extend_launches' in a['frame'] else '', '20 passes', b['value'], b['roofline']['frac'])" | tee -a gpurun_out/$T/chunks.txt
    done
  done
  ;;
heavy)  # longest-first split off (heavy_iters 2^32-1) vs the default: sync/GUI lines and the rank-of-8 shares
  for r in 1 2; do
    for h in 160 4294967295; do
      timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --iso-steps 0 --gui-steps 0 --heavy-iters $h > gpurun_out/$T/h${h}_$r.json 2> gpurun_out/$T/h${h}_$r.log || exit 1
      python -c "import json; d=json.loads(open('gpurun_out/$T/h${h}_$r.json').read().strip().splitlines()[-1]); print($r, 'heavy_iters', $h, 'sync', d['sync_steps']['value'])" | tee -a gpurun_out/$T/heavy.txt
    done
  done
  for h in 160 4294967295; do
    timeout -k 10 300 python -u tools/scale_probe.py --nranks 8 --steps 20 --set heavy_iters=$h > gpurun_out/$T/scale_h$h.txt 2>&1 || exit 1
  done
  ;;
partests)  # the wavefront/path-kernel parity suites (render-ahead, hybrid, parity)
  KHP_NO_BUILD=1 timeout -k 10 900 $PYT tests/test_gpu_parity.py tests/test_render_ahead.py tests/test_hybrid_batches.py > gpurun_out/$T/tests_par.log 2>&1 || exit 1
  ;;
wra)    # render-ahead through fusion: its tests, the synchronous-call parity tests, then the bench's sync line
  KHP_NO_BUILD=1 timeout -k 10 700 $PYT tests/test_render_ahead.py > gpurun_out/$T/tests_ra.log 2>&1 || exit 1
  KHP_NO_BUILD=1 timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "progressive or ray_sorting or wide_records or chunked or fused" > gpurun_out/$T/tests_par.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --gui-steps 0 --iso-steps 0 > gpurun_out/$T/bench_sync.json 2> gpurun_out/$T/bench_sync.log || exit 1
  ;;
*) echo "unknown step $1"; exit 2 ;;
esac
