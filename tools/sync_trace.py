"""Synchronous khp_render calls for a rocprofv3 kernel trace (dev tool, GPU box).

KIRK's own usage is synchronous: PathTracer::render adds one sample per call
(CPU_PathTracer.cpp:17-52) and the GUI then reads the 8-bit texture.  This
runs the metric scene and, after a warmup, N calls of each pattern:
  gui  -- khp_render 1 spp (synchronous, no readback) + khp_read_rgba8
  sync -- khp_render 8 spp (synchronous, no readback)
printing each call's host wall time (perf_counter, ms) as one JSON line on
stdout, so tools/sync_breakdown.py can line the trace's kernels up with them.
usage: rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d D -o run -- \
         python3 tools/sync_trace.py [calls=4] [path_kernel=0] [wide_from=2] [path_order=1] > calls.json
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
PK = int(sys.argv[2]) if len(sys.argv) > 2 else 0
WF = int(sys.argv[3]) if len(sys.argv) > 3 else 2
PO = int(sys.argv[4]) if len(sys.argv) > 4 else 1
W, H, D = 1920, 1080, 5
ctx = HipContext(0)
ctx.set_params(path_kernel=PK, wide_from=WF, path_order=PO)
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()
k = 0
for _ in range(3):  # warmup: both patterns once, buffers allocated
    ctx.render(W, H, 1, D, first_sample=k, readback=False)
    ctx.read_rgba8(W, H)
    k += 1
    ctx.render(W, H, 8, D, first_sample=k, readback=False)
    k += 8
out = {"gui": [], "sync": [], "params": ctx.params()}
for name, spp, tex in (("gui", 1, True), ("sync", 8, False)):
    for _ in range(N):
        t0 = time.perf_counter()
        ctx.render(W, H, spp, D, first_sample=k, readback=False)
        t1 = time.perf_counter()
        if tex:
            ctx.read_rgba8(W, H)
        t2 = time.perf_counter()
        st = ctx.stats()
        out[name].append({"wall_ms": round((t2 - t0) * 1e3, 3), "render_ms": round((t1 - t0) * 1e3, 3),
                          "device_ms": round(st["render_ms"], 3), "extend_ms": round(st["extend_ms"], 3),
                          "shade_ms": round(st["shade_ms"], 3), "shadow_ms": round(st["shadow_ms"], 3),
                          "bounce_extend_ms": [round(x, 3) for x in st["bounce_extend_ms"][:D]],
                          "bounce_shadow_ms": [round(x, 3) for x in st["bounce_shadow_ms"][:D]],
                          "step_cycles": st["step_cycles"], "extend_rays": st["extend_rays"],
                          "shadow_rays": st["shadow_rays"]})
        k += spp
print(json.dumps(out), flush=True)
ctx.close()
