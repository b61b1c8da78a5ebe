"""Synchronous-call timing at the metric row (dev tool, GPU box): KIRK's GUI call
(1-spp khp_render + 8-bit texture) and the 8-spp synchronous pass through the
path kernel (path_kernel 2) and the automatic choice (0), with render-ahead on
(the default) and off, with the library in
KHP_LIB (tools/build_variant.sh) or the in-tree one.  Prints one JSON line of
median wall ms per call and the Msamples/s they give.
usage: [KHP_LIB=variants/libkirk_x.so] python tools/sync_calls.py [calls=8]"""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W, H, D = 1920, 1080, 5
ctx = HipContext(0)
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()
out = {"lib": os.path.basename(os.environ.get("KHP_LIB", "in-tree"))}
k = 0
CASES = (("gui", 1, 0, True, 1), ("gui_ra0", 1, 0, True, 0), ("sync8_pk2", 8, 2, False, 1),
         ("sync8_pk2_ra0", 8, 2, False, 0), ("sync8_auto", 8, 0, False, 1))
for name, spp, pk, tex, ra in CASES:
    ctx.set_params(path_kernel=pk, render_ahead=ra)
    ms = []
    for it in range(N + 2):
        t0 = time.perf_counter()
        ctx.render(W, H, spp, D, first_sample=k, readback=False)
        if tex:
            ctx.read_rgba8(W, H)
        ms.append((time.perf_counter() - t0) * 1e3)
        k += spp
    med = statistics.median(ms[2:])
    out[name] = {"ms": round(med, 3), "Msamples_s": round(W * H * spp / med / 1e3, 1),
                 "min_ms": round(min(ms[2:]), 3)}
from ba_pathtracing_fur_amd import native as Nat  # noqa: E402
for key, tmo in (("rgba8", None), ("tonemap_rgba8", Nat.Tonemap.defaults(gamma=2.2))):
    ctx.read_rgba8(W, H, tmo)
    ms = []
    for _ in range(7):
        t0 = time.perf_counter()
        ctx.read_rgba8(W, H, tmo)
        ms.append((time.perf_counter() - t0) * 1e3)
    out[key + "_ms"] = round(statistics.median(ms), 3)
print(json.dumps(out), flush=True)
ctx.close()
