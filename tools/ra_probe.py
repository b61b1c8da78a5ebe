"""Render-ahead probe (dev tool, GPU box): per-call wall time and khp_stats.ahead_*
of KIRK's synchronous calls at the metric row -- the GUI call (1 spp + 8-bit
texture) and the 8-spp pass through the path kernel -- with render_ahead 1 and
0, with the library in KHP_LIB (tools/build_variant.sh) or the in-tree one.
usage: [KHP_LIB=variants/libkirk_x.so] python tools/ra_probe.py [calls=12] [spp list, default 1,8]
       [render_ahead list, default 1,0]"""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 12
SPPS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
RAS = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,0").split(",")]
W, H, D = 1920, 1080, 5
ctx = HipContext(0)
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()
lib = os.path.basename(os.environ.get("KHP_LIB", "in-tree"))
k = 0
for spp in SPPS:
    for ra in RAS:
        ctx.set_params(path_kernel=2, render_ahead=ra)
        ms, fin, res, dev = [], [], [], []
        for it in range(N + 2):
            t0 = time.perf_counter()
            ctx.render(W, H, spp, D, first_sample=k, readback=False)
            if spp == 1:
                ctx.read_rgba8(W, H)
            ms.append((time.perf_counter() - t0) * 1e3)
            st = ctx.stats()
            fin.append(st["ahead_finished"])
            res.append(st["ahead_resumed"])
            dev.append(round(st["render_ms"], 3))
            k += spp
        med = statistics.median(ms[2:])
        print(json.dumps({"lib": lib, "spp": spp, "render_ahead": ra, "median_ms": round(med, 3),
                          "Msamples_s": round(W * H * spp / med / 1e3, 1), "ms": [round(x, 3) for x in ms],
                          "device_ms": dev, "ahead_finished": fin, "ahead_resumed": res}), flush=True)
ctx.close()
