"""Fused-batch probe (dev tool, GPU box): ms per 8-spp frame at the metric row
when F consecutive passes run as one fused asynchronous batch followed by a
khp_sync, for F = 1 (a synchronous call) .. 4 -- the rate a synchronous call
would see if it rendered the next F-1 passes of its series with its own.
usage: python tools/fuse_probe.py [groups=6] [F list, default 1,2,3,4] [spp=8] [path_kernel=0]
       [render_ahead=0 for the F = 1 calls]"""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 6
FS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3,4").split(",")]
SPP = int(sys.argv[3]) if len(sys.argv) > 3 else 8
PK = int(sys.argv[4]) if len(sys.argv) > 4 else 0
RA = int(sys.argv[5]) if len(sys.argv) > 5 else 0
W, H, D = 1920, 1080, 5
ctx = HipContext(0)
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()
k = 0
for F in FS:
    ctx.set_params(fuse_frames=max(F, 1), path_kernel=PK, render_ahead=RA)
    ms = []
    for g in range(G + 1):
        t0 = time.perf_counter()
        if F == 1:
            ctx.render(W, H, SPP, D, first_sample=k, readback=False)
            k += SPP
        else:
            for _ in range(F):
                ctx.render(W, H, SPP, D, first_sample=k, async_=True)
                k += SPP
            ctx.sync()
        ms.append((time.perf_counter() - t0) * 1e3 / F)
    med = statistics.median(ms[1:])
    print(json.dumps({"F": F, "spp": SPP, "path_kernel": PK, "render_ahead": RA, "ms_per_frame": round(med, 3),
                      "Msamples_s": round(W * H * SPP / med / 1e3, 1), "ms": [round(x, 3) for x in ms]}), flush=True)
ctx.close()
