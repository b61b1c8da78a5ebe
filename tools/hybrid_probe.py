"""Hybrid batches probe (dev tool, GPU box; khp_ctx_params.path_from): the metric
row's synchronous 8-spp call (the wavefront) and the driver's fused 20-pass
batch with the paths handed to one k_path launch from bounce b, b in the list.
Prints one JSON line per (mode, b): mean ms per call / per pass and Msamples/s.
usage: python tools/hybrid_probe.py [b list, default 0,2,3,4] [calls=6]"""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402

BS = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,2,3,4").split(",")]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 6
W, H, D, SPP = 1920, 1080, 5, 8
ctx = HipContext(0)
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()
k = 0
for rnd in range(2):
    for b in BS:
        ctx.set_params(path_from=b)
        ms = []
        for it in range(N + 1):
            t0 = time.perf_counter()
            ctx.render(W, H, SPP, D, first_sample=k, readback=False)
            ms.append((time.perf_counter() - t0) * 1e3)
            k += SPP
        m = statistics.mean(ms[1:])
        print(json.dumps({"mode": "sync8", "round": rnd, "path_from": b, "mean_ms": round(m, 3),
                          "Msamples_s": round(W * H * SPP / m / 1e3, 1), "ms": [round(x, 2) for x in ms[1:]]}),
              flush=True)
        for it in range(2):   # the driver's batch: 20 fused passes; the first one warms up
            ctx.sync()
            t0 = time.perf_counter()
            for s in range(20):
                ctx.render(W, H, SPP, D, first_sample=k, async_=True)
                k += SPP
            ctx.sync()
            el = (time.perf_counter() - t0) * 1e3
        print(json.dumps({"mode": "fused20", "round": rnd, "path_from": b, "ms_per_pass": round(el / 20, 3),
                          "Msamples_s": round(20 * W * H * SPP / el / 1e3, 1)}), flush=True)
ctx.close()
