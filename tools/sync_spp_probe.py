"""Probe (dev tool, GPU box): synchronous khp_render of s spp at the metric row
through the wavefront (path_kernel 1) and the path kernel (2), for the automatic
choice's threshold.  Prints one JSON line: median wall ms per call."""
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402

W, H, D, N = 1920, 1080, 5, 6
ctx = HipContext(0)
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()
out = {}
k = 0
for spp in (1, 2, 3, 4, 6, 8):
    for pk in (1, 2):
        ctx.set_params(path_kernel=pk)
        ms = []
        for it in range(N + 2):
            t0 = time.perf_counter()
            ctx.render(W, H, spp, D, first_sample=k, readback=False)
            ms.append((time.perf_counter() - t0) * 1e3)
            k += spp
        out[f"{spp}spp_pk{pk}"] = round(statistics.median(ms[2:]), 3)
    print(json.dumps(out), file=sys.stderr, flush=True)
print(json.dumps(out), flush=True)
ctx.close()
