"""Probe (dev tool, GPU box): a synchronous 8-spp pass as ONE khp_render, against the
same pass split into H asynchronous renders of 8/H spp each running as batches in
flight (frames_in_flight = H, no fusion) and completed by one khp_sync.  Prints one
JSON line of wall ms per call.  usage: python tools/split_sync_probe.py [calls=6] [H=2]"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 6
HS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
W, H, D, SPP = 1920, 1080, 5, 8
ctx = HipContext(0)
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()
out = {}
k = 0
for name, prm in (("one_call_path_kernel", dict(path_kernel=0)), ("one_call_wavefront", dict(path_kernel=1)),
                  (f"split_{HS}_in_flight", dict(path_kernel=1, fuse_frames=1, frames_in_flight=HS))):
    ctx.set_params(**prm)
    ms = []
    for it in range(N + 2):
        t0 = time.perf_counter()
        if name.startswith("split"):
            for h in range(HS):
                ctx.render(W, H, SPP // HS, D, first_sample=k + h * (SPP // HS), async_=True)
            ctx.sync()
        else:
            ctx.render(W, H, SPP, D, first_sample=k, readback=False)
        ms.append((time.perf_counter() - t0) * 1e3)
        k += SPP
    out[name] = [round(x, 2) for x in ms[2:]]
    ctx.set_params(path_kernel=0, fuse_frames=32, frames_in_flight=1)
print(json.dumps(out), flush=True)
ctx.close()
