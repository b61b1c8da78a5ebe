"""Where one rank's share of an N-GPU frame loses time (dev tool, GPU box).

Renders the metric scene's fused progressive passes for the whole frame and
for rank r of N (the tiles t % N == r, as tools/scale_probe.py) and prints,
per frame, the wall time, the device time and each bounce's k_extend and
shadow-stage time from khp_stats, with the whole frame's figures divided by N
beside them, so the rank's excess shows per stage.

usage: python tools/rank_probe.py [--nranks 8] [--rank 6] [--steps 20] [--set KEY=INT ...]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))

from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402


def run(ctx, W, H, spp, depth, steps, n, r):
    kw = dict(seed=0x4B49524B, tile_size=64, tile_rank=r, tile_nranks=n, readback=False, async_=True)
    k = 0
    for _ in range(steps):
        ctx.render(W, H, spp, depth, first_sample=k * spp, **kw)
        k += 1
    ctx.sync()
    ctx.stats()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.render(W, H, spp, depth, first_sample=k * spp, **kw)
        k += 1
    ctx.sync()
    wall = (time.perf_counter() - t0) / steps * 1e3
    st = ctx.stats()
    f = max(1, st["frames"])
    return {"wall_ms": round(wall, 3), "device_ms": round(st["render_ms"] / f, 3),
            "extend_busy_ms": round(st["extend_busy_ms"] / f, 3), "shade_ms": round(st["shade_ms"] / f, 3),
            "shadow_ms": round(st["shadow_ms"] / f, 3),
            "extend_ms": [round(x / f, 3) for x in st["bounce_extend_ms"][:depth]],
            "bounce_shadow_ms": [round(x / f, 3) for x in st["bounce_shadow_ms"][:depth]],
            "extend_launches": st["extend_launches"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, default=8)
    ap.add_argument("--rank", type=int, default=6)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--set", nargs="*", default=[], metavar="KEY=INT")
    a = ap.parse_args()
    W, H, spp, depth = 1920, 1080, 8, 5
    ctx = HipContext(0)
    if a.set:
        ctx.set_params(**{k: int(v) for k, v in (kv.split("=", 1) for kv in a.set)})
    scenes.config3_device(ctx, W, H)
    ctx.build_accel()
    full = run(ctx, W, H, spp, depth, a.steps, 1, 0)
    part = run(ctx, W, H, spp, depth, a.steps, a.nranks, a.rank)
    n = a.nranks
    share = {k: ([round(x / n, 3) for x in v] if isinstance(v, list) else round(v / n, 3))
             for k, v in full.items() if k != "extend_launches"}
    print(json.dumps({"full": full, f"rank_{a.rank}_of_{n}": part, "full_over_n": share,
                      "params": ctx.params()}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
