"""Dump a sample of the metric row's extension rays per bounce (dev tool, GPU box).

python tools/dump_rays.py OUT.npz [--n 300000] [--bounces 0,1,2,3]
Renders the metric scene (config 3 geometry, 1M strands) at 1920x1080, 1 spp,
with khp_ctx_params.dump_bounce = b and keeps a seeded random sample of that
bounce's queue (origin, direction).  Input of tools/treelet_sim.py."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--n", type=int, default=300_000)
    ap.add_argument("--bounces", default="0,1,2,3")
    ap.add_argument("--strands", type=int, default=1_000_000)
    a = ap.parse_args()
    from ba_pathtracing_fur_amd import HipContext, scenes
    W, H = 1920, 1080
    ctx = HipContext(0)
    scenes.config3_device(ctx, W, H, n_strands=a.strands)
    ctx.build_accel()
    out, rng = {}, np.random.default_rng(7)
    for b in (int(x) for x in a.bounces.split(",")):
        ctx.set_params(dump_bounce=b)
        ctx.render(W, H, 1, 5, readback=False)
        (o, d), _ = ctx.debug_queues()
        idx = np.sort(rng.choice(len(o), size=min(a.n, len(o)), replace=False))
        out[f"o{b}"], out[f"d{b}"], out[f"n{b}"] = o[idx], d[idx], np.int64(len(o))
        print(f"bounce {b}: {len(o)} rays, kept {len(idx)}", flush=True)
    np.savez_compressed(a.out, **out)
    ctx.close()


if __name__ == "__main__":
    main()
