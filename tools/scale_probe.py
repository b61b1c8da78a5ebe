"""Strong-scaling projection on ONE GPU (dev tool, run on the GPU box).

The driver's 1/2/4/8-GPU bench renders, on each rank, the tiles t with
t % N == rank (sharding.py).  Ranks share nothing but the final gather, so a
rank's frame time can be measured on one GPU by rendering exactly that rank's
tile set.  For N in --nranks this renders every rank's share (steps frames
each, after a warmup), and prints per N: the slowest rank's ms per frame and
the projected whole-job Msamples/s = W*H*spp / max-rank time (gather excluded:
≤0.1 ms over xGMI).

usage: python tools/scale_probe.py [--nranks 1 2 4 8] [--steps 3] [--strands 1000000]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))

from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--strands", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--ranks-max", type=int, default=8, help="time at most this many ranks per N (spread over 0..N-1)")
    ap.add_argument("--sync-steps", action="store_true", help="no frame pipelining (bench.py --sync-steps)")
    ap.add_argument("--path-order", type=int, default=None, help="khp_ctx_params.path_order")
    ap.add_argument("--set", nargs="*", default=[], metavar="KEY=INT", help="other khp_ctx_params fields")
    a = ap.parse_args()
    W, H, spp, depth = a.width, a.height, a.spp, a.depth
    ctx = HipContext(0)
    if a.path_order is not None:
        ctx.set_params(path_order=a.path_order)
    if a.set:
        ctx.set_params(**{k: int(v) for k, v in (kv.split("=", 1) for kv in a.set)})
    scenes.config3_device(ctx, W, H, n_strands=a.strands)
    ctx.build_accel()
    out = []
    for n in a.nranks:
        ranks = (list(range(n)) if n <= a.ranks_max else [0] if a.ranks_max <= 1 else
                 [round(i * (n - 1) / (a.ranks_max - 1)) for i in range(a.ranks_max)])
        per = {}
        for r in ranks:
            kw = dict(seed=0x4B49524B, tile_size=a.tile, tile_rank=r, tile_nranks=n, readback=False,
                      async_=not a.sync_steps)
            k = 0  # progressive passes, as bench.py: pass k renders samples [k*spp, (k+1)*spp)
            for _ in range(a.steps):  # warmup (allocations, a full fused batch)
                ctx.render(W, H, spp, depth, first_sample=k * spp, **kw)
                k += 1
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                ctx.render(W, H, spp, depth, first_sample=k * spp, **kw)
                k += 1
            ctx.sync()
            per[r] = (time.perf_counter() - t0) / a.steps * 1e3
            print(f"N={n} rank {r}: {per[r]:.3f} ms/frame", file=sys.stderr, flush=True)
        worst = max(per.values())
        rec = {"nranks": n, "max_rank_ms": round(worst, 3), "min_rank_ms": round(min(per.values()), 3),
               "projected_msamples_s": round(W * H * spp / worst / 1e3, 1), "ranks_timed": ranks}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    base = out[0]["projected_msamples_s"] if out and out[0]["nranks"] == 1 else None
    if base:
        for rec in out:
            rec["speedup_vs_1"] = round(rec["projected_msamples_s"] / base, 2)
    print(json.dumps({"scale_probe": out}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
