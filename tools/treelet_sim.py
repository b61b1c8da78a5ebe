"""Offline treelet study (dev tool, CPU): how the exact visit sequences of the
metric row's rays split between a top tree and LDS-sized bottom subtrees.

    python tools/treelet_sim.py RAYS.npz [--budgets 8,16,32,64] [--n 100000]

RAYS.npz comes from tools/dump_rays.py (a sample of each bounce's extension
queue on the GPU).  The BVH and every visit come from the CPU restatement
(oracle/, ko_trace_closest_log: KIRK's near-first traversal, node ids in DFS
preorder).  A treelet is a maximal subtree whose records (64 B per interior
node, 64 B per leaf candidate) fit in `budget` KB; every other node is "top".
Because KIRK's traversal finishes a subtree before it leaves it, a ray visits
each treelet in one contiguous run: one entry (a suspension / resumption in a
treelet-scheduled traversal) per treelet it reaches.  Printed per bounce:
records per ray in the top tree and in treelets, entries per ray, and for the
real queue size (rays per frame x fused frames) the rays per treelet per round
and the LDS fill bytes that a round-synchronous treelet scheduler would move.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]


def tree_arrays(o):
    bv = o.bvh()
    count = bv[2].astype(np.int32)
    n = len(count)
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "treelet_sim.so"))
    size, prims, right = (np.empty(n, np.int64) for _ in range(3))
    P = ctypes.POINTER(ctypes.c_int64)
    lib.subtree_sizes(ctypes.c_int64(n), count.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                      size.ctypes.data_as(P), prims.ctypes.data_as(P), right.ctypes.data_as(P))
    parent = np.full(n, -1, np.int64)
    inter = np.flatnonzero(count == 0)
    parent[inter + 1] = inter
    parent[right[inter]] = inter
    return count, size, prims, parent


def treelets(count, size, prims, parent, budget):
    leaves = (size + 1) // 2
    rec = (size - leaves) + prims                      # 64-B records of the subtree
    fits = rec * 64 <= budget
    pfit = np.where(parent >= 0, fits[np.maximum(parent, 0)], False)
    roots = np.flatnonzero(fits & ~pfit)
    mark = np.zeros(len(count) + 1, np.int64)
    ids = np.arange(1, len(roots) + 1)
    np.add.at(mark, roots, ids)
    np.add.at(mark, roots + size[roots], -ids)
    tid = np.cumsum(mark[:-1]) - 1                     # -1: top
    return tid, roots, rec[roots] * 64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rays")
    ap.add_argument("--budgets", default="8,16,32,64")
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--strands", type=int, default=1_000_000)
    ap.add_argument("--fused", type=int, default=8, help="frames per launch (the real queue = rays x fused)")
    a = ap.parse_args()
    import oracle_ffi
    from ba_pathtracing_fur_amd import scenes
    t0 = time.time()
    sd = scenes.build_config("config3", width=1920, height=1080, n_strands=a.strands)
    o = oracle_ffi.Oracle(sd)
    count, size, prims, parent = tree_arrays(o)
    print(f"tree: {len(count)} nodes, {int(prims[0])} candidates, built in {time.time() - t0:.0f}s", flush=True)
    lib = o.lib
    lib.ko_trace_closest_log.restype = ctypes.c_int
    lib.ko_trace_closest_log.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    R = np.load(a.rays)
    budgets = [int(x) * 1024 for x in a.budgets.split(",")]
    parts = {B: treelets(count, size, prims, parent, B) for B in budgets}
    for B, (tid, roots, tb) in parts.items():
        print(f"budget {B >> 10} KB: {len(roots)} treelets, mean {tb.mean() / 1024:.1f} KB, top nodes "
              f"{int((tid < 0).sum())} ({int((tid < 0).sum()) * 64 / 1e6:.1f} MB)", flush=True)
    for b in range(8):
        if f"o{b}" not in R:
            continue
        # a random subset: the dump is in queue order (longest-first rays at the front)
        pick = np.sort(np.random.default_rng(b).permutation(len(R[f"o{b}"]))[:a.n])
        orig, dirs = np.ascontiguousarray(R[f"o{b}"][pick]), np.ascontiguousarray(R[f"d{b}"][pick])
        n_real = int(R[f"n{b}"]) * a.fused
        m = len(orig)
        cap = m * 1200
        log = np.empty(cap, np.int32)
        off = np.empty(m + 1, np.uint64)
        tt = np.empty(m, np.float32)
        t1 = time.time()
        lib.ko_trace_closest_log(o.ptr, m, orig.ctypes.data, dirs.ctypes.data, tt.ctypes.data, log.ctypes.data,
                                 ctypes.c_uint64(cap), off.ctypes.data)
        if off[-1] > cap:
            raise SystemExit("visit log overflow")
        raw = log[:int(off[-1])]
        v, pend = raw & 0x1FFFFFF, raw >> 25
        ray = np.repeat(np.arange(m), np.diff(off).astype(np.int64))
        recs = np.where(count[v] > 0, count[v], 1)     # records fetched per visit
        print(f"\nbounce {b}: {m} rays sampled of {n_real // a.fused} per frame, traced in {time.time() - t1:.0f}s; "
              f"records per ray {recs.sum() / m:.1f} (visits {len(v) / m:.1f})", flush=True)
        for B, (tid, roots, tb) in parts.items():
            tv = tid[v]
            top = tv < 0
            # entries: runs of one treelet id in a ray's sequence
            start = np.ones(len(v), bool)
            start[1:] = (tv[1:] != tv[:-1]) | (ray[1:] != ray[:-1])
            ent = start & ~top
            e_ray, e_tid = ray[ent], tv[ent]
            per_ray = np.bincount(e_ray, minlength=m)
            # round r = the ray's r-th entry
            order = np.cumsum(ent) - 1
            first_of_ray = np.searchsorted(np.flatnonzero(ent), np.searchsorted(ray, np.arange(m)))
            rnd = order[ent] - first_of_ray[e_ray]
            scale = n_real / m
            fill, served, rounds = 0.0, 0.0, int(rnd.max()) + 1 if len(rnd) else 0
            kpr = []
            for r in range(rounds):
                sel = e_tid[rnd == r]
                u, c = np.unique(sel, return_counts=True)
                # expected distinct treelets among n_real*|sel|/m draws with these frequencies
                N_r = len(sel) * scale
                p = c / len(sel)
                distinct = np.sum(1.0 - np.exp(-N_r * p))
                fill += float(np.sum(tb[u] * (1.0 - np.exp(-N_r * p))))
                kpr.append((r, N_r, distinct))
            bottom = recs[~top].sum() * scale * 64
            k_all = sum(x[1] for x in kpr) / max(1e-9, sum(x[2] for x in kpr))
            ps = pend[ent]
            inside = ~top & ~start
            print(f"         top stack at entry: mean {ps.mean():.1f} p99 {np.percentile(ps, 99):.0f} max {ps.max()}; "
                  f"treelet-local depth p99 {np.percentile(pend[inside] - np.repeat(ps, np.diff(np.append(np.flatnonzero(ent), len(v)))[:len(ps)])[:0].size if False else 0, 99) if False else 0}",
                  flush=True) if False else None
            # local depth inside a treelet = pending at the visit - pending at the treelet's entry
            ent_idx = np.flatnonzero(ent)
            run_id = np.cumsum(start) - 1                      # run index of every visit
            run_first = np.flatnonzero(start)
            base = pend[run_first][run_id]
            loc = (pend - base)[~top]
            print(f"         top stack at entry: mean {ps.mean():.1f} p99 {np.percentile(ps, 99):.0f} max {ps.max()}; "
                  f"treelet-local stack p99 {np.percentile(loc, 99):.0f} max {loc.max()}", flush=True)
            print(f"  {B >> 10:3d} KB: top {recs[top].sum() / m:6.1f} rec/ray, treelets {recs[~top].sum() / m:6.1f} "
                  f"rec/ray, entries/ray mean {per_ray.mean():.1f} p50 {np.median(per_ray):.0f} "
                  f"p99 {np.percentile(per_ray, 99):.0f} max {per_ray.max()}; rounds {rounds}; rays per treelet-round "
                  f"{k_all:.0f}; LDS fill {fill / 1e9:.1f} GB vs {bottom / 1e9:.1f} GB of treelet records read "
                  f"per launch ({a.fused} frames)", flush=True)
            head = ", ".join(f"r{r}:{N_r / 1e6:.1f}M/{d / 1e3:.0f}k" for r, N_r, d in kpr[:6])
            print(f"         rounds (rays/distinct treelets): {head}", flush=True)


if __name__ == "__main__":
    main()
