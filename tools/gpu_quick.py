"""Quick GPU-vs-oracle check (dev tool)."""
import sys, os, time
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ba_pathtracing_fur_amd import scenes, HipContext
import oracle_ffi

def cmp(name, a, b):
    fa, fb = np.isfinite(a), np.isfinite(b)
    mask_eq = np.array_equal(fa, fb)
    both = fa.all(-1) & fb.all(-1)
    d = np.linalg.norm((a - b)[both], axis=-1) if both.any() else np.zeros(1)
    print(f"{name}: nonfinite_mask_equal={mask_eq} nonfinite={int((~fa).any(-1).sum())} "
          f"bitexact={np.array_equal(a.view(np.uint32), b.view(np.uint32))} maxL2={d.max():.3g} meanL2={d.mean():.3g} "
          f"diverged(>1e-3)={(d > 1e-3).sum()}", flush=True)

for cfg, W, H, spp, kw in [("config1", 64, 64, 4, {}), ("config2", 96, 64, 4, {"n_strands": 3000}),
                           ("config3", 96, 64, 2, {"n_strands": 5000})]:
    sd = scenes.build_config(cfg, width=W, height=H, **kw)
    ctx = HipContext(0, stats=True)
    t = time.time(); ctx.set_scene(sd); ctx.build_accel(); print(cfg, "build", time.time() - t, ctx.stats()["bvh_depth"], flush=True)
    img = ctx.render(W, H, spp, 5)
    o = oracle_ffi.Oracle(sd)
    ref = o.render(W, H, spp, 5, threads=16)
    cmp(cfg, img, ref)
    # rays
    rng = np.random.default_rng(1)
    n = 20000
    orig = rng.uniform(-1, 2, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    t1, ob1, uv1 = ctx.trace_closest(orig, d)
    t2, ob2, uv2, nv, pt = o.trace_closest(orig, d)
    st = ctx.stats()
    print("  closest: obj_eq", np.array_equal(ob1, ob2), "t_eq", np.array_equal(t1, t2), "uv_eq", np.array_equal(uv1, uv2),
          "visits gpu/cpu", st["node_visits"], nv, st["prim_tests"], pt, flush=True)
    tm = rng.uniform(0, 3, n).astype(np.float32)
    h1 = ctx.trace_any(orig, d, tm); h2 = o.trace_any(orig, d, tm)
    print("  any: eq", np.array_equal(h1, h2), h1.mean(), flush=True)
