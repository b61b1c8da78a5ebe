"""Dev tool: parity of one library variant (KHP_LIB) vs the oracle on small scenes.

    KHP_LIB=.../libkirk_hip_x.so python tools/diag_parity.py
Prints one line per check; exits 0 even on mismatch (it is a diagnostic).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "oracle")]
import oracle_ffi  # noqa: E402
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402

lib = os.path.basename(os.environ.get("KHP_LIB", "libkirk_hip.so"))
for cfg, W, H, spp, depth, kw in [("config1", 64, 48, 2, 1, {}), ("config1", 64, 48, 2, 5, {}),
                                  ("config2", 64, 48, 2, 5, {"n_strands": 2000})]:
    sd = scenes.build_config(cfg, width=W, height=H, **kw)
    ctx = HipContext(0)
    ctx.set_scene(sd)
    ctx.build_accel()
    o = oracle_ffi.Oracle(sd)
    rng = np.random.default_rng(3)
    n = 4000
    orig = rng.uniform(-0.6, 1.2, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tm = rng.uniform(0.01, 2, n).astype(np.float32)
    t, obj, uv = ctx.trace_closest(orig, d)
    t0, obj0, uv0, _, _ = o.trace_closest(orig, d)
    a = ctx.trace_any(orig, d, tm)
    a0 = o.trace_any(orig, d, tm)
    img = ctx.render(W, H, spp, depth)
    ref = o.render(W, H, spp, depth, threads=8)
    bad = ~np.all(img.view(np.uint32) == ref.view(np.uint32), axis=-1)
    print(f"{lib} {cfg} depth{depth}: closest_obj_mismatch={int((obj != obj0).sum())} "
          f"t_mismatch={int((t.view(np.uint32) != t0.view(np.uint32)).sum())} any_mismatch={int((a != a0).sum())} "
          f"frame_bad_px={int(bad.sum())}", flush=True)
    ctx.close()

# determinism: the same frame twice
sd = scenes.config1(64, 48)
ctx = HipContext(0)
ctx.set_scene(sd)
ctx.build_accel()
a = ctx.render(64, 48, 2, 5)
b = ctx.render(64, 48, 2, 5)
print(f"{lib} rerun_identical={np.array_equal(a.view(np.uint32), b.view(np.uint32))} "
      f"diff_px={int((~np.all(a.view(np.uint32) == b.view(np.uint32), axis=-1)).sum())}", flush=True)

# production kernels ray by ray (KHP_TRACE_PERSISTENT=1 routes the batch API through k_extend / k_shadow)
for cfg, kw in [("config1", {}), ("config2", {"n_strands": 2000})]:
    sd = scenes.build_config(cfg, width=32, height=32, **kw)
    ctx = HipContext(0)
    ctx.set_scene(sd)
    ctx.build_accel()
    o = oracle_ffi.Oracle(sd)
    rng = np.random.default_rng(5)
    n = 200000
    orig = rng.uniform(-0.6, 1.2, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tm = rng.uniform(0.01, 2, n).astype(np.float32)
    t0, obj0, uv0, nv0, np0 = o.trace_closest(orig, d)
    a0 = o.trace_any(orig, d, tm)
    for rep, mode in enumerate(("1", "2")):
        os.environ["KHP_TRACE_PERSISTENT"] = mode
        t, obj, uv = ctx.trace_closest(orig, d)
        st = ctx.stats()
        a = ctx.trace_any(orig, d, tm)
        print(f"{lib} persistent mode{mode} {cfg}: closest_obj_mismatch={int((obj != obj0).sum())} "
              f"t_mismatch={int((t.view(np.uint32) != t0.view(np.uint32)).sum())} "
              f"visits={st['node_visits']}/{nv0} prims={st['prim_tests']}/{np0} any_mismatch={int((a != a0).sum())}",
              flush=True)
    del os.environ["KHP_TRACE_PERSISTENT"]
    ctx.close()
