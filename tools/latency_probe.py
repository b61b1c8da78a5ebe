"""Dev tool: intrinsic per-iteration latency of the persistent traversal kernel.
One ray (and one wave of rays) through k_extend on an otherwise idle GPU."""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..")]
from ba_pathtracing_fur_amd import HipContext, scenes
sd = scenes.config3(1920, 1080, n_strands=1_000_000)
ctx = HipContext(0)
ctx.set_scene(sd); ctx.build_accel()
rng = np.random.default_rng(3)
for n in (1, 64, 4096, 327680):
    orig = (rng.uniform(-0.5, 0.5, (n, 3)) + np.array([0, 1.0, 0])).astype(np.float32)  # inside the hairball
    d = rng.normal(size=(n, 3)).astype(np.float32); d /= np.linalg.norm(d, axis=1, keepdims=True)
    for mode in ("1", "2"):
        os.environ["KHP_TRACE_PERSISTENT"] = mode
        ms = []
        for rep in range(3):
            ctx.trace_closest(orig, d)
            st = ctx.stats()
            ms.append(st["render_ms"])
        if mode == "1":
            fetches = st["node_visits"] + st["prim_tests"]
        print(f"n={n:6d} mode{mode}: kernel {min(ms):.3f} ms, fetches/ray {fetches / n:.0f}, "
              f"us per fetch per ray {min(ms) * 1e3 / (fetches / n):.3f}", flush=True)
