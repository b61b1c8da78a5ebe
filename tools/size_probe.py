"""Dev tool: k_extend (production persistent kernel) time vs queue size for camera
rays of the metric scene, through the batch query hook (KHP_TRACE_PERSISTENT=2).
A fit ms = a + b*n separates the per-launch floor (a) from throughput (b)."""
import os, sys, time
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..")]
from ba_pathtracing_fur_amd import HipContext, scenes
ctx = HipContext(0)
sd = scenes.config3_device(ctx, 1920, 1080, n_strands=1_000_000)
ctx.build_accel()
cam = sd.cam
pos = np.array(cam.position[:3], np.float32)
bl, ax, ay = (np.array(getattr(cam, k)[:3], np.float32) for k in ("bottom_left", "axis_x", "axis_y"))
ps = cam.pixel_size
rng = np.random.default_rng(5)
os.environ["KHP_TRACE_PERSISTENT"] = os.environ.get("MODE", "2")
res = []
for n in (1, 64, 4096, 16384, 65536, 262144, 1048576, 4194304):
    x = rng.uniform(0, 1920, n).astype(np.float32); y = rng.uniform(0, 1080, n).astype(np.float32)
    d = bl[None] + ax[None] * (x * ps)[:, None] + ay[None] * (y * ps)[:, None] - pos[None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.repeat(pos[None], n, 0)
    ms = []
    for rep in range(3):
        ctx.trace_closest(o, d)
        ms.append(ctx.stats()["render_ms"])
    print(f"camera n={n:8d}: k_extend {min(ms):.3f} ms", flush=True)
    # inside-hairball rays (bounce 2+ like)
    oi = (rng.uniform(-0.5, 0.5, (n, 3)) + np.array([0, 1.0, 0])).astype(np.float32)
    di = rng.normal(size=(n, 3)).astype(np.float32); di /= np.linalg.norm(di, axis=1, keepdims=True)
    ms = []
    for rep in range(3):
        ctx.trace_closest(oi, di)
        ms.append(ctx.stats()["render_ms"])
    print(f"inside n={n:8d}: k_extend {min(ms):.3f} ms", flush=True)
