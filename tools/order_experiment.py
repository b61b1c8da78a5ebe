"""Dev experiment: how much does ray order matter for the production extend kernel?
Dumps the real bounce-b extension queue of the metric frame and replays it via
KHP_TRACE_PERSISTENT=2 in several orders; prints kernel ms per order."""
import ctypes, os, sys, time
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..")]
from ba_pathtracing_fur_amd import HipContext, scenes, native as N

def morton3(q):
    q = q.astype(np.uint64)
    def spread(x):
        x &= 0x3FF
        x = (x | (x << 16)) & 0x030000FF
        x = (x | (x << 8)) & 0x0300F00F
        x = (x | (x << 4)) & 0x030C30C3
        x = (x | (x << 2)) & 0x09249249
        return x
    return spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)

b = int(sys.argv[1]) if len(sys.argv) > 1 else 1
sd = scenes.config3(1920, 1080, n_strands=1_000_000)
ctx = HipContext(0)
ctx.set_scene(sd); ctx.build_accel()
os.environ["KHP_DUMP_BOUNCE"] = str(b)
ctx.render(1920, 1080, 8, 5, readback=False)
del os.environ["KHP_DUMP_BOUNCE"]
lib = ctx.lib
n = ctypes.c_uint32(0)
N.check(lib, lib.khp_debug_queue(ctx.ptr, ctypes.byref(n), None, None), "dbg")
o = np.empty((n.value, 3), np.float32); d = np.empty((n.value, 3), np.float32)
N.check(lib, lib.khp_debug_queue(ctx.ptr, ctypes.byref(n), N.fptr(o), N.fptr(d)), "dbg")
print(f"bounce {b}: {n.value} rays", flush=True)
lo, hi = o.min(0), o.max(0)
q = ((o - lo) / (hi - lo + 1e-9) * 1023).astype(np.int64)
mort = morton3(q)
octant = ((d[:, 0] < 0).astype(np.int64) | ((d[:, 1] < 0) << 1) | ((d[:, 2] < 0) << 2))
qd = ((d * 0.5 + 0.5) * 7.99).astype(np.int64)
dmort = morton3(qd)
rng = np.random.default_rng(0)
orders = {
    "queue": np.arange(n.value),
    "random": rng.permutation(n.value),
    "octant": np.argsort(octant, kind="stable"),
    "morton": np.argsort(mort, kind="stable"),
    "octant+morton": np.lexsort((mort, octant)),
    "morton+octant": np.lexsort((octant, mort >> 9)),
    "dir8^3+morton": np.lexsort((mort, dmort)),
}
os.environ["KHP_TRACE_PERSISTENT"] = "2"
ref = None
for name, perm in orders.items():
    oo, dd = np.ascontiguousarray(o[perm]), np.ascontiguousarray(d[perm])
    ms = []
    for rep in range(3):
        t, obj, uv = ctx.trace_closest(oo, dd)
        ms.append(ctx.stats()["render_ms"])
    if ref is None:
        ref = obj[np.argsort(perm)]
    assert np.array_equal(obj[np.argsort(perm)], ref)
    print(f"{name:16s} kernel ms {min(ms):.3f} (runs {', '.join(f'{m:.3f}' for m in ms)})", flush=True)
