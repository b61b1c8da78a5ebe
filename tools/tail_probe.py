"""Dev tool: per-wave timeline of one k_extend launch (KHP_TAIL_PROBE=1 build,
libkirk_hip_tp.so): when each wave started, when the queue drained under it,
when it ended, its rays, its longest ray and its iterations after the drain."""
import ctypes, os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..")]
os.environ.setdefault("KHP_LIB", os.path.join(HERE, "..", "ba_pathtracing_fur_amd", "lib", "libkirk_hip_tp.so"))
from ba_pathtracing_fur_amd import HipContext, scenes, native as N
lib = N.load_library()
fn = lib.khp_debug_tail_probe
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = np.zeros(6 * 65536, np.uint64)
ctx = HipContext(0)
sd = scenes.config3_device(ctx, 1920, 1080, n_strands=1_000_000)
ctx.build_accel()

def report(tag):
    fn(buf.ctypes.data, 0)
    r = buf.reshape(-1, 6)
    r = r[r[:, 2] > 0].astype(np.float64)
    t0 = r[:, 0].min()
    st, ex, en = (r[:, 0] - t0) / 100.0, np.where(r[:, 1] > 0, (r[:, 1] - t0) / 100.0, np.nan), (r[:, 2] - t0) / 100.0
    span = en.max()
    q = lambda a, p: np.nanpercentile(a, p)
    late = en > q(en, 99)
    per_it = (en - ex) / np.maximum(r[:, 5], 1)
    print(f"{tag}: waves {len(r)}, span {span:.0f} us; start p50/max {q(st,50):.0f}/{st.max():.0f}; "
          f"drain p50/p90/max {q(ex,50):.0f}/{q(ex,90):.0f}/{np.nanmax(ex):.0f}; end p50/p90/p99/max "
          f"{q(en,50):.0f}/{q(en,90):.0f}/{q(en,99):.0f}/{en.max():.0f} us; rays/wave p50 {q(r[:,3],50):.0f}; "
          f"longest ray (it) p50/p99/max {q(r[:,4],50):.0f}/{q(r[:,4],99):.0f}/{r[:,4].max():.0f}; "
          f"last 1% waves: longest ray p50 {q(r[late,4],50):.0f}, it after drain p50 {q(r[late,5],50):.0f}, "
          f"us/iter after drain p50 {q(per_it[late],50):.2f}", flush=True)

cam = sd.cam
pos = np.array(cam.position[:3], np.float32)
bl, ax, ay = (np.array(getattr(cam, k)[:3], np.float32) for k in ("bottom_left", "axis_x", "axis_y"))
rng = np.random.default_rng(5)
os.environ["KHP_TRACE_PERSISTENT"] = "2"
for n in (4096, 262144, 2073600, 16588800 // 2):
    x = rng.uniform(0, 1920, n).astype(np.float32); y = rng.uniform(0, 1080, n).astype(np.float32)
    d = bl[None] + ax[None] * (x * cam.pixel_size)[:, None] + ay[None] * (y * cam.pixel_size)[:, None] - pos[None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.repeat(pos[None], n, 0)
    ctx.trace_closest(o, d)
    fn(buf.ctypes.data, 1)
    ctx.trace_closest(o, d)
    report(f"camera rays n={n} ({ctx.stats()['render_ms']:.3f} ms)")
    oi = (rng.uniform(-0.5, 0.5, (n, 3)) + np.array([0, 1.0, 0])).astype(np.float32)
    di = rng.normal(size=(n, 3)).astype(np.float32); di /= np.linalg.norm(di, axis=1, keepdims=True)
    fn(buf.ctypes.data, 1)
    ctx.trace_closest(oi, di)
    report(f"inside rays n={n} ({ctx.stats()['render_ms']:.3f} ms)")
del os.environ["KHP_TRACE_PERSISTENT"]
# primary-ray launch of a rank-of-8 frame and of the full frame (depth 1: one extend launch)
for nr in (8, 1):
    kw = dict(tile_size=64, tile_rank=0, tile_nranks=nr, readback=False)
    ctx.render(1920, 1080, 8, 1, **kw)
    fn(buf.ctypes.data, 1)
    ctx.render(1920, 1080, 8, 1, **kw)
    report(f"frame bounce-0 launch, rank 0 of {nr} ({ctx.stats()['extend_ms']:.3f} ms)")
