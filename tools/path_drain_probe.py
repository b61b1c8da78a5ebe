"""Per-wave timeline of k_path's drain (dev tool, GPU box; KHP_PATH_PROFILE builds).

Runs KIRK's GUI pattern (synchronous 1-spp khp_render + 8-bit texture) and the
8-spp synchronous pass on the metric scene with a diagnostic build of the
library (tools/build_variant.sh <name> -DKHP_PATH_PROFILE, then KHP_LIB=...),
reads every k_path wave's record (khp_debug_wave_profile: start, claim
exhaustion seen, end, loop iterations, traversing lanes in the drain) and prints
one JSON line per pattern:
  * exh_ms / end_ms: when the last wave saw the claims exhausted, when the last
    wave ended (ms after the first wave started);
  * alive_after_exh: waves still running 0, 0.25, 0.5, 1, 2, 3 ms after the
    last exhaustion;
  * longest: the 8 waves that ended last -- drain ms, drain iterations, us per
    drain iteration, mean traversing lanes per drain iteration.
usage: KHP_LIB=variants/libkirk_prof.so python tools/path_drain_probe.py [calls=4] [extra params k=v ...]
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, scenes  # noqa: E402
from ba_pathtracing_fur_amd import native  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
extra = dict(a.split("=") for a in sys.argv[2:])
W, H, D = 1920, 1080, 5
lib = native.load_library()
ctx = HipContext(0)
lib = ctx.lib
if not hasattr(lib, "khp_debug_wave_profile"):
    raise SystemExit("not a KHP_PATH_PROFILE build (set KHP_LIB)")
MAXW = 65536
buf = (ctypes.c_uint64 * (6 * MAXW))()
nw = ctypes.c_uint32(0)
if extra:
    ctx.set_params(**{k: int(v) for k, v in extra.items()})
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()


RA = (ctypes.c_uint64 * 2)()


def read_ahead():
    """khp_debug_ahead_profile: clock of the last own path's end, of the first wave seeing it."""
    if not hasattr(lib, "khp_debug_ahead_profile"):
        return None
    lib.khp_debug_ahead_profile.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    native.check(lib, lib.khp_debug_ahead_profile(ctx.ptr, RA), "khp_debug_ahead_profile")
    return RA[0], RA[1]


def read_waves():
    lib.khp_debug_wave_profile.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
    native.check(lib, lib.khp_debug_wave_profile(ctx.ptr, buf, MAXW, ctypes.byref(nw)), "khp_debug_wave_profile")
    return [tuple(buf[6 * i + j] for j in range(6)) for i in range(nw.value)]


k = 0
for _ in range(2):  # warmup
    ctx.render(W, H, 1, D, first_sample=k, readback=False)
    k += 1
    ctx.render(W, H, 8, D, first_sample=k, readback=False)
    k += 8
read_waves()
read_ahead()
for name, spp in (("gui", 1), ("sync8", 8)):
    for call in range(N):
        ctx.render(W, H, spp, D, first_sample=k, readback=False)
        k += spp
        st = ctx.stats()
        rec = read_waves()
        ra = read_ahead()
        if not rec:
            continue
        t0 = min(r[0] for r in rec)
        exh = [r[1] for r in rec if r[1]]
        last_exh = max(exh)
        end = max(r[2] for r in rec)
        alive = {str(dt): sum(1 for r in rec if r[2] > last_exh + dt * 1e5) for dt in (0, 0.25, 0.5, 1, 2, 3)}
        longest = sorted(rec, key=lambda r: r[2])[-8:]
        lw = []
        for r in reversed(longest):
            dit = r[3] & 0xFFFFFFFF
            dms = (r[2] - r[1]) / 1e5 if r[1] else 0.0
            lw.append({"block": r[5] >> 32, "start_ms": round((r[0] - t0) / 1e5, 3),
                       "exh_ms": round((r[1] - t0) / 1e5, 3) if r[1] else None,
                       "end_ms": round((r[2] - t0) / 1e5, 3), "drain_ms": round(dms, 3),
                       "iters": r[3] >> 32, "drain_iters": dit,
                       "us_per_drain_iter": round(dms * 1e3 / dit, 3) if dit else None,
                       "lanes_per_drain_iter": round(r[4] / dit, 2) if dit else None,
                       "lanes_at_exh": r[5] & 0xFFFFFFFF})
        ra_line = None
        if ra and ra[0]:
            ra_line = {"own_end_ms": round((ra[0] - t0) / 1e5, 3),
                       "stop_seen_ms": round((ra[1] - t0) / 1e5, 3) if ra[1] != 2 ** 64 - 1 else None,
                       "ahead_finished": st["ahead_finished"], "ahead_resumed": st["ahead_resumed"]}
        print(json.dumps({"pattern": name, "call": call, "waves": len(rec), "device_ms": round(st["render_ms"], 3),
                          "ahead": ra_line,
                          "first_exh_ms": round((min(exh) - t0) / 1e5, 3), "exh_ms": round((last_exh - t0) / 1e5, 3),
                          "end_ms": round((end - t0) / 1e5, 3), "alive_after_exh": alive, "longest": lw}), flush=True)
ctx.close()
