"""Dev tool: phase breakdown of k_extend's loop (needs a KHP_PROFILE_STEPS=1 build via KHP_LIB)."""
import os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..")]
from ba_pathtracing_fur_amd import HipContext, scenes
sd = scenes.config3(1920, 1080, n_strands=1_000_000)
ctx = HipContext(0)
ctx.set_scene(sd); ctx.build_accel()
ctx.render(1920, 1080, 8, 5, readback=False)
ctx.render(1920, 1080, 8, 5, readback=False, stats=True)
st = ctx.stats()
cy = st["step_cycles"]
tot = sum(cy)
print("extend ms", st["extend_ms"], "iters", sum(st["bounce_wave_iters"]))
for name, v in zip(("resolve", "fetch", "compute", "loop+refill"), cy):
    print(f"{name:12s} {v / tot:.3f}  cycles/iter {v / max(1, sum(st['bounce_wave_iters'])):.0f}")
