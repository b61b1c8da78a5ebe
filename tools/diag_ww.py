"""Dev tool: are WW mismatches per-ray (logic) or cross-lane (interference)?"""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "oracle")]
import oracle_ffi
from ba_pathtracing_fur_amd import HipContext, scenes
sd = scenes.config1(32, 32)
ctx = HipContext(0); ctx.set_scene(sd); ctx.build_accel()
o = oracle_ffi.Oracle(sd)
rng = np.random.default_rng(5)
n = 200000
orig = rng.uniform(-0.6, 1.2, (n, 3)).astype(np.float32)
d = rng.normal(size=(n, 3)).astype(np.float32); d /= np.linalg.norm(d, axis=1, keepdims=True)
t0, obj0, uv0, _, _ = o.trace_closest(orig, d)
os.environ["KHP_TRACE_PERSISTENT"] = "1"
t, obj, uv = ctx.trace_closest(orig, d)
bad = np.nonzero(obj != obj0)[0]
print("batch mismatches", len(bad), "first", bad[:10].tolist())
ok_alone = 0
for i in bad[:20]:
    t1, ob1, _ = ctx.trace_closest(orig[i:i+1], d[i:i+1])
    _, _, _, nv, npr = o.trace_closest(orig[i:i+1], d[i:i+1])
    st = ctx.stats()
    ok_alone += int(ob1[0] == obj0[i])
    print(f"ray {i}: batch obj {obj[i]} t {t[i]:.6g} | alone obj {ob1[0]} t {t1[0]:.6g} visits {st['node_visits']}/{nv} prims {st['prim_tests']}/{npr} | oracle obj {obj0[i]} t {t0[i]:.6g}")
print("correct when alone:", ok_alone, "of", min(20, len(bad)))
# batch of 64 consecutive rays containing a bad one
j = bad[0] - bad[0] % 64
tb, obb, _ = ctx.trace_closest(orig[j:j+64], d[j:j+64])
print("64-batch mismatches", int((obb != obj0[j:j+64]).sum()))
