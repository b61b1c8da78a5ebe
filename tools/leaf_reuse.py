"""Leaf-record reuse inside a wave (dev tool, GPU box).

With a KHP_LEAF_REUSE build (tools/build_variant.sh leafreuse -DKHP_LEAF_REUSE),
one instrumented pass (KHP_RENDER_STATS: the STATS k_extend instances) of the
metric row counts, per bounce and per wave traversal iteration, how many lanes
fetch the SAME candidate (cone / triangle) record: every leaf-record fetch is
binned by the size of its group of lanes fetching that record in the same
iteration.  Prints one JSON line: per bounce the share of fetches in groups of
1, 2, 3-4, 5-8, 9-16, 17-32, 33-64 lanes and lanes per distinct record.
usage: KHP_LIB=variants/libkirk_leafreuse.so python tools/leaf_reuse.py [spp=8]"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import HipContext, native, scenes  # noqa: E402

SPP = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W, H, D = 1920, 1080, 5
ctx = HipContext(0)
lib = ctx.lib
if not hasattr(lib, "khp_debug_leaf_reuse"):
    raise SystemExit("not a KHP_LEAF_REUSE build (set KHP_LIB)")
lib.khp_debug_leaf_reuse.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
buf = (ctypes.c_uint64 * 128)()
scenes.config3_device(ctx, W, H, n_strands=1_000_000)
ctx.build_accel()
native.check(lib, lib.khp_debug_leaf_reuse(ctx.ptr, buf), "khp_debug_leaf_reuse")   # reset
ctx.render(W, H, SPP, D, first_sample=0, readback=False, stats=True)
native.check(lib, lib.khp_debug_leaf_reuse(ctx.ptr, buf), "khp_debug_leaf_reuse")
st = ctx.stats()
names = ["1", "2", "3-4", "5-8", "9-16", "17-32", "33-64"]
out = {"config": f"metric row {W}x{H} {SPP} spp depth {D}, one instrumented pass", "bounces": []}
for b in range(D):
    row = [buf[b * 8 + k] for k in range(8)]
    fetches = sum(row[:7])
    if not fetches:
        continue
    out["bounces"].append({"bounce": b, "leaf_fetches": fetches, "distinct_records": row[7],
                           "lanes_per_record": round(fetches / row[7], 3),
                           "share_by_group": {n: round(row[k] / fetches, 4) for k, n in enumerate(names)},
                           "records_tested": st["bounce_prims"][b]})
print(json.dumps(out), flush=True)
ctx.close()
