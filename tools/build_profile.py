"""Dev tool: config3 (1M strands) generated, flattened and built on the device; prints the setup stats.

    python tools/build_profile.py [n_strands] [reps]
Run under rocprofv3 --kernel-trace --stats for per-kernel times of the build.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from ba_pathtracing_fur_amd import scenes  # noqa: E402
from ba_pathtracing_fur_amd.pathtracer import HipContext  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = HipContext(0)
for r in range(reps):
    scenes.config3_device(ctx, 1920, 1080, n_strands=n)
    ctx.build_accel()
    st = ctx.stats()
    print(f"rep {r}: flatten {st['flatten_ms']:.1f} ms ({st['flatten_kernel_ms']:.2f} k), bvh {st['bvh_ms']:.1f} ms "
          f"({st['bvh_kernel_ms']:.1f} k), layout {st['layout_ms']:.1f} ms ({st['layout_kernel_ms']:.2f} k), "
          f"upload {st['upload_ms']:.1f} ms, nodes {st['n_nodes']}, depth {st['bvh_depth']}", flush=True)
ctx.close()
