"""MI355X-native fur path-tracing core (the hot path of lucashilbig/BA_Pathtracing_Fur).

The product is libkirk_hip.so (HIP kernels for gfx950 behind the C-ABI in
include/kirk_hip.h).  This package holds its ctypes binding, the seeded scene
inputs, and a KIRK-shaped host interface.  No pixel is computed in Python and
there is no CPU fallback.
"""
import os as _os

# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues per process (4 by
# default).  Two frames in flight use four path-set streams plus the context
# stream; with only 4 queues two streams share one, and a queue whose head
# waits on an event stalls the other stream's kernels behind it (measured:
# 386 -> 426 Msamples/s and 12.2 -> 8.9 ms per rank-of-8 frame with 8 queues).
# Read when the HIP runtime initialises, i.e. before the first khp_create.
# Values below 8 (HIP's default of 4 is often exported explicitly) are raised
# to 8 unless KHP_KEEP_HW_QUEUES=1.
_HW_QUEUES = 8
if _os.environ.get("KHP_KEEP_HW_QUEUES") != "1":
    try:
        _q = int(_os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        _q = 0
    if _q < _HW_QUEUES:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(_HW_QUEUES)

from . import native  # noqa: E402
from .pathtracer import BVH, BsdfFactory, HipContext, PathTracer, ShaderFactory, comm_unique_id  # noqa: E402
from .scenes import SceneData, build_config  # noqa: E402

__all__ = ["native", "BVH", "BsdfFactory", "HipContext", "PathTracer", "ShaderFactory", "SceneData",
           "build_config", "comm_unique_id"]
