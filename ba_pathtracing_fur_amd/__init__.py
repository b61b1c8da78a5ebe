"""MI355X-native fur path-tracing core (the hot path of lucashilbig/BA_Pathtracing_Fur).

The product is libkirk_hip.so (HIP kernels for gfx950 behind the C-ABI in
include/kirk_hip.h).  This package holds its ctypes binding, the seeded scene
inputs, and a KIRK-shaped host interface.  No pixel is computed in Python and
there is no CPU fallback.
"""
import os as _os


def set_hw_queues(n: int = 8) -> None:
    """Set GPU_MAX_HW_QUEUES (hardware queues per process; HIP's default is 4)
    for this process.  HIP reads it once, when the runtime initialises, so this
    must run before the first khp_create (or any other HIP call) in the process.
    The default context (one batch in flight) uses three streams, which fit in
    the default four queues; with khp_ctx_params.frames_in_flight = 2 or 3 the
    extra streams share queues unless this is raised.  Never
    called implicitly: the host program decides."""
    _os.environ["GPU_MAX_HW_QUEUES"] = str(int(n))


from . import native  # noqa: E402,F401
from .pathtracer import BVH, BsdfFactory, HipContext, PathTracer, ShaderFactory, comm_unique_id  # noqa: E402
from .scenes import SceneData, build_config  # noqa: E402

__all__ = ["set_hw_queues", "native", "BVH", "BsdfFactory", "HipContext", "PathTracer", "ShaderFactory", "SceneData",
           "build_config", "comm_unique_id"]
