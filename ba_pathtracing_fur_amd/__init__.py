"""MI355X-native fur path-tracing core (the hot path of lucashilbig/BA_Pathtracing_Fur).

The product is libkirk_hip.so (HIP kernels for gfx950 behind the C-ABI in
include/kirk_hip.h).  This package holds its ctypes binding, the seeded scene
inputs, and a KIRK-shaped host interface.  No pixel is computed in Python and
there is no CPU fallback.
"""
from . import native
from .pathtracer import BVH, BsdfFactory, HipContext, PathTracer, ShaderFactory, comm_unique_id
from .scenes import SceneData, build_config

__all__ = ["native", "BVH", "BsdfFactory", "HipContext", "PathTracer", "ShaderFactory", "SceneData",
           "build_config", "comm_unique_id"]
