"""ctypes view of the C-ABI in include/kirk_hip.h.

The product path is libkirk_hip.so (HIP kernels for gfx950).  There is no CPU
fallback: if the library is missing or no GPU is present, the calls fail
loudly (RuntimeError), they never route anywhere else.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int32, c_uint8, c_uint32, c_uint64, c_double, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libkirk_hip.so")

# enums (kirk_hip.h)
KHP_OK, KHP_EINVAL, KHP_ENOMEM, KHP_EDEVICE, KHP_ENOTREADY, KHP_EUNSUPPORTED = range(6)
STATUS_NAMES = {0: "KHP_OK", 1: "KHP_EINVAL", 2: "KHP_ENOMEM", 3: "KHP_EDEVICE", 4: "KHP_ENOTREADY",
                5: "KHP_EUNSUPPORTED"}

BSDF_NAMES = ["LambertianReflectionBSDF", "SpecularReflectionBSDF", "SpecularTransmissionBSDF", "GlossyBSDF",
              "GlassBSDF", "MilkGlassBSDF", "LambertianTransmissionBSDF", "EmissionBSDF", "TransparentBSDF",
              "MarschnerHairBSDF", "DEonHairBSDF"]
SHADER_NAMES = ["SimpleShader", "MarschnerHairShader"]
LIGHT_POINT, LIGHT_QUAD, LIGHT_SPOT, LIGHT_SUN = 0, 1, 2, 3

RENDER_OUT_DEVICE = 1 << 0
RENDER_NO_READBACK = 1 << 1
RENDER_STATS = 1 << 2
RENDER_ASYNC = 1 << 3
CTX_STATS = 1 << 0
CTX_HOST_BUILD = 1 << 1

F3 = c_float * 3


class Material(ctypes.Structure):
    _fields_ = [("bsdf", c_int32), ("shader", c_int32), ("diffuse", F3), ("specular", F3), ("volume", F3),
                ("emission", F3), ("ior", c_float), ("roughness", c_float)]


class Light(ctypes.Structure):
    _fields_ = [("kind", c_int32), ("color", F3), ("position", F3), ("direction", F3), ("size", c_float * 2),
                ("radius", c_float), ("att_const", c_float), ("att_lin", c_float), ("att_quad", c_float),
                ("inner_angle", c_float), ("outer_angle", c_float)]


class Environment(ctypes.Structure):
    _fields_ = [("color", F3), ("ambient", F3)]


class Camera(ctypes.Structure):
    _fields_ = [("position", F3), ("bottom_left", F3), ("axis_x", F3), ("axis_y", F3), ("pixel_size", c_float)]


TEX_WRAP_CLAMP, TEX_WRAP_TILE = 0, 1
ENV_COLOR, ENV_CUBE_MAP, ENV_SPHERE_MAP = 0, 1, 2


class Texture(ctypes.Structure):
    """khp_texture (ABI 6): KIRK::Texture's 8-bit texels."""
    _fields_ = [("width", c_uint32), ("height", c_uint32), ("channels", c_uint32), ("wrap_mode", c_uint32),
                ("data", POINTER(c_uint8))]


class MaterialTextures(ctypes.Structure):
    """khp_material_textures (ABI 6): texture index per parameter, -1 = the material value."""
    _fields_ = [("diffuse", c_int32), ("specular", c_int32), ("volume", c_int32), ("emission", c_int32),
                ("roughness", c_int32)]


class EnvMap(ctypes.Structure):
    """khp_env_map (ABI 6): Environment::m_type and its textures."""
    _fields_ = [("type", c_int32), ("tex", c_int32 * 6)]


class SceneDesc(ctypes.Structure):
    _fields_ = [("n_tris", c_uint32), ("tri_v", POINTER(c_float)), ("tri_n", POINTER(c_float)),
                ("tri_mat", POINTER(c_uint32)), ("n_cones", c_uint32), ("cone_base_r0", POINTER(c_float)),
                ("cone_apex_r1", POINTER(c_float)), ("cone_mat", POINTER(c_uint32)), ("n_materials", c_uint32),
                ("materials", POINTER(Material)), ("n_lights", c_uint32), ("lights", POINTER(Light)),
                ("env", Environment), ("camera", Camera), ("tri_frame", POINTER(c_float)),
                ("n_cone_models", c_uint32), ("cone_models", POINTER(c_float)), ("cone_model", POINTER(c_uint32)),
                ("n_textures", c_uint32), ("textures", POINTER(Texture)),
                ("material_textures", POINTER(MaterialTextures)), ("tri_uv", POINTER(c_float)), ("env_map", EnvMap)]


class RenderParams(ctypes.Structure):
    _fields_ = [("width", c_uint32), ("height", c_uint32), ("spp", c_uint32), ("depth", c_uint32),
                ("seed", c_uint32), ("first_sample", c_uint32), ("tile_size", c_uint32), ("tile_rank", c_uint32),
                ("tile_nranks", c_uint32), ("flags", c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("n_objects", c_uint64), ("n_nodes", c_uint64), ("n_leaves", c_uint64), ("bvh_depth", c_uint32),
                ("max_leaf_size", c_uint32), ("device_bytes", c_uint64), ("build_ms", c_double),
                ("upload_ms", c_double), ("render_ms", c_double), ("extend_ms", c_double), ("shade_ms", c_double),
                ("shadow_ms", c_double), ("other_ms", c_double), ("extend_rays", c_uint64),
                ("shadow_rays", c_uint64), ("extend_launches", c_uint64), ("node_visits", c_uint64),
                ("prim_tests", c_uint64), ("shadow_node_visits", c_uint64), ("shadow_prim_tests", c_uint64),
                ("stack_spills", c_uint64), ("bounce_rays", c_uint64 * 16), ("bounce_nodes", c_uint64 * 16),
                ("bounce_prims", c_uint64 * 16), ("bounce_shadow_rays", c_uint64 * 16),
                ("bounce_shadow_nodes", c_uint64 * 16), ("bounce_shadow_prims", c_uint64 * 16),
                ("bounce_extend_ms", c_double * 16), ("bounce_shadow_ms", c_double * 16),
                ("bounce_wave_iters", c_uint64 * 16), ("bounce_lanes_busy", c_uint64 * 16),
                ("bounce_shadow_wave_iters", c_uint64 * 16), ("bounce_shadow_lanes_busy", c_uint64 * 16),
                ("step_cycles", c_uint64 * 4), ("bvh_on_device", c_uint32), ("subframes", c_uint32),
                ("flatten_ms", c_double), ("bvh_ms", c_double), ("bvh_kernel_ms", c_double), ("layout_ms", c_double),
                ("flatten_kernel_ms", c_double), ("layout_kernel_ms", c_double),
                ("extend_pruned_pops", c_uint64), ("shadow_pruned_pops", c_uint64), ("frames", c_uint64),
                ("extend_busy_ms", c_double), ("shadow_finish_ms", c_double), ("shadow_launches", c_uint64),
                ("ahead_finished", c_uint64), ("ahead_resumed", c_uint64)]

    def as_dict(self) -> dict:
        return {k: (list(getattr(self, k)) if not isinstance(getattr(self, k), (int, float)) else getattr(self, k))
                for k, _ in self._fields_}


class CtxParams(ctypes.Structure):
    """khp_ctx_params (ABI 13 layout, 64 bytes; path_order since ABI 9, wide_from since
    ABI 10, path_kernel since ABI 11, ray_sort_from and lds_nodes since ABI 12, render_ahead since
    ABI 13): scheduling knobs of a context; no value changes any result."""
    _fields_ = [("fuse_frames", c_uint32), ("frames_in_flight", c_uint32), ("chunk_paths", c_uint64),
                ("heavy_iters", c_uint32), ("dump_bounce", c_int32), ("trace_kernels", c_uint32),
                ("shade_order", c_uint32), ("serial_stages", c_uint32), ("path_order", c_uint32),
                ("wide_from", c_uint32), ("path_kernel", c_uint32), ("ray_sort_from", c_uint32),
                ("lds_nodes", c_uint32), ("render_ahead", c_uint32), ("path_from", c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class BdptParams(ctypes.Structure):
    """khp_bdpt_params (ABI 7): the light-path (bidirectional) variant, SURVEY §8(f)4."""
    _fields_ = [("enabled", c_uint32), ("light_paths", c_uint32), ("vertices", c_uint32), ("bias", c_float),
                ("bounce_bias", c_float), ("min_pdf", c_float), ("image_plane", c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class Tonemap(ctypes.Structure):
    """khp_tonemap: KIRK::Tonemapper's parameters (Utils/Tonemapping.h:22-33)."""
    _fields_ = [("exposure", c_float), ("bias", c_float), ("gamma", c_float), ("contrast", c_float),
                ("white", c_float), ("black", c_float), ("rec_gamma", c_int32), ("center_weight", c_int32),
                ("kernel_multiplier", c_float), ("center_x", c_int32), ("center_y", c_int32)]

    @classmethod
    def defaults(cls, **kw) -> "Tonemap":
        t = cls(exposure=0.0, bias=0.85, gamma=1.0, contrast=0.0, white=1.0, black=0.0, rec_gamma=0,
                center_weight=0, kernel_multiplier=0.125, center_x=-1, center_y=-1)
        for k, v in kw.items():
            if not hasattr(t, k):
                raise AttributeError(f"khp_tonemap has no field {k}")
            setattr(t, k, v)
        return t


# every symbol the header declares (checked by tests/test_abi.py)
EXPORTED = ["khp_create", "khp_destroy", "khp_last_error", "khp_abi_version", "khp_set_scene", "khp_build_accel",
            "khp_render", "khp_read_framebuffer", "khp_trace_closest", "khp_trace_any", "khp_get_stats",
            "khp_comm_unique_id", "khp_comm_init", "khp_gather_framebuffer", "khp_bsdf_kind_from_name",
            "khp_bsdf_name", "khp_shader_kind_from_name", "khp_camera_setup", "khp_fibers_to_cones",
            "khp_gen_hairball", "khp_gen_icosphere", "khp_gen_torus", "khp_host_build", "khp_debug_queue",
            "khp_read_rgba8", "khp_tonemap_defaults", "khp_read_bvh",
            "khp_read_layout", "khp_set_scene_device", "khp_gen_hairball_device", "khp_device_alloc",
            "khp_device_free", "khp_device_copy", "khp_fibers_to_triangles", "khp_gen_hairball_tris_device",
            "khp_sync", "khp_ctx_params_defaults", "khp_set_params", "khp_get_params", "khp_debug_shadow_queue",
            "khp_bdpt_params_defaults", "khp_set_bdpt", "khp_get_bdpt", "khp_gather_plan",
            "khp_read_rgba8_async", "khp_snapshot_wait", "khp_comm_init_local", "khp_comm_set_timeout",
            "khp_tonemap_log_sum", "khp_set_camera", "khp_debug_comm_wait"]

# the include/kirk_hip.h this module mirrors (load_library refuses another)
ABI_VERSION = 13

_lib = None


def fptr(a: np.ndarray):
    return a.ctypes.data_as(POINTER(c_float))


def uptr(a: np.ndarray):
    return a.ctypes.data_as(POINTER(c_uint32))


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libkirk_hip.so; raises RuntimeError if it was not built.

    `path`, or the KHP_LIB environment variable, selects another build of the
    same ABI (tools/build_variant.sh + tools/gpu_variants.sh A/B runs); the
    library itself reads no environment."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("KHP_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"HIP core not built: {p} missing (run __graft_entry__.build())")
    lib = ctypes.CDLL(p)
    P = POINTER
    sig = {
        "khp_create": (c_int, [P(c_void_p), c_int, c_uint32]),
        "khp_destroy": (None, [c_void_p]),
        "khp_last_error": (c_char_p, []),
        "khp_abi_version": (c_int, []),
        "khp_set_scene": (c_int, [c_void_p, P(SceneDesc)]),
        "khp_build_accel": (c_int, [c_void_p]),
        "khp_render": (c_int, [c_void_p, P(RenderParams), c_void_p]),
        "khp_sync": (c_int, [c_void_p]),
        "khp_ctx_params_defaults": (None, [P(CtxParams)]),
        "khp_set_params": (c_int, [c_void_p, P(CtxParams)]),
        "khp_get_params": (c_int, [c_void_p, P(CtxParams)]),
        "khp_bdpt_params_defaults": (None, [P(BdptParams)]),
        "khp_set_bdpt": (c_int, [c_void_p, P(BdptParams)]),
        "khp_set_camera": (c_int, [c_void_p, P(Camera)]),
        "khp_debug_comm_wait": (c_int, [c_void_p, c_int, c_uint32, c_uint32, P(c_double)]),
        "khp_get_bdpt": (c_int, [c_void_p, P(BdptParams)]),
        "khp_read_framebuffer": (c_int, [c_void_p, P(c_float)]),
        "khp_read_rgba8": (c_int, [c_void_p, P(Tonemap), P(c_uint8)]),
        "khp_tonemap_defaults": (None, [P(Tonemap)]),
        "khp_read_rgba8_async": (c_int, [c_void_p, P(c_uint8), P(c_uint64)]),
        "khp_snapshot_wait": (c_int, [c_void_p, c_uint64, c_int]),
        "khp_set_scene_device": (c_int, [c_void_p, P(SceneDesc)]),
        "khp_gen_hairball_device": (c_int, [c_void_p, c_uint32, c_uint32, P(c_float), c_float, c_float, c_uint32,
                                            c_void_p, c_void_p]),
        "khp_fibers_to_triangles": (c_int, [c_uint32, c_uint32, P(c_float), P(c_float), c_uint32, P(c_float),
                                            P(c_float), P(c_float)]),
        "khp_gen_hairball_tris_device": (c_int, [c_void_p, c_uint32, c_uint32, P(c_float), c_float, c_float,
                                                 c_uint32, c_uint32, c_void_p, c_void_p, c_void_p]),
        "khp_device_alloc": (c_int, [c_void_p, ctypes.c_size_t, P(c_void_p)]),
        "khp_device_free": (c_int, [c_void_p, c_void_p]),
        "khp_device_copy": (c_int, [c_void_p, c_void_p, c_void_p, ctypes.c_size_t, c_int]),
        "khp_read_layout": (c_int, [c_void_p, P(c_uint32), P(c_uint32), c_void_p, P(c_float), P(c_uint32)]),
        "khp_read_bvh": (c_int, [c_void_p, P(c_uint32), P(c_uint32), P(c_float), P(c_int32), P(c_int32), P(c_int32)]),
        "khp_trace_closest": (c_int, [c_void_p, c_uint32, P(c_float), P(c_float), P(c_float), P(c_int32),
                                      P(c_float)]),
        "khp_trace_any": (c_int, [c_void_p, c_uint32, P(c_float), P(c_float), P(c_float), P(c_uint8)]),
        "khp_get_stats": (c_int, [c_void_p, P(Stats)]),
        "khp_comm_unique_id": (c_int, [P(c_uint8)]),
        "khp_comm_init": (c_int, [c_void_p, c_int, c_int, P(c_uint8)]),
        "khp_comm_set_timeout": (c_int, [c_void_p, c_uint32]),
        "khp_tonemap_log_sum": (c_int, [P(ctypes.c_double), ctypes.c_uint64, c_float, P(c_float)]),
        "khp_gather_framebuffer": (c_int, [c_void_p, P(RenderParams), c_int]),
        "khp_comm_init_local": (c_int, [P(c_void_p), c_int]),
        "khp_gather_plan": (c_int, [c_uint32, c_uint32, c_uint32, c_int, c_int, c_int, P(c_uint64), P(c_uint32),
                                    P(c_uint64)]),
        "khp_bsdf_kind_from_name": (c_int, [c_char_p]),
        "khp_bsdf_name": (c_char_p, [c_int]),
        "khp_shader_kind_from_name": (c_int, [c_char_p]),
        "khp_camera_setup": (c_int, [P(c_float), P(c_float), P(c_float), c_float, c_float, c_float, c_uint32,
                                     c_uint32, P(Camera)]),
        "khp_fibers_to_cones": (c_int, [c_uint32, c_uint32, P(c_float), P(c_float), P(c_float), P(c_float)]),
        "khp_gen_hairball": (c_int, [c_uint32, c_uint32, P(c_float), c_float, c_float, c_uint32, P(c_float),
                                     P(c_float)]),
        "khp_gen_icosphere": (c_int, [c_uint32, P(c_float), c_float, P(c_float), P(c_float)]),
        "khp_gen_torus": (c_int, [c_uint32, c_uint32, P(c_float), c_float, c_float, P(c_float), P(c_float)]),
        "khp_debug_queue": (c_int, [c_void_p, P(c_uint32), P(c_float), P(c_float)]),
        "khp_debug_shadow_queue": (c_int, [c_void_p, P(c_uint32), P(c_float), P(c_float), P(c_float)]),
        "khp_host_build": (c_int, [P(SceneDesc), P(c_uint32), P(c_uint32), P(c_float), P(c_int32), P(c_int32),
                                   P(c_int32), P(c_float), P(c_float)]),
    }
    lib.khp_abi_version.restype = c_int
    lib.khp_abi_version.argtypes = []
    abi = lib.khp_abi_version()
    if abi != ABI_VERSION:   # the structs above would be read with the wrong layout
        raise RuntimeError(f"{p}: ABI {abi}, this package needs ABI {ABI_VERSION} (rebuild: __graft_entry__.build())")
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


class KhpError(RuntimeError):
    def __init__(self, status: int, where: str, msg: str):
        super().__init__(f"{where}: {STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


def check(lib, status: int, where: str):
    if status != KHP_OK:
        raise KhpError(status, where, (lib.khp_last_error() or b"").decode())


def tonemap_log_sum(terms: np.ndarray, start: float = 0.0) -> np.float32:
    """khp_tonemap_log_sum (host only): KIRK's float running sum of double terms, in order."""
    lib = load_library()
    t = np.ascontiguousarray(terms, dtype=np.float64)
    out = c_float(0.0)
    check(lib, lib.khp_tonemap_log_sum(t.ctypes.data_as(POINTER(ctypes.c_double)), t.size, float(start),
                                       ctypes.byref(out)), "khp_tonemap_log_sum")
    return np.float32(out.value)


def host_build(scene) -> dict:
    """Flatten + BVH build of the product, run on the host (no GPU): khp_host_build."""
    lib = load_library()
    d = scene.desc()
    nn, dep = c_uint32(), c_uint32()
    ip = lambda a: a.ctypes.data_as(POINTER(c_int32))
    check(lib, lib.khp_host_build(ctypes.byref(d), ctypes.byref(nn), ctypes.byref(dep), None, None, None, None, None,
                                  None), "khp_host_build")
    n, m = nn.value, scene.n_objects
    boxes = np.empty((n, 6), np.float32)
    first = np.empty(n, np.int32)
    count = np.empty(n, np.int32)
    ids = np.empty(m, np.int32)
    bounds = np.empty((m, 9), np.float32)
    rec = np.empty((m, 16), np.float32)
    check(lib, lib.khp_host_build(ctypes.byref(d), ctypes.byref(nn), ctypes.byref(dep), fptr(boxes), ip(first),
                                  ip(count), ip(ids), fptr(bounds), fptr(rec)), "khp_host_build")
    return {"boxes": boxes, "first": first, "count": count, "ids": ids, "bounds": bounds, "records": rec,
            "depth": dep.value}


def gather_plan(width: int, height: int, tile: int, nranks: int, rank: int, root: int = 0):
    """khp_gather_plan (host only): (counts[nranks], pixel indices) that
    khp_gather_framebuffer moves, as seen from `rank`."""
    lib = load_library()
    n = c_uint64()
    check(lib, lib.khp_gather_plan(width, height, tile, nranks, rank, root, None, None, ctypes.byref(n)),
          "khp_gather_plan")
    counts = np.zeros(nranks, np.uint64)
    pix = np.zeros(max(1, n.value), np.uint32)
    check(lib, lib.khp_gather_plan(width, height, tile, nranks, rank, root, counts.ctypes.data_as(POINTER(c_uint64)),
                                   uptr(pix), ctypes.byref(n)), "khp_gather_plan")
    return counts, pix[:n.value]
