"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU restatement (oracle/).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline import this.
The product (ba_pathtracing_fur_amd / libkirk_hip.so) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_float, c_int, c_int32, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libkirk_oracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def _fp(a):
    return a.ctypes.data_as(POINTER(c_float))


def _ip(a):
    return a.ctypes.data_as(POINTER(c_int32))


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    P = POINTER
    sig = {
        "ko_create": (c_int, [P(c_void_p), c_void_p]),
        "ko_destroy": (None, [c_void_p]),
        "ko_render": (c_int, [c_void_p, c_void_p, c_int, P(c_float)]),
        "ko_render_rows": (c_int, [c_void_p, c_void_p, c_int, c_uint32, c_uint32, P(c_float)]),
        "ko_render_rows_step": (c_int, [c_void_p, c_void_p, c_int, c_uint32, c_uint32, c_uint32, P(c_float)]),
        "ko_trace_closest": (c_int, [c_void_p, c_uint32, P(c_float), P(c_float), P(c_float), P(c_int32),
                                     P(c_float), P(c_uint64), P(c_uint64)]),
        "ko_trace_any": (c_int, [c_void_p, c_uint32, P(c_float), P(c_float), P(c_float), P(c_uint8)]),
        "ko_n_objects": (c_uint32, [c_void_p]),
        "ko_set_bdpt": (c_int, [c_void_p, c_void_p]),
        "ko_light_paths": (c_int, [c_void_p, c_uint32, c_uint32, P(c_float)]),
        "ko_env_color": (None, [c_void_p, P(c_float), P(c_float)]),
        "ko_tex_color": (None, [c_void_p, c_uint32, c_float, c_float, P(c_float)]),
        "ko_object_bounds": (None, [c_void_p, P(c_float)]),
        "ko_cone_records": (None, [c_void_p, P(c_float)]),
        "ko_tri_records": (None, [c_void_p, P(c_float), P(c_int32)]),
        "ko_bvh_nodes": (c_uint32, [c_void_p, P(c_float), P(c_int32), P(c_int32), P(c_int32)]),
        "ko_bvh_depth": (c_uint32, [c_void_p]),
        "ko_sinf": (c_float, [c_float]),
        "ko_cosf": (c_float, [c_float]),
        "ko_atan2f": (c_float, [c_float, c_float]),
        "ko_acosf": (c_float, [c_float]),
        "ko_asinf": (c_float, [c_float]),
        "ko_expf": (c_float, [c_float]),
        "ko_sinhf": (c_float, [c_float]),
        "ko_j0": (c_double, [c_double]),
        "ko_log_d": (c_double, [c_double]),
        "ko_exp_d": (c_double, [c_double]),
        "ko_pow_d": (c_double, [c_double, c_double]),
        "ko_rand_u32": (c_uint32, [c_uint32, c_uint32, c_uint32, c_uint32]),
        "ko_bsdf_sample": (c_int, [c_void_p, c_int, c_void_p, P(c_float), P(c_float), P(c_float), P(c_float), c_int,
                                   P(c_float), P(c_float), P(c_float)]),
        "ko_to_rgba8": (None, [c_uint32, P(c_float), P(c_uint8)]),
        "ko_tonemap": (c_int, [c_uint32, c_uint32, P(c_float), c_void_p, P(c_float), P(c_float), P(c_float)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class Oracle:
    """CPU restatement of KIRK's path tracer on a flattened scene (scenes.SceneData)."""

    def __init__(self, scene):
        self.lib = load()
        self.scene = scene
        self._desc = scene.desc()
        self.ptr = c_void_p()
        rc = self.lib.ko_create(ctypes.byref(self.ptr), ctypes.addressof(self._desc))
        if rc != 0:
            raise ValueError(f"ko_create failed ({rc})")

    def __del__(self):
        if getattr(self, "ptr", None):
            self.lib.ko_destroy(self.ptr)
            self.ptr = None

    @staticmethod
    def params(width, height, spp, depth, seed=0x4B49524B, first_sample=0, tile_size=64, tile_rank=0,
               tile_nranks=1):
        from ba_pathtracing_fur_amd import native as N
        return N.RenderParams(width, height, spp, depth, seed, first_sample, tile_size, tile_rank, tile_nranks, 0)

    def render(self, width, height, spp, depth, seed=0x4B49524B, first_sample=0, threads=None, out=None,
               tile_size=64, tile_rank=0, tile_nranks=1, rows=None):
        p = self.params(width, height, spp, depth, seed, first_sample, tile_size, tile_rank, tile_nranks)
        if out is None:
            out = np.zeros((height, width, 3), np.float32)
        n = threads or os.cpu_count() or 1
        if rows is None:
            rc = self.lib.ko_render(self.ptr, ctypes.addressof(p), n, _fp(out))
        else:
            step = rows[2] if len(rows) > 2 else 1
            rc = self.lib.ko_render_rows_step(self.ptr, ctypes.addressof(p), n, rows[0], rows[1], step, _fp(out))
        if rc != 0:
            raise ValueError(f"ko_render failed ({rc})")
        return out

    def set_bdpt(self, enabled=1, light_paths=256, vertices=4, bias=1e-4, bounce_bias=1e-4, min_pdf=1e-4,
                 image_plane=1):
        """The light-path variant (khp_bdpt_params, ABI 7) for the following renders."""
        from ba_pathtracing_fur_amd import native as N
        self._bd = N.BdptParams(enabled, light_paths, vertices, bias, bounce_bias, min_pdf, image_plane)
        rc = self.lib.ko_set_bdpt(self.ptr, ctypes.addressof(self._bd))
        if rc != 0:
            raise ValueError(f"ko_set_bdpt failed ({rc})")

    def light_paths(self, k, seed=0x4B49524B):
        """Subpaths of sample index k: [light_paths, n_lights, vertices, 10] (valid, pos, din, hit_color)."""
        n = self._bd.light_paths * len(self.scene.lights) * self._bd.vertices
        out = np.zeros((n, 10), np.float32)
        rc = self.lib.ko_light_paths(self.ptr, seed, k, _fp(out))
        if rc != 0:
            raise ValueError(f"ko_light_paths failed ({rc})")
        return out.reshape(self._bd.light_paths, len(self.scene.lights), self._bd.vertices, 10)

    def trace_closest(self, orig, direction):
        o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
        n = len(o)
        t = np.empty(n, np.float32)
        obj = np.empty(n, np.int32)
        uv = np.empty((n, 2), np.float32)
        nv = c_uint64()
        pt = c_uint64()
        self.lib.ko_trace_closest(self.ptr, n, _fp(o), _fp(d), _fp(t), _ip(obj), _fp(uv), ctypes.byref(nv),
                                  ctypes.byref(pt))
        return t, obj, uv, nv.value, pt.value

    def trace_any(self, orig, direction, tmax):
        o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
        tm = np.ascontiguousarray(tmax, np.float32).reshape(-1)
        hit = np.empty(len(o), np.uint8)
        self.lib.ko_trace_any(self.ptr, len(o), _fp(o), _fp(d), _fp(tm), hit.ctypes.data_as(POINTER(c_uint8)))
        return hit.astype(bool)

    def env_color(self, direction):
        """Environment::getColor for each direction (n, 3) -> (n, 3)."""
        d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
        out = np.empty_like(d)
        for i in range(len(d)):
            self.lib.ko_env_color(self.ptr, _fp(d[i]), _fp(out[i]))
        return out

    def tex_color(self, tex, x, y):
        """Texture::getColor of scene texture `tex` at (x, y) -> rgba."""
        out = np.empty(4, np.float32)
        self.lib.ko_tex_color(self.ptr, tex, x, y, _fp(out))
        return out

    def object_bounds(self):
        n = self.lib.ko_n_objects(self.ptr)
        out = np.empty((n, 9), np.float32)
        self.lib.ko_object_bounds(self.ptr, _fp(out))
        return out

    def cone_records(self):
        n = len(self.scene.cone_base_r0)
        out = np.empty((n, 18), np.float32)
        self.lib.ko_cone_records(self.ptr, _fp(out))
        return out

    def tri_records(self):
        n = len(self.scene.tri_v)
        out = np.empty((n, 24), np.float32)
        la = np.empty(n, np.int32)
        self.lib.ko_tri_records(self.ptr, _fp(out), _ip(la))
        return out, la

    def bvh(self):
        n = self.lib.ko_bvh_nodes(self.ptr, None, None, None, None)
        boxes = np.empty((n, 6), np.float32)
        first = np.empty(n, np.int32)
        count = np.empty(n, np.int32)
        ids = np.empty(self.lib.ko_n_objects(self.ptr), np.int32)
        self.lib.ko_bvh_nodes(self.ptr, _fp(boxes), _ip(first), _ip(count), _ip(ids))
        return boxes, first, count, ids, self.lib.ko_bvh_depth(self.ptr)

    def bsdf_sample(self, obj, mat, ray_in, n, sample, hair_u, flags_in=0):
        ri = np.asarray(ray_in, np.float32)
        nn = np.asarray(n, np.float32)
        s = np.asarray(sample, np.float32).copy()
        hu = np.asarray(hair_u, np.float32)
        out = np.empty(3, np.float32)
        pdf = c_float()
        f = np.empty(3, np.float32)
        fl = self.lib.ko_bsdf_sample(self.ptr, obj, ctypes.addressof(mat), _fp(ri), _fp(nn), _fp(s), _fp(hu),
                                     flags_in, _fp(out), ctypes.byref(pdf), _fp(f))
        return {"out": out, "pdf": pdf.value, "f": f, "flags": fl, "sample": s}


def to_rgba8(rgb: np.ndarray) -> np.ndarray:
    """Texture::setPixel byte conversion (oracle/kirk_tonemap.c): (H, W, 3) -> (H, W, 4) uint8."""
    lib = load()
    a = np.ascontiguousarray(rgb, np.float32)
    out = np.empty(a.shape[:2] + (4,), np.uint8)
    lib.ko_to_rgba8(a.shape[0] * a.shape[1], _fp(a), out.ctypes.data_as(POINTER(c_uint8)))
    return out


def tonemap(rgb: np.ndarray, tm) -> tuple[np.ndarray, float, float]:
    """Tonemapper::map (oracle/kirk_tonemap.c) on (H, W, 3) floats; tm: native.Tonemap.
    Returns (mapped floats, max luminance, world luminance)."""
    lib = load()
    a = np.ascontiguousarray(rgb, np.float32)
    out = np.empty_like(a)
    mx, wl = c_float(), c_float()
    rc = lib.ko_tonemap(a.shape[1], a.shape[0], _fp(a), ctypes.addressof(tm), _fp(out), ctypes.byref(mx),
                        ctypes.byref(wl))
    if rc != 0:
        raise ValueError("ko_tonemap: center window outside the image")
    return out, mx.value, wl.value
