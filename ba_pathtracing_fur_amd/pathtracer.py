"""KIRK-shaped host interface over the C-ABI.

Mirrors the plugin surface the HIP core drops in behind:
  * `PathTracer` ~ KIRK::CPU::PathTracer / CPU_Raytracer (CPU_PathTracer.h:33-166,
    CPU_Raytracer.h:16-78): init(scene), set_sample_count, set_depth, render()
    (one sample of every pixel, like one full pass of KIRK's segmented render),
    render_to_texture(), get_current_sample_count(), reset();
  * `BVH` ~ KIRK::CPU::CPU_DataStructure (CPU_DataStructure.h:25-28):
    closest_intersection / is_intersection, batched over ray arrays;
  * `BsdfFactory` / `ShaderFactory` ~ the name registries (BsdfFactory.cpp:28-55,
    ShaderFactory.cpp:29-67): unknown names raise ValueError where KIRK throws
    std::invalid_argument.
Everything runs on the GPU through libkirk_hip.so; nothing here computes pixels.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native as N
from .scenes import SceneData


class BsdfFactory:
    @staticmethod
    def get_bsdf(name: str) -> int:
        lib = N.load_library()
        k = lib.khp_bsdf_kind_from_name(name.encode())
        if k < 0:
            raise ValueError(f"There is no BSDF registered with the name {name}")
        return k

    @staticmethod
    def names() -> list[str]:
        return list(N.BSDF_NAMES)


class ShaderFactory:
    @staticmethod
    def get_shader(name: str) -> int:
        lib = N.load_library()
        k = lib.khp_shader_kind_from_name(name.encode())
        if k < 0:
            raise ValueError(f"There is no Shader registered with the name {name}")
        return k


class DeviceBuffer:
    """A device allocation on a context's GPU (khp_device_alloc); freed with the object."""

    def __init__(self, ctx: "HipContext", nbytes: int):
        self.ctx, self.nbytes = ctx, int(nbytes)
        p = ctypes.c_void_p()
        N.check(ctx.lib, ctx.lib.khp_device_alloc(ctx.ptr, self.nbytes, ctypes.byref(p)), "khp_device_alloc")
        self.ptr = p.value

    @classmethod
    def from_array(cls, ctx: "HipContext", a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(ctx, a.nbytes)
        N.check(ctx.lib, ctx.lib.khp_device_copy(ctx.ptr, b.ptr, a.ctypes.data_as(ctypes.c_void_p), a.nbytes, 1),
                "khp_device_copy")
        return b

    def to_array(self, shape, dtype) -> np.ndarray:
        out = np.empty(shape, dtype)
        assert out.nbytes <= self.nbytes
        N.check(self.ctx.lib, self.ctx.lib.khp_device_copy(self.ctx.ptr, out.ctypes.data_as(ctypes.c_void_p), self.ptr,
                                                           out.nbytes, 0), "khp_device_copy")
        return out

    def free(self):
        if self.ptr and self.ctx.ptr:
            self.ctx.lib.khp_device_free(self.ctx.ptr, self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class HipContext:
    """One khp_ctx: one GPU, one stream (one process per GPU)."""

    def __init__(self, device: int = 0, stats: bool = False, host_build: bool = False):
        self.lib = N.load_library()
        self.ptr = ctypes.c_void_p()
        flags = (N.CTX_STATS if stats else 0) | (N.CTX_HOST_BUILD if host_build else 0)
        N.check(self.lib, self.lib.khp_create(ctypes.byref(self.ptr), device, flags), "khp_create")
        self._scene = None

    def close(self):
        if self.ptr:
            self.lib.khp_destroy(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, scene: SceneData):
        d = scene.desc()
        N.check(self.lib, self.lib.khp_set_scene(self.ptr, ctypes.byref(d)), "khp_set_scene")
        self._scene = scene
        self._n_objects = scene.n_objects

    def hairball_device(self, n_strands: int, center, ball_radius: float, root_radius: float = 0.004,
                        verts: int = 10, seed: int = 0x4B49524B):
        """Seeded hairball cones generated in HBM (khp_gen_hairball_device): (base_r0, apex_r1, n_cones)."""
        nc = n_strands * (verts - 1)
        base, apex = DeviceBuffer(self, 16 * nc), DeviceBuffer(self, 16 * nc)
        c = np.asarray(center, np.float32)
        N.check(self.lib, self.lib.khp_gen_hairball_device(self.ptr, n_strands, verts, N.fptr(c), ball_radius,
                                                           root_radius, seed, base.ptr, apex.ptr),
                "khp_gen_hairball_device")
        return base, apex, nc

    def set_scene_device(self, scene: SceneData, cones=None):
        """khp_set_scene_device: the scene's geometry copied to HBM first, or, with
        cones=(base_r0, apex_r1, n, material) from hairball_device, those cones in
        place of the scene's own (which must then be empty)."""
        d = scene.desc()
        keep = []

        def dev(a):
            b = DeviceBuffer.from_array(self, a)
            keep.append(b)
            return b.ptr

        if len(scene.tri_v):
            d.tri_v = ctypes.cast(dev(scene.tri_v), ctypes.POINTER(ctypes.c_float))
            d.tri_n = ctypes.cast(dev(scene.tri_n), ctypes.POINTER(ctypes.c_float))
            d.tri_mat = ctypes.cast(dev(scene.tri_mat), ctypes.POINTER(ctypes.c_uint32))
            d.tri_frame = ctypes.cast(dev(scene.frames()), ctypes.POINTER(ctypes.c_float))
            if scene.textures:
                d.tri_uv = ctypes.cast(dev(scene.uvs()), ctypes.POINTER(ctypes.c_float))
        if cones is not None:
            if len(scene.cone_base_r0):
                raise ValueError("scene already has cones")
            base, apex, nc, mat = cones
            d.n_cones = nc
            d.cone_base_r0 = ctypes.cast(base.ptr, ctypes.POINTER(ctypes.c_float))
            d.cone_apex_r1 = ctypes.cast(apex.ptr, ctypes.POINTER(ctypes.c_float))
            d.cone_mat = ctypes.cast(dev(np.full(nc, mat, np.uint32)), ctypes.POINTER(ctypes.c_uint32))
        elif len(scene.cone_base_r0):
            d.cone_base_r0 = ctypes.cast(dev(scene.cone_base_r0), ctypes.POINTER(ctypes.c_float))
            d.cone_apex_r1 = ctypes.cast(dev(scene.cone_apex_r1), ctypes.POINTER(ctypes.c_float))
            d.cone_mat = ctypes.cast(dev(scene.cone_mat), ctypes.POINTER(ctypes.c_uint32))
            if len(scene.cone_models):
                d.cone_model = ctypes.cast(dev(scene.cone_model), ctypes.POINTER(ctypes.c_uint32))
        N.check(self.lib, self.lib.khp_set_scene_device(self.ptr, ctypes.byref(d)), "khp_set_scene_device")
        for b in keep:
            b.free()
        self._scene = scene
        self._n_objects = d.n_tris + d.n_cones

    def build_accel(self):
        N.check(self.lib, self.lib.khp_build_accel(self.ptr), "khp_build_accel")

    def params(self) -> dict:
        """khp_get_params: the context's scheduling parameters (khp_ctx_params)."""
        prm = N.CtxParams()
        N.check(self.lib, self.lib.khp_get_params(self.ptr, ctypes.byref(prm)), "khp_get_params")
        return prm.as_dict()

    def set_params(self, **kw) -> dict:
        """khp_set_params with the given fields changed (fuse_frames, frames_in_flight,
        chunk_paths, heavy_iters, dump_bounce, trace_kernels, shade_order, serial_stages,
        path_order, wide_from, path_kernel, ray_sort_from, lds_nodes, render_ahead); returns the previous values."""
        prm = N.CtxParams()
        N.check(self.lib, self.lib.khp_get_params(self.ptr, ctypes.byref(prm)), "khp_get_params")
        old = prm.as_dict()
        for k, v in kw.items():
            if k not in old:
                raise AttributeError(f"khp_ctx_params has no field {k}")
            setattr(prm, k, int(v))
        N.check(self.lib, self.lib.khp_set_params(self.ptr, ctypes.byref(prm)), "khp_set_params")
        return old

    def set_camera(self, camera: "N.Camera"):
        """khp_set_camera (ABI 13): a new camera for the next render, nothing rebuilt
        (KIRK's GUI moving the Camera between PathTracer::render calls)."""
        N.check(self.lib, self.lib.khp_set_camera(self.ptr, ctypes.byref(camera)), "khp_set_camera")

    def set_bdpt(self, **kw) -> dict:
        """khp_set_bdpt with the given khp_bdpt_params fields changed (enabled,
        light_paths, vertices, bias, bounce_bias, min_pdf); returns the previous values."""
        prm = N.BdptParams()
        N.check(self.lib, self.lib.khp_get_bdpt(self.ptr, ctypes.byref(prm)), "khp_get_bdpt")
        old = prm.as_dict()
        for k, v in kw.items():
            if k not in old:
                raise AttributeError(f"khp_bdpt_params has no field {k}")
            setattr(prm, k, v)
        N.check(self.lib, self.lib.khp_set_bdpt(self.ptr, ctypes.byref(prm)), "khp_set_bdpt")
        return old

    def render(self, width, height, spp, depth, seed=0x4B49524B, first_sample=0, tile_size=64, tile_rank=0,
               tile_nranks=1, out: np.ndarray | None = None, readback=True, stats=False,
               async_: bool = False) -> np.ndarray | None:
        """khp_render.  async_=True (no readback, no stats) enqueues the frame and
        returns at once; frames in flight overlap; sync() completes them."""
        if async_:
            readback = False
        flags = ((0 if readback else N.RENDER_NO_READBACK) | (N.RENDER_STATS if stats else 0) |
                 (N.RENDER_ASYNC if async_ else 0))
        p = N.RenderParams(width, height, spp, depth, seed, first_sample, tile_size, tile_rank, tile_nranks, flags)
        if readback and out is None:
            out = np.zeros((height, width, 3), np.float32)
        ptr = out.ctypes.data_as(ctypes.c_void_p) if (readback and out is not None) else None
        N.check(self.lib, self.lib.khp_render(self.ptr, ctypes.byref(p), ptr), "khp_render")
        return out

    def sync(self):
        """khp_sync: complete every asynchronous frame; stats() then sums them."""
        N.check(self.lib, self.lib.khp_sync(self.ptr), "khp_sync")

    def read_bvh(self) -> dict:
        """The tree khp_build_accel built (khp_read_bvh), in khp_host_build's layout."""
        nn, dep = ctypes.c_uint32(), ctypes.c_uint32()
        N.check(self.lib, self.lib.khp_read_bvh(self.ptr, ctypes.byref(nn), ctypes.byref(dep), None, None, None, None),
                "khp_read_bvh")
        n = nn.value
        boxes = np.empty((n, 6), np.float32)
        first = np.empty(n, np.int32)
        count = np.empty(n, np.int32)
        ids = np.empty(getattr(self, "_n_objects", None) or self._scene.n_objects, np.int32)
        ip = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        N.check(self.lib, self.lib.khp_read_bvh(self.ptr, ctypes.byref(nn), ctypes.byref(dep), N.fptr(boxes), ip(first),
                                                ip(count), ip(ids)), "khp_read_bvh")
        return {"boxes": boxes, "first": first, "count": count, "ids": ids, "depth": dep.value}

    def read_layout(self) -> dict:
        """The traversal records in HBM (khp_read_layout): node records as (n, 16)
        uint32 words, primitive records (n_slots, 16) float32, aux (n_slots, 4) uint32."""
        nr, ns = ctypes.c_uint32(), ctypes.c_uint32()
        N.check(self.lib, self.lib.khp_read_layout(self.ptr, ctypes.byref(nr), ctypes.byref(ns), None, None, None),
                "khp_read_layout")
        nodes = np.zeros((nr.value, 16), np.uint32)
        prims = np.zeros((ns.value, 16), np.float32)
        aux = np.zeros((ns.value, 4), np.uint32)
        N.check(self.lib, self.lib.khp_read_layout(self.ptr, ctypes.byref(nr), ctypes.byref(ns),
                                                   nodes.ctypes.data_as(ctypes.c_void_p), N.fptr(prims),
                                                   N.uptr(aux)), "khp_read_layout")
        return {"nodes": nodes, "prims": prims, "aux": aux}

    def read_framebuffer(self, width, height) -> np.ndarray:
        out = np.zeros((height, width, 3), np.float32)
        N.check(self.lib, self.lib.khp_read_framebuffer(self.ptr, N.fptr(out)), "khp_read_framebuffer")
        return out

    def read_rgba8(self, width, height, tonemap: "N.Tonemap | None" = None) -> np.ndarray:
        """Device output stage (khp_read_rgba8): (H, W, 4) uint8, row 0 = bottom.

        tonemap=None: Texture::setPixel of the running mean; otherwise
        Tonemapper::map first (PathTracer::applyToneMapping)."""
        out = np.zeros((height, width, 4), np.uint8)
        tm = ctypes.byref(tonemap) if tonemap is not None else None
        N.check(self.lib, self.lib.khp_read_rgba8(self.ptr, tm, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))),
                "khp_read_rgba8")
        return out

    def read_rgba8_async(self, out: np.ndarray) -> int:
        """khp_read_rgba8_async: enqueue the 8-bit texture after the frames enqueued so
        far into `out` ((H, W, 4) uint8, kept alive by the caller); returns the ticket."""
        assert out.dtype == np.uint8 and out.flags.c_contiguous
        t = ctypes.c_uint64()
        N.check(self.lib, self.lib.khp_read_rgba8_async(self.ptr, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                                        ctypes.byref(t)), "khp_read_rgba8_async")
        return t.value

    def snapshot_wait(self, ticket: int, wait: bool = True) -> bool:
        """khp_snapshot_wait: True once snapshot `ticket` is in its buffer."""
        st = self.lib.khp_snapshot_wait(self.ptr, ticket, 1 if wait else 0)
        if st == N.KHP_ENOTREADY and not wait:
            return False
        N.check(self.lib, st, "khp_snapshot_wait")
        return True

    def trace_closest(self, orig, direction):
        o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
        n = len(o)
        t = np.empty(n, np.float32)
        obj = np.empty(n, np.int32)
        uv = np.empty((n, 2), np.float32)
        N.check(self.lib, self.lib.khp_trace_closest(self.ptr, n, N.fptr(o), N.fptr(d), N.fptr(t),
                                                     obj.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                     N.fptr(uv)), "khp_trace_closest")
        return t, obj, uv

    def trace_any(self, orig, direction, tmax):
        o = np.ascontiguousarray(orig, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(direction, np.float32).reshape(-1, 3)
        tm = np.ascontiguousarray(tmax, np.float32).reshape(-1)
        hit = np.empty(len(o), np.uint8)
        N.check(self.lib, self.lib.khp_trace_any(self.ptr, len(o), N.fptr(o), N.fptr(d), N.fptr(tm),
                                                 hit.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))),
                "khp_trace_any")
        return hit.astype(bool)

    def debug_queues(self):
        """The extension rays and the shadow rays (o, d, t_max) of bounce
        khp_ctx_params.dump_bounce of the last synchronous render."""
        n = ctypes.c_uint32()
        N.check(self.lib, self.lib.khp_debug_queue(self.ptr, ctypes.byref(n), None, None), "khp_debug_queue")
        o, d = np.empty((n.value, 3), np.float32), np.empty((n.value, 3), np.float32)
        N.check(self.lib, self.lib.khp_debug_queue(self.ptr, ctypes.byref(n), N.fptr(o), N.fptr(d)), "khp_debug_queue")
        m = ctypes.c_uint32()
        N.check(self.lib, self.lib.khp_debug_shadow_queue(self.ptr, ctypes.byref(m), None, None, None),
                "khp_debug_shadow_queue")
        so, sd, st = np.empty((m.value, 3), np.float32), np.empty((m.value, 3), np.float32), np.empty(m.value, np.float32)
        N.check(self.lib, self.lib.khp_debug_shadow_queue(self.ptr, ctypes.byref(m), N.fptr(so), N.fptr(sd), N.fptr(st)),
                "khp_debug_shadow_queue")
        return (o, d), (so, sd, st)

    def stats(self) -> dict:
        s = N.Stats()
        N.check(self.lib, self.lib.khp_get_stats(self.ptr, ctypes.byref(s)), "khp_get_stats")
        return s.as_dict()

    # --- multi-GPU --------------------------------------------------------------
    def comm_init(self, nranks: int, rank: int, uid: bytes, timeout_ms: int | None = None):
        """khp_comm_init; timeout_ms (khp_comm_set_timeout, ABI 11) bounds the init and
        every later wait of this context while the communicator exists."""
        if timeout_ms is not None:
            self.comm_set_timeout(timeout_ms)
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        N.check(self.lib, self.lib.khp_comm_init(self.ptr, nranks, rank, buf), "khp_comm_init")

    def comm_set_timeout(self, timeout_ms: int):
        N.check(self.lib, self.lib.khp_comm_set_timeout(self.ptr, int(timeout_ms)), "khp_comm_set_timeout")

    def gather_framebuffer(self, width, height, spp, depth, tile_size, nranks, rank, root=0):
        p = N.RenderParams(width, height, spp, depth, 0, 0, tile_size, rank, nranks, 0)
        N.check(self.lib, self.lib.khp_gather_framebuffer(self.ptr, ctypes.byref(p), root), "khp_gather_framebuffer")


def comm_init_local(ctxs) -> None:
    """khp_comm_init_local: contexts of this process as the ranks of one gather group
    (rank = position), the framebuffer gather moving over device copies, not RCCL."""
    lib = N.load_library()
    arr = (ctypes.c_void_p * len(ctxs))(*[c.ptr.value for c in ctxs])
    N.check(lib, lib.khp_comm_init_local(arr, len(ctxs)), "khp_comm_init_local")


def comm_unique_id() -> bytes:
    lib = N.load_library()
    buf = (ctypes.c_uint8 * 128)()
    N.check(lib, lib.khp_comm_unique_id(buf), "khp_comm_unique_id")
    return bytes(buf)


class BVH:
    """CPU_DataStructure-shaped batched queries on the GPU BVH."""

    def __init__(self, ctx: HipContext):
        self.ctx = ctx

    def closest_intersection(self, orig, direction):
        return self.ctx.trace_closest(orig, direction)

    def is_intersection(self, orig, direction, tmax):
        return self.ctx.trace_any(orig, direction, tmax)


class PathTracer:
    """KIRK::CPU::PathTracer on the HIP core (progressive, seeded)."""

    def __init__(self, scene: SceneData | None = None, depth: int = 8, device: int = 0, width: int = 256,
                 height: int = 256, seed: int = 0x4B49524B):
        self.ctx = HipContext(device)
        self.m_depth = depth                # CPU_Raytracer.h:73-75 default 8
        self.m_samples_per_pixel = 1        # PathTracer() default
        self.c_sample = 0
        self.width, self.height = width, height
        self.seed = seed
        self.m_use_tonemapping = False      # CPU_PathTracer.h:152
        self.m_tonemapper = N.Tonemap.defaults()  # CPU_PathTracer.h:38, Tonemapping.h:23-33
        if scene is not None:
            self.init(scene)

    def init(self, scene: SceneData):
        self.ctx.set_scene(scene)
        self.ctx.build_accel()
        self.reset()

    def set_depth(self, depth: int):
        self.m_depth = int(depth)

    def set_sample_count(self, samples: int):
        self.m_samples_per_pixel = int(samples)

    def get_current_sample_count(self) -> int:
        return self.c_sample

    def reset(self):
        self.c_sample = 0

    def render(self, n: int = 1):
        """Add up to `n` samples (KIRK's render() adds one sample per full pass)."""
        n = min(n, self.m_samples_per_pixel - self.c_sample)
        if n <= 0:
            return
        self.ctx.render(self.width, self.height, n, self.m_depth, self.seed, first_sample=self.c_sample,
                        readback=False)
        self.c_sample += n

    def render_to_texture(self) -> np.ndarray:
        """Render every remaining sample; returns the float RGB framebuffer (H, W, 3), row 0 = bottom."""
        self.render(self.m_samples_per_pixel - self.c_sample)
        return self.ctx.read_framebuffer(self.width, self.height)

    def texture_rgba8(self) -> np.ndarray:
        """The 8-bit render texture after the current samples, on the device:
        drawTexture's setPixel, or applyToneMapping when m_use_tonemapping
        (CPU_PathTracer.cpp:43-47, 61-104).  (H, W, 4) uint8, row 0 = bottom."""
        tm = self.m_tonemapper if self.m_use_tonemapping else None
        return self.ctx.read_rgba8(self.width, self.height, tm)

    @staticmethod
    def to_rgba8(fb: np.ndarray) -> np.ndarray:
        """Texture::setPixel's 8-bit clamp (Texture.cpp:222-241), top row first."""
        rgb = np.clip(fb, 0.0, 1.0) * 255.0
        rgba = np.concatenate([rgb, np.full(fb.shape[:2] + (1,), 255.0, np.float32)], axis=-1)
        return rgba.astype(np.uint8)[::-1]
