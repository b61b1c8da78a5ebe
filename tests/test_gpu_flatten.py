"""Device flatten and device fur generation (flatten.hip).

The per-object state of CPU::Scene::flattenNode (Triangle / Cylinder ctors,
CPU_Scene.cpp:73-197) and the seeded hairball (Mesh::addFurToFaces recurrence,
Mesh.cpp:111-142, with the fiber -> cone rule of CPU_Scene.cpp:121-144) run on
the GPU from the same source as the host (objects.h).  The bar is identity with
the host path: the same cones bit for bit, the same tree and records, the same
frames.
"""
import numpy as np
import pytest

import oracle_ffi
from _util import assert_parity
from ba_pathtracing_fur_amd import native as N
from ba_pathtracing_fur_amd import scenes as S
from ba_pathtracing_fur_amd.pathtracer import HipContext

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,verts", [(1, 2), (777, 10), (20_000, 10), (300, 64)])
def test_device_hairball_equals_host(hip_ctx, n, verts):
    base, apex, nc = hip_ctx.hairball_device(n, (0.1, 0.9, -0.2), 0.8, 0.005, verts=verts, seed=1234)
    got_b = base.to_array((nc, 4), np.float32)
    got_a = apex.to_array((nc, 4), np.float32)
    pos, rad = S.hairball(n, (0.1, 0.9, -0.2), 0.8, 0.005, verts=verts, seed=1234)
    sd = S.SceneData()
    sd.add_fibers(pos, rad, 0)
    assert np.array_equal(got_b.view(np.uint32), sd.cone_base_r0.view(np.uint32))
    assert np.array_equal(got_a.view(np.uint32), sd.cone_apex_r1.view(np.uint32))


def _frame(ctx, w, h, spp, depth):
    ctx.build_accel()
    return ctx.render(w, h, spp, depth)


def test_set_scene_device_matches_host_arrays():
    sd = S.config5(48, 32, n_strands=2000, torus_grid=30, glass_subdiv=2)
    a = HipContext(0)
    a.set_scene(sd)
    fa = _frame(a, 48, 32, 2, 5)
    b = HipContext(0)
    b.set_scene_device(sd)
    fb = _frame(b, 48, 32, 2, 5)
    assert np.array_equal(fa.view(np.uint32), fb.view(np.uint32))
    ta, tb = a.read_bvh(), b.read_bvh()
    for k in ("boxes", "first", "count", "ids"):
        assert np.array_equal(ta[k], tb[k]), k
    a.close()
    b.close()


def test_set_scene_device_refuses_device_tables():
    """khp_set_scene_device reads the tables (materials, cone_models, ...) on the
    host: a device pointer there is refused with KHP_EINVAL, not dereferenced."""
    import ctypes
    from ba_pathtracing_fur_amd.pathtracer import DeviceBuffer
    sd = S.config1(16, 16)
    c = HipContext(0)
    d = sd.desc()
    mats = DeviceBuffer(c, ctypes.sizeof(N.Material) * max(1, d.n_materials))
    d.materials = ctypes.cast(mats.ptr, ctypes.POINTER(N.Material))
    st = c.lib.khp_set_scene_device(c.ptr, ctypes.byref(d))
    assert st == N.KHP_EINVAL and b"materials" in c.lib.khp_last_error()
    d = sd.desc()
    models = DeviceBuffer(c, 64)
    d.n_cone_models, d.cone_models = 1, ctypes.cast(models.ptr, ctypes.POINTER(ctypes.c_float))
    st = c.lib.khp_set_scene_device(c.ptr, ctypes.byref(d))
    assert st == N.KHP_EINVAL and b"cone_models" in c.lib.khp_last_error()
    mats.free()
    models.free()
    c.close()


def test_config3_device_equals_host_config3():
    w, h = 64, 36
    c = HipContext(0)
    S.config3_device(c, w, h, n_strands=20_000)
    got = _frame(c, w, h, 2, 5)
    st = c.stats()
    host = S.config3(w, h, n_strands=20_000)
    hb = N.host_build(host)
    t = c.read_bvh()
    for k in ("boxes", "first", "count", "ids"):
        assert np.array_equal(t[k], hb[k]), k
    want = oracle_ffi.Oracle(host).render(w, h, 2, 5, threads=16)
    assert_parity(got, want, exact=True)
    assert st["n_objects"] == host.n_objects
    c.close()


def test_config3_device_full_size():
    """The metric-row scene generated, flattened and built in HBM; its tree equals
    the host build of the host-generated scene."""
    c = HipContext(0)
    S.config3_device(c, 64, 36, n_strands=1_000_000)
    c.build_accel()
    st = c.stats()
    t = c.read_bvh()
    hb = N.host_build(S.config3(64, 36, n_strands=1_000_000))
    for k in ("boxes", "first", "count", "ids"):
        assert np.array_equal(t[k], hb[k]), k
    print(f"config3 1M on device: flatten {st['flatten_ms']:.1f} ms ({st['flatten_kernel_ms']:.2f} ms kernels), "
          f"bvh {st['bvh_ms']:.1f} ms ({st['bvh_kernel_ms']:.1f} ms kernels), layout {st['layout_ms']:.1f} ms "
          f"({st['layout_kernel_ms']:.2f} ms kernels)")
    c.close()


def test_device_flatten_rejects_bad_material():
    sd = S.config1(16, 16)
    sd.tri_mat[5] = 99
    c = HipContext(0)
    with pytest.raises(N.KhpError) as e:
        c.set_scene(sd)
    assert e.value.status == N.KHP_EINVAL
    with pytest.raises(N.KhpError) as e:
        c.build_accel()
    assert e.value.status == N.KHP_ENOTREADY
    c.close()
    h = HipContext(0, host_build=True)
    with pytest.raises(N.KhpError) as e:
        h.set_scene_device(S.config1(16, 16))
    assert e.value.status == N.KHP_EUNSUPPORTED
    h.close()


# ---- fibers as triangle tubes (fiberToTriangles, CPU_Scene.cpp:232-345) ----------

def test_device_hairball_tris_equals_host(hip_ctx):
    n, verts, res = 120, 10, 5
    nt = n * (verts - 1) * 2 * res * res
    from ba_pathtracing_fur_amd.pathtracer import DeviceBuffer
    bufs = [DeviceBuffer(hip_ctx, 36 * nt) for _ in range(3)]
    c = np.float32([0.0, 0.5, 0.0])
    N.check(hip_ctx.lib, hip_ctx.lib.khp_gen_hairball_tris_device(hip_ctx.ptr, n, verts, N.fptr(c), 0.25, 0.004,
                                                                  S.SEED, res, *[b.ptr for b in bufs]),
            "khp_gen_hairball_tris_device")
    got = [b.to_array((nt, 3, 3), np.float32) for b in bufs]
    pos, rad = S.hairball(n, (0.0, 0.5, 0.0), 0.25)
    sd = S.SceneData()
    sd.add_fibers(pos, rad, 0, as_triangles=True, resolution=res)
    for g, w in zip(got, (sd.tri_v, sd.tri_n, sd.frames())):
        assert np.array_equal(g.view(np.uint32), w.view(np.uint32))


def _triangle_fur(w, h, n_strands, bsdf="MarschnerHairBSDF"):
    sd = S.config2(w, h, n_strands=0, bsdf=bsdf)
    pos, rad = S.hairball(n_strands, (0.0, 0.5, 0.0), 0.25)
    sd.add_fibers(pos, rad, len(sd.materials) - 1, as_triangles=True)
    return sd


@pytest.mark.parametrize("bsdf", ["MarschnerHairBSDF", "DEonHairBSDF"])
def test_triangle_fur_frame_parity(hip_ctx, bsdf):
    """Hair BSDFs on triangles read the fiber frame (Object::getU/V/W) on both sides."""
    sd = _triangle_fur(48, 32, 300, bsdf)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    got = hip_ctx.render(48, 32, 4, 5)
    want = oracle_ffi.Oracle(sd).render(48, 32, 4, 5, threads=16)
    assert_parity(got, want, exact=True)


def test_triangle_fur_device_scene_path(hip_ctx):
    sd = _triangle_fur(32, 24, 100)
    c = HipContext(0)
    c.set_scene_device(sd)
    c.build_accel()
    got = c.render(32, 24, 2, 4)
    c.close()
    want = oracle_ffi.Oracle(sd).render(32, 24, 2, 4, threads=16)
    assert_parity(got, want, exact=True)
