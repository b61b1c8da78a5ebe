"""ABI 6 boundary features on the CPU: the Cylinder node transform
(Cylinder.cpp:5-29), textures (Texture::getColor, Texture.cpp:243-287;
Material::getFromParam, Material.cpp:15-23), texcoords (calcTcoord,
Cylinder.cpp:239-260, Triangle.cpp:250-254) and environment maps
(Environment::getColor, Environment.cpp:91-133).

The oracle (test infrastructure) is checked against analytic answers and
independent numpy restatements; the product's host flatten (khp_host_build,
the same objects.h the device flatten runs) is checked against the oracle's
constructor state bit for bit.  Parity of the rendered frames on the GPU is in
test_gpu_parity.py.
"""
import numpy as np
import pytest

import oracle_ffi
from ba_pathtracing_fur_amd import native as N
from ba_pathtracing_fur_amd import scenes as S

f32 = np.float32


def _cone_scene(models, model_of, n=40):
    sd = S.SceneData(name="cones")
    sd.add_material(S.material())
    pos, rad = S.hairball(n, (0.1, -0.2, 0.3), 0.4)
    fur = sd.add_material(S.fiber_material())
    base = np.empty((n * 9, 4), f32)
    apex = np.empty((n * 9, 4), f32)
    lib = N.load_library()
    N.check(lib, lib.khp_fibers_to_cones(n, 10, N.fptr(pos), N.fptr(rad), N.fptr(base), N.fptr(apex)), "cones")
    ids = [sd.add_cone_model(M) for M in models]
    for k, m in enumerate(model_of):
        sl = slice(k * 9 * n // len(model_of), (k + 1) * 9 * n // len(model_of))
        sd.add_cones(base[sl], apex[sl], fur, model=ids[m])
    sd.cam = S.camera((0, 0, 3), (0, 0, -1), (0, 1, 0), 16, 16)
    return sd, base, apex


def test_glm_inverse_transpose_frame_matches_float64():
    """u, v, w = normalize(mat3(inverse(M)^T) * frame_pre), base = M base,
    slope and height from the PRE-transform points (KIRK's quirk), min/max_d
    along the transformed axis."""
    M = S.node_transform((0.3, -1.2, 2.0), (0.2, 1.0, -0.4), 1.1, (1.7, 0.6, 1.2))
    sd, base, apex = _cone_scene([M], [0])
    rec = oracle_ffi.Oracle(sd).cone_records()
    Mi = np.linalg.inv(M.astype(np.float64)).T[:3, :3]
    for i in range(0, len(base), 7):
        b, a = base[i, :3].astype(np.float64), apex[i, :3].astype(np.float64)
        h = np.linalg.norm(a - b)
        v0 = (a - b) / h
        tmp = np.array([0, 1, 0.0]) if 1 - abs(v0[1]) >= 1e-4 else np.array([0, 0, 1.0])
        u0 = np.cross(v0, tmp)
        u0 /= np.linalg.norm(u0)
        w0 = np.cross(u0, v0)
        w0 /= np.linalg.norm(w0)
        frame = [Mi @ x for x in (u0, v0, w0)]
        frame = [x / np.linalg.norm(x) for x in frame]
        bw = (M.astype(np.float64) @ np.r_[b, 1])[:3]
        aw = (M.astype(np.float64) @ np.r_[a, 1])[:3]
        r = rec[i]
        np.testing.assert_allclose(r[0:3], bw, rtol=0, atol=2e-6)
        for k, col in enumerate((4, 8, 12)):
            np.testing.assert_allclose(r[col:col + 3], frame[k], rtol=0, atol=3e-6)
        e = (apex[i, :3] - base[i, :3]).astype(f32)
        assert r[17] == np.sqrt(f32(f32(e[0] * e[0] + e[1] * e[1]) + e[2] * e[2]))   # pre-transform height
        np.testing.assert_allclose(r[7], (base[i, 3] - apex[i, 3]) / h, rtol=2e-6)
        d0, d1 = sorted((frame[1] @ bw, frame[1] @ aw))
        np.testing.assert_allclose([r[11], r[15]], [d0, d1], rtol=0, atol=3e-6)


def test_translation_model_keeps_the_frame():
    """A pure translation has M_ti = I: frames and radii are those of the
    world-space ctor, base/apex are shifted by exactly t."""
    t = (0.25, -0.5, 1.5)
    sd, base, apex = _cone_scene([S.node_transform(t)], [0])
    got = oracle_ffi.Oracle(sd).cone_records()
    plain = S.SceneData(name="plain", materials=list(sd.materials), cam=sd.cam)
    plain.add_cones(base, apex, 1)
    ref = oracle_ffi.Oracle(plain).cone_records()
    for col in (4, 5, 6, 8, 9, 10, 12, 13, 14, 3, 7, 17):
        assert np.array_equal(got[:, col], ref[:, col]), col
    assert np.array_equal(got[:, 0:3], (base[:, :3] + f32(t)).astype(f32))


def test_host_build_runs_the_transformed_ctor_like_the_oracle():
    """khp_host_build (the product's objects.h ctor, as the device flatten runs
    it) gives the oracle's cone state bit for bit, per model, and the same BVH."""
    Ms = [S.node_transform((0.1, 0.2, 0.3), (1, 1, 0), 0.4, (1.2, 0.9, 1.0)),
          S.node_transform((-1, 0, 0), (0, 0, 1), 2.5, (0.5, 0.5, 0.5)), np.eye(4, dtype=f32)]
    sd, _, _ = _cone_scene(Ms, [0, 1, 2, 0], n=60)
    hb = N.host_build(sd)
    o = oracle_ffi.Oracle(sd)
    rec = o.cone_records()
    nt = len(sd.tri_v)
    got = hb["records"][nt:]
    assert np.array_equal(got.view(np.uint32), rec[:, :16].view(np.uint32))
    boxes, first, count, ids, depth = o.bvh()
    assert np.array_equal(hb["boxes"].view(np.uint32), boxes.view(np.uint32))
    assert np.array_equal(hb["ids"], ids)


def test_bad_model_index_is_rejected():
    sd, _, _ = _cone_scene([np.eye(4, dtype=f32)], [0])
    sd.cone_model[3] = 7
    with pytest.raises(N.KhpError) as e:
        N.host_build(sd)
    assert e.value.status == N.KHP_EINVAL
    with pytest.raises(ValueError):
        oracle_ffi.Oracle(sd)


# ---- textures ----------------------------------------------------------------------------
def _np_tex_get(tex, wrap, x, y):
    """Texture::getColor restated in numpy float32 (Texture.cpp:243-287)."""
    h, w, ch = tex.shape
    if np.isnan(x) or np.isnan(y):
        return np.float32([1, 0, 0, 1])

    def wr(v):
        v = f32(v)
        if v > 1.0 or v < 0.0:
            fr = f32(v - np.floor(v))
            return f32(np.power(np.float64(fr), np.float64(wrap)))
        return v
    ux, uy = wr(x), wr(y)
    sx = int(np.clip(int(f32(ux * f32(w - 1))), 0, w - 1))
    sy = int(np.clip(int(f32(uy * f32(h - 1))), 0, h - 1))
    p = tex[sy, sx].astype(f32) / f32(255)
    if ch == 4:
        return p
    if ch == 3:
        return np.r_[p, f32(1)]
    if ch == 2:
        return np.r_[p[0], p[0], p[0], p[1]]
    return np.r_[p[0], p[0], p[0], p[0]]


@pytest.mark.parametrize("ch", [1, 2, 3, 4])
@pytest.mark.parametrize("wrap", [N.TEX_WRAP_CLAMP, N.TEX_WRAP_TILE, 2])
def test_texture_lookup_known_answers(ch, wrap):
    sd = S.config1(8, 8)
    tex = S.checker(13, 7, ch, 5, seed=ch)
    k = sd.add_texture(tex, wrap)
    o = oracle_ffi.Oracle(sd)
    rng = np.random.default_rng(ch * 10 + wrap)
    pts = list(rng.uniform(-2.5, 3.5, (200, 2)).astype(f32)) + [(0, 0), (1, 1), (1, 0), (0.5, 1.0), (-1.0, 2.0),
                                                                  (np.nan, 0.3), (0.2, np.nan), (1e-8, -1e-8)]
    for x, y in pts:
        got = o.tex_color(k, float(f32(x)), float(f32(y)))
        want = _np_tex_get(tex, wrap, f32(x), f32(y))
        assert np.array_equal(got.view(np.uint32), np.asarray(want, f32).view(np.uint32)), (x, y)


def _np_cube(faces, d):
    d = np.asarray(d, f32)
    d = (d * f32(1.0 / np.sqrt(f32((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])))).astype(f32)
    a = np.abs(d)
    mx = max(max(a[0], a[1]), a[2])
    sg = np.sign(d).astype(f32)
    one, two = f32(1), f32(2)
    if mx == a[0]:
        side = int(f32(1.5) - f32(1.5) * sg[0])
        uv = ((d[2] / d[0] + one) / two, (d[1] / a[0] + one) / two)
    elif mx == a[1]:
        side = int(f32(2.5) - f32(1.5) * sg[1])
        uv = ((d[0] / a[1] + one) / two, (d[2] / d[1] + one) / two)
    else:
        side = int(f32(3.5) + f32(1.5) * sg[2])
        uv = (-(d[0] / d[2] + one) / two, (d[1] / a[2] + one) / two)
    return side, uv


def test_cube_map_faces_and_texels():
    """Cube map: face of the dominant axis (+x 0, +y 1, +z 5 (!), -x 3, -y 4,
    -z 2: KIRK's z faces use the opposite sign), texel from KIRK's uv."""
    sd = S.config1(8, 8)
    faces = [S.checker(6, 6, 3, 3, seed=40 + k) for k in range(6)]
    sd.set_environment_map(N.ENV_CUBE_MAP, [sd.add_texture(f) for f in faces])
    o = oracle_ffi.Oracle(sd)
    rng = np.random.default_rng(3)
    dirs = list(rng.normal(size=(300, 3)).astype(f32)) + [np.float32(v) for v in
                                                          ([1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1],
                                                           [0, 0, -1], [1, 1, 0], [0.3, -0.3, 0.3])]
    got = o.env_color(np.stack(dirs))
    seen = set()
    for d, g in zip(dirs, got):
        side, (u, v) = _np_cube(faces, d)
        seen.add(side)
        want = _np_tex_get(faces[side], 1, f32(u), f32(v))[:3]
        assert np.array_equal(g.view(np.uint32), want.view(np.uint32)), d
    assert seen == {0, 1, 2, 3, 4, 5}
    # the z quirk itself: +z reads the -z texture slot
    assert _np_cube(faces, [0, 0, 1])[0] == 5 and _np_cube(faces, [0, 0, -1])[0] == 2


def test_sphere_map_texels():
    sd = S.config1(8, 8)
    tex = S.checker(16, 16, 3, 4, seed=9)
    sd.set_environment_map(N.ENV_SPHERE_MAP, [sd.add_texture(tex)])
    o = oracle_ffi.Oracle(sd)
    dirs = np.random.default_rng(5).normal(size=(200, 3)).astype(f32)
    got = o.env_color(dirs)
    for d, g in zip(dirs, got):
        d = (d * f32(1.0 / np.sqrt(f32((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2])))).astype(f32)
        m = f32(2.0 * np.sqrt(np.float64(f32(d[0] * d[0] + d[1] * d[1])) + (np.float64(d[2]) + 1.0) ** 2))
        u, v = f32(np.float64(d[0] / m) + 0.5), f32(np.float64(d[1] / m) + 0.5)
        assert np.array_equal(g.view(np.uint32), _np_tex_get(tex, 1, u, v)[:3].view(np.uint32))


def test_emission_texture_fills_the_frame():
    """End-to-end KAT: a quad with an emission texture in front of the camera,
    no lights, no ambient, depth 1: every pixel away from the texel block
    edges is exactly its texel's colour (SimpleShader emits
    fetchParameterColor<EMISSION>(hit.m_texcoord), SimpleShader.h:44, 74-80)."""
    W = H = 32
    sd = S.SceneData(name="emit_kat")
    tex = S.checker(4, 4, 3, 4, seed=11)
    mat = sd.add_material(S.material("EmissionBSDF"))
    sd.set_material_texture(mat, "emission", sd.add_texture(tex))
    v, n = S.quad((-2, -2, 0), (2, -2, 0), (2, 2, 0), (-2, 2, 0), (0, 0, 1))
    sd.add_triangles(v, n, mat, uv=np.float32([[[0, 0], [1, 0], [1, 1]], [[0, 0], [1, 1], [0, 1]]]))
    sd.env_ambient = (0.0, 0.0, 0.0)
    sd.cam = S.camera((0, 0, 1.0), (0, 0, -1), (0, 1, 0), W, H)
    img = oracle_ffi.Oracle(sd).render(W, H, 1, 1, threads=4)
    # the camera sees x, y in [-s, s] at z = 0 (s = tan(fov/2) * aspect); texcoord = (x + 2) / 4
    cam = sd.cam
    for y in range(2, H - 2, 3):
        for x in range(2, W - 2, 3):
            px = np.float64(cam.bottom_left[0]) + (x + 0.5) * cam.pixel_size * np.float64(cam.axis_x[0])
            py = np.float64(cam.bottom_left[1]) + (y + 0.5) * cam.pixel_size * np.float64(cam.axis_y[1])
            u, v = (px + 2) / 4 * 1.0, (py + 2) / 4 * 1.0  # ray from (0,0,1) through the film at z = 0 + f
            tx, ty = int(u * 3), int(v * 3)
            if abs(u * 3 - round(u * 3)) < 0.08 or abs(v * 3 - round(v * 3)) < 0.08:
                continue
            assert np.array_equal(img[y, x], tex[ty, tx].astype(f32) / f32(255)), (x, y)


def test_fixture_roundtrip_keeps_abi6_fields(tmp_path):
    sd = S.textured(16, 12, n_strands=30, env="sphere")
    sd2 = S.transformed_hairball(16, 12, n_strands=30)
    for s in (sd, sd2):
        f = tmp_path / "s.npz"
        np.savez(f, **s.to_arrays())
        back = S.SceneData.from_arrays(np.load(f))
        a, b = s.desc(), back.desc()
        assert (a.n_textures, a.n_cone_models, a.env_map.type) == (b.n_textures, b.n_cone_models, b.env_map.type)
        assert np.array_equal(oracle_ffi.Oracle(s).render(16, 12, 1, 3, threads=2).view(np.uint32),
                              oracle_ffi.Oracle(back).render(16, 12, 1, 3, threads=2).view(np.uint32))
