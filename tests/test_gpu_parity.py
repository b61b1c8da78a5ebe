"""Parity of the HIP core (libkirk_hip.so via the C-ABI) with the oracle, on an MI355X.

Bar (BASELINE.json north_star): per-pixel L2 <= 1e-3 on identical seeds; the
core and the oracle share every float operation, so frames are also required
to be identical bit for bit (tests/_util.assert_parity(exact=True)).
"""
import os

import numpy as np
import pytest

import oracle_ffi
from _util import assert_parity
from ba_pathtracing_fur_amd import native as N
from ba_pathtracing_fur_amd import scenes as S
from ba_pathtracing_fur_amd import sharding
from ba_pathtracing_fur_amd.pathtracer import BVH, HipContext, PathTracer

pytestmark = pytest.mark.gpu

CASES = [
    ("config1", dict(), 64, 48, 4, 5),
    ("config2", dict(n_strands=2000), 64, 48, 4, 5),
    ("config2", dict(n_strands=2000, bsdf="DEonHairBSDF"), 64, 48, 4, 5),
    ("config3", dict(n_strands=20000), 96, 54, 4, 5),
    ("config5", dict(n_strands=5000, torus_grid=40, glass_subdiv=3), 96, 54, 4, 6),
    ("zoo", dict(n_strands=400), 96, 72, 4, 8),
    ("transformed", dict(n_strands=1500), 64, 48, 4, 5),
    ("transformed", dict(n_strands=1200, bsdf="DEonHairBSDF"), 48, 40, 3, 5),
    ("textured", dict(n_strands=600, env="cube"), 80, 60, 4, 6),
    ("textured", dict(n_strands=600, env="sphere"), 64, 48, 3, 6),
]


def _render_both(hip_ctx, sd, w, h, spp, depth, **kw):
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    got = hip_ctx.render(w, h, spp, depth, **kw)
    want = oracle_ffi.Oracle(sd).render(w, h, spp, depth, threads=16, **kw)
    return got, want


@pytest.mark.parametrize("name,kw,w,h,spp,depth", CASES,
                         ids=[f"{c[0]}-{c[1].get('bsdf', '')}{c[1].get('env', '')}{c[1].get('n_strands', '')}"
                              for c in CASES])
def test_frame_parity(hip_ctx, name, kw, w, h, spp, depth):
    sd = S.build_config(name, width=w, height=h, **kw)
    got, want = _render_both(hip_ctx, sd, w, h, spp, depth)
    r = assert_parity(got, want, exact=True)
    assert r["n_nonfinite"] < 0.05 * w * h


@pytest.mark.parametrize("name,kw", [("transformed", dict(n_strands=1500)), ("textured", dict(n_strands=600))])
def test_device_flatten_of_abi6_scenes(name, kw):
    """khp_set_scene_device (geometry, texcoords and cone model indices in HBM,
    flattened by flatten.hip) gives the frames of khp_set_scene and the oracle."""
    sd = S.build_config(name, width=64, height=40, **kw)
    want = oracle_ffi.Oracle(sd).render(64, 40, 3, 5, threads=16)
    ctx = HipContext(0)
    try:
        ctx.set_scene_device(sd)
        ctx.build_accel()
        assert_parity(ctx.render(64, 40, 3, 5), want, exact=True)
    finally:
        ctx.close()
    ctx = HipContext(0, host_build=True)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        assert_parity(ctx.render(64, 40, 3, 5), want, exact=True)
    finally:
        ctx.close()


def test_bvh_is_the_oracle_bvh(hip_ctx):
    sd = S.config2(32, 32, n_strands=3000)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    st = hip_ctx.stats()
    boxes, first, count, ids, depth = oracle_ffi.Oracle(sd).bvh()
    assert st["n_nodes"] == len(boxes) and st["bvh_depth"] == depth and st["n_objects"] == sd.n_objects


def test_progressive_samples(hip_ctx):
    sd = S.config2(48, 32, n_strands=1000)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    hip_ctx.render(48, 32, 3, 5, readback=False)
    got = hip_ctx.render(48, 32, 2, 5, first_sample=3)
    want = oracle_ffi.Oracle(sd).render(48, 32, 5, 5, threads=16)
    assert_parity(got, want, exact=True)


def test_pathtracer_api(hip_ctx):
    sd = S.config1(40, 30)
    pt = PathTracer(sd, depth=4, width=40, height=30)
    pt.set_sample_count(5)
    pt.render(2)
    assert pt.get_current_sample_count() == 2
    img = pt.render_to_texture()
    assert pt.get_current_sample_count() == 5
    want = oracle_ffi.Oracle(sd).render(40, 30, 5, 4, threads=16)
    assert_parity(img, want, exact=True)
    rgba = PathTracer.to_rgba8(img)
    assert rgba.shape == (30, 40, 4) and rgba.dtype == np.uint8
    pt.ctx.close()


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_tile_shards_match_oracle(hip_ctx, nranks):
    sd = S.config2(80, 56, n_strands=1500)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    o = oracle_ffi.Oracle(sd)
    full = o.render(80, 56, 2, 5, threads=16)
    for r in range(nranks):
        got = hip_ctx.render(80, 56, 2, 5, tile_size=16, tile_rank=r, tile_nranks=nranks)
        m = sharding.owned_mask(80, 56, r, nranks, 16)
        assert_parity(got[m][None], full[m][None], exact=True)


EDGE = [("config1", 1, 1, 1, 1), ("config1", 1, 1, 33, 5), ("config2", 37, 23, 3, 1), ("config2", 37, 23, 2, 5),
        ("zoo", 32, 24, 2, 20)]


@pytest.mark.parametrize("path_kernel", [1, 2])
@pytest.mark.parametrize("name,w,h,spp,depth", EDGE, ids=[f"{c[0]}-{c[1]}x{c[2]}-{c[3]}spp-d{c[4]}" for c in EDGE])
def test_edge_sizes(hip_ctx, name, w, h, spp, depth, path_kernel):
    """A 1x1 frame (one pixel: a single, partly filled wave; 33 spp: more paths
    than a wave), a ragged 37x23 frame, and depth 1 (camera rays and their
    shadow rays only) -- through the wavefront (path_kernel 1) and the path
    kernel (2), as one synchronous render and as fused 1-spp asynchronous
    passes; and depth 20 on the all-BSDF scene (glass and mirrors keep paths
    alive past the usual 5-8 bounces).  Bit-exact against the oracle."""
    sd = S.build_config(name, width=w, height=h,
                        **({} if name == "config1" else dict(n_strands=400 if name == "zoo" else 800)))
    want = oracle_ffi.Oracle(sd).render(w, h, spp, depth, threads=16)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    old = hip_ctx.set_params(path_kernel=path_kernel)
    try:
        assert_parity(hip_ctx.render(w, h, spp, depth), want, exact=True)
        for k in range(spp):
            hip_ctx.render(w, h, 1, depth, first_sample=k, async_=True)
        hip_ctx.sync()
        assert_parity(hip_ctx.read_framebuffer(w, h), want, exact=True)
    finally:
        hip_ctx.set_params(**old)


def _tiny_scene(centers, size=0.3, planar=False):
    sd = S.SceneData(name="tiny")
    m = sd.add_material(S.material(diffuse=(0.7, 0.6, 0.5)))
    c = np.asarray(centers, np.float32)
    off = np.array([[0, 0, 0], [size, 0, 0], [0, size, 0 if planar else size]], np.float32)
    v = c[:, None, :] + off[None]
    sd.add_triangles(v, np.broadcast_to(np.float32([0, 0, 1]), v.shape).copy(), m)
    sd.lights.append(S.point_light((0.6, 0.6, 1.5), (3.0, 3.0, 3.0), radius=0.05, att_const=1.0, att_quad=0.0))
    sd.env_color = (0.2, 0.3, 0.4)
    sd.env_ambient = (0.05, 0.05, 0.05)
    sd.cam = S.camera((0, 0, 3), (0, 0, -1), (0, 1, 0), 24, 16)
    return sd


TINY = {
    "one_object": lambda: _tiny_scene([[-0.1, -0.1, 0.0]]),
    "two_objects": lambda: _tiny_scene([[-0.4, -0.2, 0.0], [0.1, 0.0, 0.2]]),
    "three_objects": lambda: _tiny_scene(np.random.default_rng(3).uniform(-0.5, 0.5, (3, 3))),
    # every centroid on one plane: the root is ONE leaf of 3000 candidates (the escaped leaf count)
    "root_leaf_3000": lambda: _tiny_scene(np.c_[np.random.default_rng(7).uniform(-1, 1, (3000, 2)), np.zeros(3000)],
                                          size=0.02, planar=True),
}


@pytest.mark.parametrize("path_kernel,lds_nodes", [(1, 0), (2, 0), (1, 7)])
@pytest.mark.parametrize("name", list(TINY))
def test_tiny_and_degenerate_trees(hip_ctx, name, path_kernel, lds_nodes):
    """Trees whose root is a leaf (one object; 3000 coplanar centroids, whose
    leaf count needs the escape word), two- and three-object trees (no
    two-level record below the root; fewer top records than LDS slots),
    through the wavefront (also with the top records in LDS) and the path
    kernel, synchronous and fused: the oracle's frame bit for bit."""
    sd = TINY[name]()
    want = oracle_ffi.Oracle(sd).render(24, 16, 3, 4, threads=16)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    old = hip_ctx.set_params(path_kernel=path_kernel, lds_nodes=lds_nodes)
    try:
        assert_parity(hip_ctx.render(24, 16, 3, 4), want, exact=True)
        for k in range(3):
            hip_ctx.render(24, 16, 1, 4, first_sample=k, async_=True)
        hip_ctx.sync()
        assert_parity(hip_ctx.read_framebuffer(24, 16), want, exact=True)
    finally:
        hip_ctx.set_params(**old)


def _quirk_scenes():
    import test_oracle_kat as K
    pl = lambda att=(1.0, 0.0, 0.0): S.point_light((0.5, 0.0, -0.5), (4.0, 3.0, 2.0), radius=0.01, att_const=att[0],
                                                    att_lin=att[1], att_quad=att[2])
    return {
        "two_identical_lights": K._plane_scene([pl(), pl()]),
        "occluder_0.6_above": K._plane_scene([pl()], occluder=(-2.4, 0.24, 0.0)),
        "occluder_1.5_above": K._plane_scene([pl()], occluder=(-1.5, 0.15, 0.0)),
        "ambient_only": K._plane_scene([], diffuse=(0.5, 0.25, 1.0), ambient=(0.3, 0.6, 0.9)),
        "quadratic_attenuation_only": K._plane_scene([pl((0.0, 0.0, 0.5))]),
        "dark_box_depth9": K._dark_box(),
        "mirror_under_environment": K._mirror_scene(),
        "inside_point_light_behind": K._inside_point_light(-0.1),
        "inside_point_light_front": K._inside_point_light(0.1),
    }


@pytest.mark.parametrize("path_kernel", [1, 2])
@pytest.mark.parametrize("name", ["two_identical_lights", "occluder_0.6_above", "occluder_1.5_above", "ambient_only",
                                  "quadratic_attenuation_only", "dark_box_depth9", "mirror_under_environment",
                                  "inside_point_light_behind", "inside_point_light_front"])
def test_quirk_scenes(hip_ctx, name, path_kernel):
    """The scenes that pin KIRK's integrator quirks in the oracle's known-answer
    tests (tests/test_oracle_kat.py: one-light NEE without a count factor, the
    ~1-unit shadow ray, the per-hit ambient term, the attenuation rule, the
    throughput cut without Russian roulette, misses adding the environment at
    any depth, the point light's rejection of rays leaving its centre) render
    the oracle's frames bit for bit through both kernels."""
    sd = _quirk_scenes()[name]
    depth = 9 if name.startswith("dark_box") else 3
    want = oracle_ffi.Oracle(sd).render(24, 16, 8, depth, threads=16)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    old = hip_ctx.set_params(path_kernel=path_kernel)
    try:
        assert_parity(hip_ctx.render(24, 16, 8, depth), want, exact=True)
    finally:
        hip_ctx.set_params(**old)


@pytest.mark.parametrize("trace_kernels", [0, 1, 2])
@pytest.mark.parametrize("n_extra", [0, 64])
def test_equal_t_within_a_leaf(hip_ctx, n_extra, trace_kernels):
    """Appendix A.9: of two coincident triangles in one leaf the later candidate
    is the closest hit (t <= best inside a leaf) -- through the batch query
    kernel and the production traversal kernels (trace_kernels 1: the 64-B
    loop, 2: with the two-level records), as in the oracle's known-answer test."""
    import test_oracle_kat as K
    sd = K._coincident_tris(n_extra)
    want_t, want_obj, want_uv, _, _ = oracle_ffi.Oracle(sd).trace_closest([[0.0, -0.3, 3.0]], [[0.0, 0.0, -1.0]])
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    old = hip_ctx.set_params(trace_kernels=trace_kernels, wide_from=0 if trace_kernels == 2 else 2)
    try:
        t, obj, uv = hip_ctx.trace_closest([[0.0, -0.3, 3.0]], [[0.0, 0.0, -1.0]])
    finally:
        hip_ctx.set_params(**old)
    assert obj[0] == want_obj[0] == 1 and t[0] == want_t[0] and np.array_equal(uv, want_uv)


def test_rank_without_tiles(hip_ctx):
    """A rank that owns no tile (37x23 in 16-px tiles: 6 tiles for 8 ranks)
    renders nothing, synchronously or not, without an error; the ranks that do
    own tiles match the oracle on them."""
    sd = S.config2(37, 23, n_strands=800)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    full = oracle_ffi.Oracle(sd).render(37, 23, 2, 5, threads=16)
    for r in range(8):
        m = sharding.owned_mask(37, 23, r, 8, 16)
        assert m.any() == (r < 6)
        got = hip_ctx.render(37, 23, 2, 5, tile_size=16, tile_rank=r, tile_nranks=8)
        if m.any():
            assert_parity(got[m][None], full[m][None], exact=True)
    # asynchronous passes with an 8-bit snapshot after each: an empty rank's
    # batch has no chunk, its snapshots must still be delivered
    bufs, tickets = [], []
    for r in (0, 6, 7):
        for k in range(2):
            hip_ctx.render(37, 23, 1, 5, first_sample=k, tile_size=16, tile_rank=r, tile_nranks=8, async_=True)
            bufs.append(np.zeros((23, 37, 4), np.uint8))
            tickets.append(hip_ctx.read_rgba8_async(bufs[-1]))
    hip_ctx.sync()
    for t, b in zip(tickets, bufs):
        assert hip_ctx.snapshot_wait(t)
        assert (b[..., 3] == 255).all()


def test_path_chunking(hip_ctx):
    """khp_ctx_params.chunk_paths forces pixel and sample chunking of the wavefront; frames must not change."""
    sd = S.config2(128, 96, n_strands=1500)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    ref = hip_ctx.render(128, 96, 3, 5)
    old = hip_ctx.set_params(chunk_paths=4096)
    try:
        got = hip_ctx.render(128, 96, 3, 5)
    finally:
        hip_ctx.set_params(**old)
    assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))
    assert_parity(got, oracle_ffi.Oracle(sd).render(128, 96, 3, 5, threads=16), exact=True)


@pytest.mark.parametrize("chunk", [0, 5000])
def test_chunked_and_instrumented_frames(hip_ctx, chunk):
    """Chunked wavefronts (chunk_paths 5000: pixel and sample chunks) and the
    instrumented kernels (one stream, per-bounce snapshots) leave the frame
    equal to the oracle's, bit for bit."""
    sd = S.config2(120, 72, n_strands=1500)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    spp = 5
    want = oracle_ffi.Oracle(sd).render(120, 72, spp, 5, threads=16)
    old = hip_ctx.set_params(chunk_paths=chunk)
    try:
        got = hip_ctx.render(120, 72, spp, 5)
        assert hip_ctx.stats()["subframes"] == 1
        assert_parity(got, want, exact=True)
        got = hip_ctx.render(120, 72, spp, 5, stats=True)
        st = hip_ctx.stats()
        assert sum(st["bounce_rays"]) == st["extend_rays"] > 0
        assert_parity(got, want, exact=True)
    finally:
        hip_ctx.set_params(**old)


def test_params_are_validated(hip_ctx):
    for bad in (dict(fuse_frames=0), dict(fuse_frames=33), dict(frames_in_flight=4), dict(chunk_paths=100),
                dict(trace_kernels=3), dict(shade_order=2), dict(serial_stages=2), dict(path_order=3)):
        with pytest.raises(N.KhpError) as e:
            hip_ctx.set_params(**bad)
        assert e.value.status == N.KHP_EINVAL
    assert hip_ctx.params()["fuse_frames"] == 32


@pytest.mark.parametrize("name,kw,w,h,spp,depth", [CASES[4], CASES[5], CASES[8]], ids=["config5", "zoo", "textured"])
def test_hit_sorting(hip_ctx, name, kw, w, h, spp, depth):
    """shade_order 1 (hits grouped by shading class before k_shade) changes only
    the order k_shade takes the paths in: synchronous, instrumented and fused
    asynchronous frames stay the oracle's, bit for bit."""
    sd = S.build_config(name, width=w, height=h, **kw)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    want = oracle_ffi.Oracle(sd).render(w, h, spp, depth, threads=16)
    old = hip_ctx.set_params(shade_order=1, chunk_paths=4096)
    try:
        assert_parity(hip_ctx.render(w, h, spp, depth), want, exact=True)
        assert_parity(hip_ctx.render(w, h, spp, depth, stats=True), want, exact=True)
        hip_ctx.set_params(chunk_paths=0)
        for k in range(spp):
            hip_ctx.render(w, h, 1, depth, first_sample=k, async_=True)
        hip_ctx.sync()
        assert_parity(hip_ctx.read_framebuffer(w, h), want, exact=True)
    finally:
        hip_ctx.set_params(**old)


def test_serial_stages(hip_ctx):
    """serial_stages 1 (shadow stage on the extend stream; bench.py's isolated
    timings) changes only the stream the kernels run on."""
    sd = S.config2(64, 48, n_strands=1500)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    want = oracle_ffi.Oracle(sd).render(64, 48, 4, 5, threads=16)
    old = hip_ctx.set_params(serial_stages=1)
    try:
        assert_parity(hip_ctx.render(64, 48, 4, 5), want, exact=True)
        for k in range(4):
            hip_ctx.render(64, 48, 1, 5, first_sample=k, async_=True)
        hip_ctx.sync()
        assert_parity(hip_ctx.read_framebuffer(64, 48), want, exact=True)
    finally:
        hip_ctx.set_params(**old)


@pytest.mark.parametrize("fif", ["1", "2", "3"])
def test_async_frames_in_flight(hip_ctx, fif):
    """KHP_RENDER_ASYNC: progressive passes enqueued back to back (up to
    frames_in_flight overlapping on the device) accumulate in call order;
    after khp_sync the framebuffer is the oracle's 5-spp frame, and the report
    covers every pass."""
    sd = S.config2(96, 64, n_strands=1500)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    want = oracle_ffi.Oracle(sd).render(96, 64, 5, 5, threads=16)
    # frames in flight without fusion (test_fused_frames covers fusion)
    old = hip_ctx.set_params(frames_in_flight=int(fif), fuse_frames=1)
    try:
        for first, n in ((0, 1), (1, 2), (3, 1), (4, 1)):
            hip_ctx.render(96, 64, n, 5, first_sample=first, async_=True)
        hip_ctx.sync()
        st = hip_ctx.stats()
        assert st["frames"] == 4 and st["extend_launches"] == 4 * 5
        assert_parity(hip_ctx.read_framebuffer(96, 64), want, exact=True)
        # a synchronous render after async ones completes them first
        hip_ctx.render(96, 64, 2, 5, async_=True)
        got = hip_ctx.render(96, 64, 3, 5, first_sample=2)
        assert_parity(got, want, exact=True)
        with pytest.raises(N.KhpError):
            hip_ctx.render(96, 64, 1, 5, async_=True, stats=True)
    finally:
        hip_ctx.set_params(**old)


def test_deterministic_across_runs(hip_ctx):
    sd = S.config3(64, 36, n_strands=5000)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    a = hip_ctx.render(64, 36, 2, 5)
    b = hip_ctx.render(64, 36, 2, 5)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("name,kw", [("config2", dict(n_strands=3000)), ("config5", dict(n_strands=2000,
                                                                                          torus_grid=30))])
def test_trace_queries(hip_ctx, name, kw):
    sd = S.build_config(name, width=32, height=32, **kw)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    o = oracle_ffi.Oracle(sd)
    rng = np.random.default_rng(11)
    n = 20000
    orig = rng.uniform(-1.5, 1.5, (n, 3)).astype(np.float32) + np.float32([0, 1, 0])
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tmax = rng.uniform(0.01, 2.0, n).astype(np.float32)
    bvh = BVH(hip_ctx)
    t, obj, uv = bvh.closest_intersection(orig, d)
    st = hip_ctx.stats()
    t0, obj0, uv0, nodes, prims = o.trace_closest(orig, d)
    assert np.array_equal(obj, obj0)
    assert np.array_equal(t.view(np.uint32), t0.view(np.uint32))
    assert np.array_equal(uv.view(np.uint32), uv0.view(np.uint32))
    assert (st["node_visits"], st["prim_tests"]) == (nodes, prims)      # same traversal order, same work
    assert np.array_equal(bvh.is_intersection(orig, d, tmax), o.trace_any(orig, d, tmax))


def test_full_size_scene_sampled_rows(hip_ctx):
    """The metric scene itself (1M strands, 1080p) at 1 spp: every 45th row against the oracle."""
    sd = S.config3(1920, 1080, n_strands=1_000_000)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    got = hip_ctx.render(1920, 1080, 1, 5)
    o = oracle_ffi.Oracle(sd)
    want = o.render(1920, 1080, 1, 5, threads=16, rows=(0, 1080, 45))
    rows = list(range(0, 1080, 45))
    assert_parity(got[rows], want[rows], exact=True)


def test_config1_full_frame(hip_ctx):
    """BASELINE config 1 at its stated size: Cornell box + Lambert icosphere, 256x256, 4 spp, every pixel."""
    sd = S.config1(256, 256)
    got, want = _render_both(hip_ctx, sd, 256, 256, 4, 5)
    assert_parity(got, want, exact=True)


def test_config2_full_size_sampled_rows(hip_ctx):
    """BASELINE config 2 at its stated size: 10k-strand hairball in the Cornell
    box, 1920x1080, 8 spp; every 24th row against the oracle."""
    sd = S.config2(1920, 1080, n_strands=10_000)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    got = hip_ctx.render(1920, 1080, 8, 5)
    rows = list(range(5, 1080, 24))
    want = oracle_ffi.Oracle(sd).render(1920, 1080, 8, 5, threads=16, rows=(5, 1080, 24))
    assert_parity(got[rows], want[rows], exact=True)


def test_config5_full_size_sampled_rows():
    """BASELINE config 5 at its stated size: 1M strands (9M cones, generated in
    HBM) + 500x500x2-triangle torus + subdiv-5 glass icosphere at 3840x2160;
    8 spp as 4 fused asynchronous 2-spp passes (the path is per-sample
    independent, so 32 spp is 16 such passes), every 54th row (40 rows) against
    the oracle's 8-spp frame on the host-generated scene."""
    ctx = HipContext(0)
    try:
        S.config5_device(ctx, 3840, 2160, n_strands=1_000_000)
        ctx.build_accel()
        assert ctx.stats()["n_objects"] == 500 * 500 * 2 + 20 * 4 ** 5 + 2 + 9_000_000
        for k in range(4):
            ctx.render(3840, 2160, 2, 5, first_sample=2 * k, async_=True)
        ctx.sync()
        got = ctx.read_framebuffer(3840, 2160)
    finally:
        ctx.close()
    host = S.config5(3840, 2160, n_strands=1_000_000)
    rows = list(range(11, 2160, 54))
    assert len(rows) == 40
    want = oracle_ffi.Oracle(host).render(3840, 2160, 8, 5, threads=16, rows=(11, 2160, 54))
    assert_parity(got[rows], want[rows], exact=True)


def test_errors_are_loud():
    ctx = HipContext(0)
    with pytest.raises(N.KhpError) as e:
        ctx.render(8, 8, 1, 1)
    assert e.value.status == N.KHP_ENOTREADY
    with pytest.raises(N.KhpError):
        ctx.read_framebuffer(8, 8)
    with pytest.raises(N.KhpError) as e:
        ctx.build_accel()
    assert e.value.status == N.KHP_ENOTREADY
    ctx.set_scene(S.config1(8, 8))
    ctx.build_accel()
    with pytest.raises(N.KhpError) as e:
        ctx.render(8, 8, 1, 1, tile_size=12)
    assert e.value.status == N.KHP_EINVAL
    with pytest.raises(N.KhpError) as e:
        ctx.render(8, 8, 1, 0)
    assert e.value.status == N.KHP_EINVAL
    with pytest.raises(N.KhpError) as e:
        ctx.render(8, 8, 1, 1, tile_rank=3, tile_nranks=2)
    assert e.value.status == N.KHP_EINVAL
    with pytest.raises(N.KhpError) as e:
        ctx.gather_framebuffer(8, 8, 1, 1, 64, 2, 0)
    assert e.value.status == N.KHP_ENOTREADY        # no communicator
    ctx.close()


def test_single_rank_communicator():
    from ba_pathtracing_fur_amd.pathtracer import comm_unique_id
    sd = S.config1(16, 16)
    ctx = HipContext(0)
    ctx.set_scene(sd)
    ctx.build_accel()
    ctx.comm_init(1, 0, comm_unique_id())
    a = ctx.render(16, 16, 1, 3)
    ctx.gather_framebuffer(16, 16, 1, 3, 64, 1, 0)
    assert np.array_equal(ctx.read_framebuffer(16, 16).view(np.uint32), a.view(np.uint32))
    ctx.close()


@pytest.mark.parametrize("order", ["0", "1", "2"])
@pytest.mark.parametrize("fuse", ["2", "4", "3"])
def test_fused_frames(fuse, order):
    """fuse_frames: asynchronous passes with equal parameters run as one
    batch (one launch per bounce for all of them) and accumulate in call order
    -- the framebuffer is the oracle's 8-spp frame; with a (1-rank) gather
    after every pass, as bench.py does at N > 1, the gathers keep their place.
    Both path numberings (path_order 0 frame-major, 1 pixel-major) and the
    heavy-first pixel order (2: each batch's pixel list permuted by the previous
    batch's camera-ray lengths), with the longest-first queues on (heavy_iters
    160, off by default since round 6) so both orderings are exercised."""
    from ba_pathtracing_fur_amd.pathtracer import comm_unique_id
    sd = S.config2(72, 48, n_strands=1500)
    want = oracle_ffi.Oracle(sd).render(72, 48, 8, 5, threads=16)
    ctx = HipContext(0)
    try:
        ctx.set_params(fuse_frames=int(fuse), path_order=int(order), heavy_iters=160)
        ctx.set_scene(sd)
        ctx.build_accel()
        for first in range(0, 8, 2):
            ctx.render(72, 48, 2, 5, first_sample=first, async_=True)
        ctx.sync()
        st = ctx.stats()
        assert st["frames"] == 4
        assert_parity(ctx.read_framebuffer(72, 48), want, exact=True)
        ctx.comm_init(1, 0, comm_unique_id())
        for first in range(0, 8, 2):
            ctx.render(72, 48, 2, 5, first_sample=first, tile_size=64, tile_rank=0, tile_nranks=1, async_=True)
            ctx.gather_framebuffer(72, 48, 2, 5, 64, 1, 0)
        ctx.sync()
        assert_parity(ctx.read_framebuffer(72, 48), want, exact=True)
        # the same frame re-rendered every step (bench.py): the last one stays
        for _ in range(5):
            ctx.render(72, 48, 8, 5, async_=True)
        ctx.sync()
        assert_parity(ctx.read_framebuffer(72, 48), want, exact=True)
    finally:
        ctx.close()


def test_fused_full_size_matches_passes():
    """The metric scene (1M strands, 1080p): 16 progressive 4-spp passes
    fused into one batch (133M paths: 1 chunk at the automatic cap, 2 at 2^26;
    frame-major and pixel-major path numbering, and the heavy-first pixel order
    with the longest-first queues on, whose later batches run a permuted pixel
    list) give the
    framebuffer of the same passes rendered one by one, bit for bit; sampled
    rows are the oracle's 64-spp frame."""
    ctx = HipContext(0)
    try:
        sd = S.config3_device(ctx, 1920, 1080, n_strands=1_000_000)
        ctx.build_accel()
        for k in range(16):
            ctx.render(1920, 1080, 4, 5, first_sample=4 * k, readback=False)
        want = ctx.read_framebuffer(1920, 1080)
        for cap, order in ((0, 0), (1 << 26, 0), (0, 1), (1 << 26, 1), (0, 2), (1 << 26, 2), (0, 2)):
            ctx.set_params(chunk_paths=cap, path_order=order, heavy_iters=160 if order == 2 else 0xFFFFFFFF)
            for k in range(16):
                ctx.render(1920, 1080, 4, 5, first_sample=4 * k, async_=True)
            ctx.sync()
            assert ctx.stats()["frames"] == 16
            assert np.array_equal(ctx.read_framebuffer(1920, 1080).view(np.uint32), want.view(np.uint32)), (cap, order)
        host = S.config3(1920, 1080, n_strands=1_000_000)
        rows = list(range(7, 1080, 270))
        ref = oracle_ffi.Oracle(host).render(1920, 1080, 64, 5, threads=16, rows=(7, 1080, 270))
        assert_parity(want[rows], ref[rows], exact=True)
    finally:
        ctx.close()


@pytest.fixture(scope="module")
def metric_oracle():
    """The oracle on the host-generated metric scene (config 3: 1M strands,
    9,000,002 objects); its BVH build takes ~15 s, so the tests below share it."""
    return oracle_ffi.Oracle(S.config3(1920, 1080, n_strands=1_000_000))


def test_driver_batch_chunks(metric_oracle):
    """The driver's bench command: 20 fused 8-spp passes at the metric size
    (332M paths), default parameters.  The automatic chunk size makes it ONE
    chunk (within 5/4 of the 2^28 cap, 288 GB of HBM); an explicit chunk_paths
    is a hard cap (2^27: 3 chunks, 2^26: 5).  All give the same framebuffer, bit
    for bit, and the default batch -- exactly what the timed region renders -- is
    the oracle's 160-spp frame on every 20th row (54 rows x 1920 px x 160 spp)."""
    ctx = HipContext(0)
    try:
        S.config3_device(ctx, 1920, 1080, n_strands=1_000_000)
        ctx.build_accel()
        got = {}
        for cap in (0, 1 << 27, 1 << 26):
            ctx.set_params(chunk_paths=cap)
            for k in range(20):
                ctx.render(1920, 1080, 8, 5, first_sample=8 * k, async_=True)
            ctx.sync()
            st = ctx.stats()
            assert st["frames"] == 20
            got[cap] = (st["extend_launches"], ctx.read_framebuffer(1920, 1080))
        assert [got[c][0] for c in (0, 1 << 27, 1 << 26)] == [1 * 5, 3 * 5, 5 * 5]
        for cap in (1 << 27, 1 << 26):
            assert np.array_equal(got[cap][1].view(np.uint32), got[0][1].view(np.uint32)), cap
    finally:
        ctx.close()
    rows = list(range(3, 1080, 20))
    assert len(rows) == 54
    want = metric_oracle.render(1920, 1080, 160, 5, threads=16, rows=(3, 1080, 20))
    assert_parity(got[0][1][rows], want[rows], exact=True)


def test_config3_stated_spp_rows(metric_oracle):
    """BASELINE config 3 at its stated 16 spp (one synchronous render of the
    1M-strand scene generated in HBM): every 20th row against the oracle."""
    ctx = HipContext(0)
    try:
        S.config3_device(ctx, 1920, 1080, n_strands=1_000_000)
        ctx.build_accel()
        got = ctx.render(1920, 1080, 16, 5)
    finally:
        ctx.close()
    rows = list(range(11, 1080, 20))
    assert len(rows) >= 54
    want = metric_oracle.render(1920, 1080, 16, 5, threads=16, rows=(11, 1080, 20))
    assert_parity(got[rows], want[rows], exact=True)


@pytest.mark.parametrize("max_paths", ["14000", "4096"])
def test_fused_frames_with_gathers_split(max_paths):
    """A fused batch with gathers that does not fit one chunk is split into
    chunk-sized groups (2 frames, or 1) that keep the call order."""
    from ba_pathtracing_fur_amd.pathtracer import comm_unique_id
    sd = S.config2(72, 48, n_strands=1500)
    want = oracle_ffi.Oracle(sd).render(72, 48, 8, 5, threads=16)
    ctx = HipContext(0)
    try:
        ctx.set_params(fuse_frames=4, chunk_paths=int(max_paths))
        ctx.set_scene(sd)
        ctx.build_accel()
        ctx.comm_init(1, 0, comm_unique_id())
        for first in range(0, 8, 2):
            ctx.render(72, 48, 2, 5, first_sample=first, tile_size=64, tile_rank=0, tile_nranks=1, async_=True)
            ctx.gather_framebuffer(72, 48, 2, 5, 64, 1, 0)
        ctx.sync()
        assert ctx.stats()["frames"] == 4
        assert_parity(ctx.read_framebuffer(72, 48), want, exact=True)
    finally:
        ctx.close()


def test_async_frames_across_changes():
    """Pending/fused asynchronous frames are completed before anything that
    changes what they read: a different frame size (new framebuffer), a new
    scene, a synchronous read."""
    sd = S.config2(48, 32, n_strands=800)
    sd2 = S.config1(40, 24)
    ctx = HipContext(0)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        for _ in range(3):
            ctx.render(48, 32, 2, 5, async_=True)
        ctx.render(40, 24, 2, 5, async_=True)        # new geometry: the 48x32 frames are flushed first
        ctx.sync()
        assert ctx.stats()["frames"] == 4
        assert_parity(ctx.read_framebuffer(40, 24), oracle_ffi.Oracle(sd).render(40, 24, 2, 5, threads=16),
                      exact=True)
        ctx.render(40, 24, 3, 5, async_=True)
        ctx.set_scene(sd2)                           # scene change with a frame pending
        ctx.build_accel()
        got = ctx.render(40, 24, 2, 4)
        assert_parity(got, oracle_ffi.Oracle(sd2).render(40, 24, 2, 4, threads=16), exact=True)
        assert ctx.lib.khp_render(ctx.ptr, None, None) != 0   # null parameters: an error status, no crash
        assert ctx.lib.khp_sync(None) != 0
    finally:
        ctx.close()


def test_native_library_is_loaded():
    """The frames above came from libkirk_hip.so (no fallback exists); it must be mapped in-process."""
    maps = open("/proc/self/maps").read()
    assert "libkirk_hip.so" in maps


def test_cpp_host_program_matches(hip_ctx, tmp_path):
    """examples/render_hairball (C++ on the C-ABI, no Python) renders the same config-3 frame."""
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "render_hairball")
    out = tmp_path / "f.pfm"
    subprocess.run([exe, "3000", "64", "40", "2", "5", "1", str(out)], check=True, timeout=300)
    raw = out.read_bytes()
    hdr_end = raw.index(b"-1.0\n") + 5
    img = np.frombuffer(raw[hdr_end:], np.float32).reshape(40, 64, 3)
    sd = S.config3(64, 40, n_strands=3000)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    want = hip_ctx.render(64, 40, 2, 5)
    assert np.array_equal(img.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("wide", ["0", "2"])
@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("name,kw", [("config2", dict(n_strands=3000)), ("config5", dict(n_strands=2000,
                                                                                          torus_grid=30))])
def test_production_traversal_kernels_ray_by_ray(hip_ctx, mode, name, kw, wide):
    """khp_ctx_params.trace_kernels routes the batch queries through the renderer's own
    persistent kernels: 1 = instrumented (KIRK's node/candidate visit counts must
    match the oracle's), 2 = the production build used in timed frames.  wide_from
    0: the closest-hit queries run on the two-level node records (traverse.h
    iterw), 2: on the 64-B records; axis-parallel rays take the one-level step."""
    sd = S.build_config(name, width=32, height=32, **kw)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    o = oracle_ffi.Oracle(sd)
    rng = np.random.default_rng(17)
    n = 100000
    orig = rng.uniform(-1.5, 1.5, (n, 3)).astype(np.float32) + np.float32([0, 1, 0])
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    tmax = rng.uniform(0.01, 2.0, n).astype(np.float32)
    # NaN rays (KIRK traces them; the production kernels answer them without the walk, ray_has_nan)
    d[:40] = np.nan
    d[40:60, 0] = np.nan
    d[60:80, 1] = np.nan
    orig[80:100, 2] = np.nan
    orig[100:120] = np.nan
    orig[120:140, 0] = np.nan   # the any-hit x-slab class (any_hit_x_nan): NaN origin x, finite direction
    orig[140:150, 1] = np.nan
    tmax[150:170] = np.nan
    # axis-parallel rays (infinite inverse direction components: the slab_sel path)
    d[170:200] = np.float32([0, 0, 1])
    d[200:230] = np.float32([0, -1, 0])
    d[230:260, 0] = 0.0
    d[230:260] /= np.linalg.norm(d[230:260], axis=1, keepdims=True)
    d[260:290] = np.float32([-1, 0, 0])
    t0, obj0, uv0, nodes, prims = o.trace_closest(orig, d)
    any0 = o.trace_any(orig, d, tmax)
    old = hip_ctx.set_params(trace_kernels=int(mode), wide_from=int(wide))
    try:
        t, obj, uv = hip_ctx.trace_closest(orig, d)
        st = hip_ctx.stats()
        a = hip_ctx.trace_any(orig, d, tmax)
    finally:
        hip_ctx.set_params(**old)
    assert np.array_equal(obj, obj0)
    assert np.array_equal(t.view(np.uint32), t0.view(np.uint32))
    assert np.array_equal(uv.view(np.uint32), uv0.view(np.uint32))
    assert np.array_equal(a, any0)
    if mode == "1":
        assert (st["node_visits"], st["prim_tests"]) == (nodes, prims)


@pytest.mark.parametrize("name,kw,w,h,spp,depth", [CASES[1], CASES[4], CASES[5], CASES[8]],
                         ids=["config2", "config5", "zoo", "textured"])
def test_wide_records_frames(hip_ctx, name, kw, w, h, spp, depth):
    """khp_ctx_params.wide_from: frames whose closest-hit traversal runs on the
    two-level node records from bounce 0, 1 or never are the oracle's, bit for
    bit, synchronous and instrumented; KIRK's visit counts do not change."""
    sd = S.build_config(name, width=w, height=h, **kw)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    want = oracle_ffi.Oracle(sd).render(w, h, spp, depth, threads=16)
    counts = set()
    old = hip_ctx.params()
    try:
        for wf in (0, 1, 64):
            hip_ctx.set_params(wide_from=wf)
            assert_parity(hip_ctx.render(w, h, spp, depth), want, exact=True)
            assert_parity(hip_ctx.render(w, h, spp, depth, stats=True), want, exact=True)
            st = hip_ctx.stats()
            counts.add((st["node_visits"], st["prim_tests"]))
    finally:
        hip_ctx.set_params(**old)
    assert len(counts) == 1


@pytest.mark.parametrize("name,kw,w,h,spp,depth", [CASES[1], CASES[4], CASES[5], CASES[8]],
                         ids=["config2", "config5", "zoo", "textured"])
def test_ray_sorting_frames(hip_ctx, name, kw, w, h, spp, depth):
    """khp_ctx_params.ray_sort_from (ABI 12): the wavefront's extension rays
    regrouped by origin cell from bounce 1, 2 (the automatic choice for large
    trees), 3, never (64) or automatic (0: never for these small trees) give
    the oracle's frame bit for bit -- synchronous, instrumented and fused
    asynchronous -- and KIRK's visit counts do not change.  The path kernel never
    sorts, so the synchronous calls here run the wavefront (path_kernel 1)."""
    sd = S.build_config(name, width=w, height=h, **kw)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    want = oracle_ffi.Oracle(sd).render(w, h, spp, depth, threads=16)
    counts = set()
    old = hip_ctx.params()
    try:
        for rs in (0, 1, 2, 3, 64):
            hip_ctx.set_params(ray_sort_from=rs, path_kernel=1)
            assert_parity(hip_ctx.render(w, h, spp, depth), want, exact=True)
            assert_parity(hip_ctx.render(w, h, spp, depth, stats=True), want, exact=True)
            st = hip_ctx.stats()
            counts.add((st["node_visits"], st["prim_tests"]))
            for k in range(spp):   # fused 1-spp passes
                hip_ctx.render(w, h, 1, depth, first_sample=k, async_=True)
            hip_ctx.sync()
            assert_parity(hip_ctx.read_framebuffer(w, h), want, exact=True)
    finally:
        hip_ctx.set_params(**old)
    assert len(counts) == 1


@pytest.mark.parametrize("name,kw,w,h,spp,depth", [CASES[0], CASES[1], CASES[4], CASES[5], CASES[8]],
                         ids=["config1", "config2", "config5", "zoo", "textured"])
def test_lds_top_nodes_frames(hip_ctx, name, kw, w, h, spp, depth):
    """khp_ctx_params.lds_nodes (ABI 12): the tree's top three levels of node
    records staged in each traversal wave's LDS (the 64-B loops of k_extend and
    k_shadow) give the oracle's frame bit for bit -- synchronous through the
    wavefront, and fused asynchronous passes -- with every bounce on the 64-B
    loop (wide_from past the depth) and with the default two-level records."""
    sd = S.build_config(name, width=w, height=h, **kw)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    want = oracle_ffi.Oracle(sd).render(w, h, spp, depth, threads=16)
    old = hip_ctx.params()
    try:
        for wf in (64, 2):
            hip_ctx.set_params(lds_nodes=7, path_kernel=1, wide_from=wf)
            assert_parity(hip_ctx.render(w, h, spp, depth), want, exact=True)
            for k in range(spp):
                hip_ctx.render(w, h, 1, depth, first_sample=k, async_=True)
            hip_ctx.sync()
            assert_parity(hip_ctx.read_framebuffer(w, h), want, exact=True)
    finally:
        hip_ctx.set_params(**old)


def test_lds_top_nodes_rejects_other_counts(hip_ctx):
    old = hip_ctx.params()
    with pytest.raises(Exception):
        hip_ctx.set_params(lds_nodes=3)
    assert hip_ctx.params() == old


PK_CASES = [CASES[0], CASES[1], CASES[2], CASES[3], CASES[4], CASES[5], CASES[8]]


@pytest.mark.parametrize("name,kw,w,h,spp,depth", PK_CASES,
                         ids=[f"{c[0]}-{c[1].get('bsdf', '')}{c[1].get('env', '')}{c[1].get('n_strands', '')}"
                              for c in PK_CASES])
def test_path_kernel_frames(name, kw, w, h, spp, depth):
    """khp_ctx_params.path_kernel (ABI 11): k_path, every bounce of a path in one
    persistent launch, on the 64-B and the two-level records, synchronous and
    fused asynchronous passes, gives the oracle's frame bit for bit -- the same
    frame the per-bounce wavefront (path_kernel 1) gives."""
    sd = S.build_config(name, width=w, height=h, **kw)
    want = oracle_ffi.Oracle(sd).render(w, h, 2 * spp, depth, threads=16)
    ctx = HipContext(0)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        for pk, wide in ((1, 2), (2, 2), (2, 0), (0, 2)):
            ctx.set_params(path_kernel=pk, wide_from=wide)
            ctx.render(w, h, spp, depth, readback=False)                     # synchronous pass
            ctx.render(w, h, spp, depth, first_sample=spp, readback=False)
            assert_parity(ctx.read_framebuffer(w, h), want, exact=True)
            for k in range(2):                                                # fused asynchronous passes
                ctx.render(w, h, spp, depth, first_sample=k * spp, async_=True)
            ctx.sync()
            assert_parity(ctx.read_framebuffer(w, h), want, exact=True)
    finally:
        ctx.close()


def test_path_kernel_full_size(metric_oracle):
    """The metric scene (1M strands, 1080p) through k_path: one synchronous 1-spp
    pass (KIRK's GUI call, path_kernel automatic) equals the wavefront's frame bit
    for bit, and every 27th row is the oracle's."""
    ctx = HipContext(0)
    try:
        S.config3_device(ctx, 1920, 1080, n_strands=1_000_000)
        ctx.build_accel()
        got = ctx.render(1920, 1080, 1, 5)
        ctx.set_params(path_kernel=1)
        wf = ctx.render(1920, 1080, 1, 5)
    finally:
        ctx.close()
    assert np.array_equal(got.view(np.uint32), wf.view(np.uint32))
    rows = list(range(13, 1080, 27))
    want = metric_oracle.render(1920, 1080, 1, 5, threads=16, rows=(13, 1080, 27))
    assert_parity(got[rows], want[rows], exact=True)
