"""Render-ahead (khp_ctx_params.render_ahead, ABI 13) on an MI355X.

KIRK's GUI calls PathTracer::render once per pass and reads the texture
(CPU_PathTracer.cpp:17-52, drawTexture :61-90).  With render-ahead, the path
kernel's launch for call k lets its idle drain lanes start the paths of call
k+1 (same pixels, samples first_sample + spp ...), parks the ones still in
flight when call k's own paths are done, and call k+1 resumes them.  The bar:
after EVERY call the framebuffer and the 8-bit texture are the oracle's
progressive ones (KIRK's running mean over the same passes) bit for bit, and a
change of camera, parameters, spp or first_sample between calls drops the
ahead work instead of using it.
"""
import numpy as np
import pytest

import oracle_ffi
from _util import assert_parity
from ba_pathtracing_fur_amd import native as N
from ba_pathtracing_fur_amd import scenes as S
from ba_pathtracing_fur_amd.pathtracer import HipContext

pytestmark = pytest.mark.gpu


def _moved(cam: N.Camera, d) -> N.Camera:
    """The camera translated by d (position and image plane alike)."""
    c = N.Camera.from_buffer_copy(bytes(cam))
    for k in range(3):
        c.position[k] += d[k]
        c.bottom_left[k] += d[k]
    return c


class _Series:
    """The oracle's progressive framebuffer over the same calls (KIRK's running mean)."""

    def __init__(self, sd, w, h, depth):
        self.sd, self.w, self.h, self.depth = sd, w, h, depth
        self.orc = oracle_ffi.Oracle(sd)
        self.fb = np.zeros((h, w, 3), np.float32)

    def camera(self, cam):
        self.sd.cam = cam
        self.orc = oracle_ffi.Oracle(self.sd)

    def call(self, spp, first_sample):
        self.orc.render(self.w, self.h, spp, self.depth, first_sample=first_sample, threads=16, out=self.fb)
        return self.fb


def _check(ctx, ser, w, h, what):
    got = ctx.read_framebuffer(w, h)
    assert_parity(got, ser.fb, exact=True)
    assert np.array_equal(ctx.read_rgba8(w, h), oracle_ffi.to_rgba8(ser.fb)), what


SCENES = [("config2", dict(n_strands=2000), 64, 48, 5), ("zoo", dict(n_strands=400), 96, 72, 8),
          ("textured", dict(n_strands=600, env="cube"), 80, 60, 6), ("config3", dict(n_strands=20000), 96, 54, 5)]


@pytest.mark.parametrize("name,kw,w,h,depth", SCENES, ids=[s[0] for s in SCENES])
@pytest.mark.parametrize("spp,wide,ahead_sets", [(1, 2, 2), (2, 0, 1), (3, 2, 3)])
def test_progressive_calls_match_oracle(name, kw, w, h, depth, spp, wide, ahead_sets):
    """Synchronous calls first_sample = 0, spp, 2 spp, ...: every call's
    framebuffer and texture are the oracle's, and from the second call on the
    call found work rendered ahead for it (khp_stats.ahead_*), with 1, 2 and 3
    later calls' sets rendered ahead."""
    sd = S.build_config(name, width=w, height=h, **kw)
    ser = _Series(sd, w, h, depth)
    ctx = HipContext(0)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        ctx.set_params(path_kernel=2, wide_from=wide, render_ahead=ahead_sets)
        ahead = []
        for k in range(6):
            ctx.render(w, h, spp, depth, first_sample=k * spp, readback=False)
            st = ctx.stats()
            ahead.append(st["ahead_finished"] + st["ahead_resumed"])
            ser.call(spp, k * spp)
            _check(ctx, ser, w, h, f"call {k}")
        assert ahead[0] == 0
        # each later call found work rendered ahead for it -- unless the previous call
        # had found ITS whole set finished: that call returns at once and renders nothing ahead
        n = w * h * spp
        assert all(ahead[k] > 0 or ahead[k - 1] == n for k in range(1, 6)), ahead
        assert max(ahead[1:]) > 0, ahead
    finally:
        ctx.close()


def test_changes_between_calls_drop_the_ahead_work():
    """Between calls: a camera move (khp_set_camera) with the next first_sample,
    a parameter change, a skipped and a repeated first_sample, another spp, a
    fused asynchronous pass and a wavefront call -- each call's frame is the
    oracle's series, which a stale ahead set would break."""
    w, h, depth = 64, 48, 5
    sd = S.config2(w, h, n_strands=2000)
    ser = _Series(sd, w, h, depth)
    ctx = HipContext(0)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        ctx.set_params(path_kernel=2)
        plan = [("call", 1, 0), ("call", 1, 1), ("camera", (0.05, 0.0, -0.1)), ("call", 1, 2), ("call", 1, 3),
                ("params", dict(wide_from=0)), ("call", 1, 4), ("call", 1, 6), ("call", 1, 6), ("call", 2, 7),
                ("call", 2, 9), ("async", 2, 11), ("call", 2, 13), ("call", 2, 15), ("wavefront", 2, 17),
                ("call", 2, 19), ("camera", (0.0, 0.02, 0.0)), ("call", 2, 21), ("call", 2, 23)]
        resumed = 0
        for step in plan:
            kind = step[0]
            if kind == "camera":
                cam = _moved(sd.cam, step[1])
                ctx.set_camera(cam)
                ser.camera(cam)
                continue
            if kind == "params":
                ctx.set_params(**step[1])
                continue
            spp, fs = step[1], step[2]
            if kind == "async":
                ctx.render(w, h, spp, depth, first_sample=fs, async_=True)
                ctx.sync()
            elif kind == "wavefront":
                old = ctx.set_params(path_kernel=1)
                ctx.render(w, h, spp, depth, first_sample=fs, readback=False)
                ctx.set_params(path_kernel=old["path_kernel"])
            else:
                ctx.render(w, h, spp, depth, first_sample=fs, readback=False)
                st = ctx.stats()
                resumed += st["ahead_finished"] + st["ahead_resumed"]
            ser.call(spp, fs)
            _check(ctx, ser, w, h, str(step))
        assert resumed > 0
    finally:
        ctx.close()


def test_render_ahead_off_and_validation(hip_ctx):
    """render_ahead 0 renders the same frames with nothing ahead; values > 1 are refused."""
    w, h, depth = 48, 32, 5
    sd = S.config2(w, h, n_strands=1000)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    old = hip_ctx.set_params(render_ahead=0, path_kernel=2)
    try:
        for k in range(3):
            hip_ctx.render(w, h, 1, depth, first_sample=k, readback=False)
            st = hip_ctx.stats()
            assert st["ahead_finished"] == 0 and st["ahead_resumed"] == 0
        got = hip_ctx.read_framebuffer(w, h)
        assert_parity(got, oracle_ffi.Oracle(sd).render(w, h, 3, depth, threads=16), exact=True)
        with pytest.raises(N.KhpError):
            hip_ctx.set_params(render_ahead=4)
    finally:
        hip_ctx.set_params(**old)


def test_set_camera_equals_a_rebuilt_scene(hip_ctx):
    """khp_set_camera renders what khp_set_scene with that camera renders."""
    w, h, depth = 48, 32, 5
    sd = S.config2(w, h, n_strands=1000)
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    cam = _moved(sd.cam, (0.1, -0.05, 0.2))
    hip_ctx.set_camera(cam)
    got = hip_ctx.render(w, h, 2, depth)
    sd.cam = cam
    want = oracle_ffi.Oracle(sd).render(w, h, 2, depth, threads=16)
    assert_parity(got, want, exact=True)


@pytest.fixture(scope="module")
def metric_scene_oracle():
    return oracle_ffi.Oracle(S.config3(1920, 1080, n_strands=1_000_000))


def test_gui_calls_full_size(metric_scene_oracle):
    """The metric scene at 1080p, KIRK's GUI call (1 spp + texture) four times
    with render-ahead (the default): each call's framebuffer equals the same
    calls without it bit for bit, the later calls found paths finished ahead
    (and, unless their whole set was, parked ones), and every 27th row of the
    last frame is the oracle's."""
    W, H, D = 1920, 1080, 5
    frames = {}
    counts = []
    for ra in (1, 0):
        ctx = HipContext(0)
        try:
            S.config3_device(ctx, W, H, n_strands=1_000_000)
            ctx.build_accel()
            ctx.set_params(render_ahead=ra)
            fbs, tex = [], []
            for k in range(4):
                ctx.render(W, H, 1, D, first_sample=k, readback=False)
                if ra:
                    st = ctx.stats()
                    counts.append((st["ahead_finished"], st["ahead_resumed"]))
                fbs.append(ctx.read_framebuffer(W, H))
                tex.append(ctx.read_rgba8(W, H))
            frames[ra] = (fbs, tex)
        finally:
            ctx.close()
    for k in range(4):
        assert np.array_equal(frames[1][0][k].view(np.uint32), frames[0][0][k].view(np.uint32)), k
        assert np.array_equal(frames[1][1][k], frames[0][1][k]), k
    assert counts[0] == (0, 0)
    assert all(f > 0 and (r > 0 or f == W * H) for f, r in counts[1:]), counts
    rows = (13, 1080, 27)
    want = np.zeros((H, W, 3), np.float32)
    for k in range(4):
        metric_scene_oracle.render(W, H, 1, D, first_sample=k, threads=16, rows=rows, out=want)
    idx = list(range(*rows))
    assert_parity(frames[1][0][3][idx], want[idx], exact=True)


# ---- render-ahead through fusion: the wavefront's synchronous calls -------------------------


@pytest.mark.parametrize("name,kw,w,h,depth", SCENES, ids=[s[0] for s in SCENES])
@pytest.mark.parametrize("spp,ahead_sets", [(2, 2), (3, 1), (1, 3)])
def test_wavefront_series_match_oracle(name, kw, w, h, depth, spp, ahead_sets):
    """Synchronous wavefront calls (path_kernel 1) first_sample = 0, spp, ...:
    the series' second call renders itself and the next ahead_sets calls' passes
    as one fused batch, those calls only accumulate (khp_stats.ahead_finished =
    all their paths), then the next call renders a batch again -- and every
    call's framebuffer and texture are the oracle's progressive ones."""
    sd = S.build_config(name, width=w, height=h, **kw)
    ser = _Series(sd, w, h, depth)
    ctx = HipContext(0)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        ctx.set_params(path_kernel=1, render_ahead=ahead_sets)
        ahead = []
        calls = 2 + 2 * (ahead_sets + 1)
        for k in range(calls):
            out = ctx.render(w, h, spp, depth, first_sample=k * spp, readback=(k == 2))   # call 2 only accumulates
            ahead.append(ctx.stats()["ahead_finished"])
            ser.call(spp, k * spp)
            _check(ctx, ser, w, h, f"call {k}")
            if k == 2:   # the readback of a call whose pass was rendered ahead
                assert_parity(out, ser.fb, exact=True)
        n = w * h * spp
        group = [0] + [n] * ahead_sets
        assert ahead == [0] + group * 2 + [0], ahead
    finally:
        ctx.close()


def test_wavefront_changes_between_calls_drop_the_batch():
    """Between wavefront calls whose batch holds later passes: a camera move, a
    parameter change, a skipped and a repeated first_sample, another spp, a
    fused asynchronous pass, a path-kernel call and a batch ray query (which
    reuses the batch's path set) -- each call's frame is the oracle's series,
    which a stale batch would break."""
    w, h, depth = 64, 48, 5
    sd = S.config2(w, h, n_strands=2000)
    ser = _Series(sd, w, h, depth)
    ctx = HipContext(0)
    rng = np.random.default_rng(7)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        ctx.set_params(path_kernel=1, trace_kernels=2, render_ahead=3)
        plan = [("call", 2, 0), ("call", 2, 2), ("call", 2, 4), ("camera", (0.05, 0.0, -0.1)), ("call", 2, 6),
                ("call", 2, 8), ("call", 2, 10), ("params", dict(wide_from=0)), ("call", 2, 12), ("call", 2, 14),
                ("call", 2, 16), ("call", 2, 20), ("call", 2, 22), ("call", 2, 24), ("call", 2, 24), ("call", 2, 26),
                ("call", 2, 28), ("call", 1, 30), ("call", 2, 31), ("call", 2, 33), ("async", 2, 35), ("call", 2, 37),
                ("call", 2, 39), ("call", 2, 41), ("pathk", 2, 43), ("call", 2, 45), ("call", 2, 47), ("call", 2, 49),
                ("query",), ("call", 2, 51), ("call", 2, 53), ("call", 2, 55)]
        hits = 0
        for step in plan:
            kind = step[0]
            if kind == "camera":
                cam = _moved(sd.cam, step[1])
                ctx.set_camera(cam)
                ser.camera(cam)
                continue
            if kind == "params":
                ctx.set_params(**step[1])
                continue
            if kind == "query":
                o = np.tile(np.asarray(sd.cam.position, np.float32), (4096, 1))
                d = rng.normal(size=(4096, 3)).astype(np.float32)
                d /= np.linalg.norm(d, axis=1, keepdims=True)
                ctx.trace_closest(o, d)
                continue
            spp, fs = step[1], step[2]
            if kind == "async":
                ctx.render(w, h, spp, depth, first_sample=fs, async_=True)
                ctx.sync()
            elif kind == "pathk":
                ctx.set_params(path_kernel=2)
                ctx.render(w, h, spp, depth, first_sample=fs, readback=False)
                ctx.set_params(path_kernel=1)
            else:
                ctx.render(w, h, spp, depth, first_sample=fs, readback=False)
                hits += ctx.stats()["ahead_finished"] == w * h * spp
            ser.call(spp, fs)
            _check(ctx, ser, w, h, str(step))
        assert hits >= 4, hits
    finally:
        ctx.close()


def test_wavefront_calls_full_size(metric_scene_oracle):
    """The metric scene at 1080p, 8-spp synchronous calls (the automatic choice
    runs them through the wavefront): six calls with render-ahead (the default)
    equal the same calls without it bit for bit, calls 2 and 3 found their pass
    in call 1's batch, and every 54th row of the last frame is the oracle's."""
    W, H, D, SPP = 1920, 1080, 5, 8
    frames, ahead = {}, []
    for ra in (2, 0):
        ctx = HipContext(0)
        try:
            S.config3_device(ctx, W, H, n_strands=1_000_000)
            ctx.build_accel()
            ctx.set_params(render_ahead=ra)
            fbs = []
            for k in range(6):
                ctx.render(W, H, SPP, D, first_sample=k * SPP, readback=False)
                if ra:
                    ahead.append(ctx.stats()["ahead_finished"])
                fbs.append(ctx.read_framebuffer(W, H))
            frames[ra] = fbs
        finally:
            ctx.close()
    for k in range(6):
        assert np.array_equal(frames[2][k].view(np.uint32), frames[0][k].view(np.uint32)), k
    n = W * H * SPP
    assert ahead == [0, 0, n, n, 0, n], ahead
    rows = (13, 1080, 54)
    want = np.zeros((H, W, 3), np.float32)
    for k in range(6):
        metric_scene_oracle.render(W, H, SPP, D, first_sample=k * SPP, threads=16, rows=rows, out=want)
    idx = list(range(*rows))
    assert_parity(frames[2][5][idx], want[idx], exact=True)
