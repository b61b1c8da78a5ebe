"""The multi-GPU path with real ranks: one process per GPU, tiles t % N, the RCCL
framebuffer gather (khp_gather_framebuffer: k_pack -> ncclSend/ncclRecv ->
k_unpack) and bench.py --gpus N launching its own ranks.  Needs >= 2 GPUs on
one node; skipped (not failed) on a single-GPU box, where tests/test_multirank.py
covers the sharding logic on gloo and test_gpu_parity.py every rank's tile set."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle_ffi
from _util import assert_parity
from ba_pathtracing_fur_amd import native as N
from ba_pathtracing_fur_amd import scenes as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _n_gpus() -> int:
    import torch
    return torch.cuda.device_count()   # counts devices without initialising HIP


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,W,H", [(2, 96, 64), (4, 96, 64), (8, 37, 23)])
def test_rccl_gather_assembles_the_single_gpu_frame(tmp_path, world, W, H):
    """Real ranks over RCCL; at 8 ranks a ragged 37x23 frame (6 tiles of 16 px),
    so ranks 6 and 7 own no pixel and post no send."""
    if _n_gpus() < world:
        pytest.skip(f"needs {world} GPUs, this box has {_n_gpus()}")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "tests", "_rccl_gather_worker.py"),
           str(tmp_path), str(W), str(H)]
    subprocess.run(cmd, check=True, timeout=240)
    got = np.load(tmp_path / "frame.npy")
    want = oracle_ffi.Oracle(S.config2(W, H, n_strands=1500)).render(W, H, 6, 5, threads=16)
    assert_parity(got, want, exact=True)


def test_bench_launches_its_own_ranks():
    if _n_gpus() < 2:
        pytest.skip(f"needs 2 GPUs, this box has {_n_gpus()}")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "1", "--steps",
                          "4", "--warmup", "2", "--sync-check-steps", "1", "--no-cpu-baseline"], check=True,
                         timeout=300, capture_output=True, text=True).stdout
    line = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("async_", [False, True])
def test_local_group_gather_assembles_the_frame(world, async_):
    """The product's gather on ONE GPU: `world` contexts of this process as the
    ranks (khp_comm_init_local), each rendering its tiles (t % world == rank),
    the gather moving the senders' pixels with the same plan (khp_gather_plan),
    k_pack and k_unpack as the RCCL path -- only the transport differs (device
    copies instead of ncclSend/ncclRecv).  Rank 0's frame must be the oracle's
    single-rank frame bit for bit, for synchronous passes and for fused
    asynchronous passes with a gather after each."""
    from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_init_local
    W, H, SPP, TILE, PASSES = 96, 64, 2, 16, 3
    sd = S.config2(W, H, n_strands=1500)
    want = oracle_ffi.Oracle(sd).render(W, H, SPP * PASSES, 5, threads=16)
    ctxs = [HipContext(0) for _ in range(world)]
    try:
        for c in ctxs:
            c.set_scene(sd)
            c.build_accel()
        comm_init_local(ctxs)
        for k in range(PASSES):
            for r in reversed(range(world)):   # senders enqueue their k-th gather before the root
                ctxs[r].render(W, H, SPP, 5, first_sample=k * SPP, tile_size=TILE, tile_rank=r, tile_nranks=world,
                               readback=False, async_=async_)
                ctxs[r].gather_framebuffer(W, H, SPP, 5, TILE, world, r, 0)
        for c in ctxs[1:]:                     # flush the senders' fused batches first
            c.sync()
        ctxs[0].sync()
        assert_parity(ctxs[0].read_framebuffer(W, H), want, exact=True)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("async_", [False, True])
def test_local_group_gather_with_empty_ranks(async_):
    """Ragged edges and ranks that own no tile: a 37x23 frame in 16-px tiles has
    6 tiles (the last column 5 px wide, the last row 7 px high), so of 8 ranks
    6 and 7 render and send nothing.  Their passes and gathers must still
    complete, and rank 0's frame is the oracle's bit for bit."""
    from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_init_local
    W, H, SPP, TILE, PASSES, world = 37, 23, 2, 16, 2, 8
    counts, _ = N.gather_plan(W, H, TILE, world, 0, 0)
    assert list(counts[6:]) == [0, 0] and all(int(c) > 0 for c in counts[1:6])
    sd = S.config2(W, H, n_strands=800)
    want = oracle_ffi.Oracle(sd).render(W, H, SPP * PASSES, 5, threads=16)
    ctxs = [HipContext(0) for _ in range(world)]
    try:
        for c in ctxs:
            c.set_scene(sd)
            c.build_accel()
        comm_init_local(ctxs)
        for k in range(PASSES):
            for r in reversed(range(world)):
                ctxs[r].render(W, H, SPP, 5, first_sample=k * SPP, tile_size=TILE, tile_rank=r, tile_nranks=world,
                               readback=False, async_=async_)
                ctxs[r].gather_framebuffer(W, H, SPP, 5, TILE, world, r, 0)
        for c in ctxs[1:]:
            c.sync()
        ctxs[0].sync()
        assert_parity(ctxs[0].read_framebuffer(W, H), want, exact=True)
    finally:
        for c in ctxs:
            c.close()


def test_local_group_config5_stated_form_eight_ranks():
    """BASELINE config 5 in its stated form -- 1M strands + 500x500x2-triangle
    torus + glass icosphere at 3840x2160, 32 spp, tiled over 8 ranks -- with the
    8 ranks as contexts of this process (khp_comm_init_local): four synchronous
    8-spp passes per rank (KIRK's progressive calls) with a gather after each.
    Rank 0's frame equals one context's frame of the same passes bit for bit
    over all 8.3M pixels, and every 54th row (plus row 860, which holds a NaN
    pixel) is the oracle's 32-spp frame.
    Only the transport differs from the RCCL path (device copies instead of
    ncclSend/ncclRecv)."""
    from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_init_local
    W, H, SPP, PASSES, TILE, world = 3840, 2160, 8, 4, 64, 8
    one = HipContext(0)
    try:
        S.config5_device(one, W, H, n_strands=1_000_000)
        one.build_accel()
        for k in range(PASSES):
            one.render(W, H, SPP, 5, first_sample=k * SPP, readback=False)
        want = one.read_framebuffer(W, H)
    finally:
        one.close()
    ctxs = [HipContext(0) for _ in range(world)]
    try:
        for c in ctxs:
            S.config5_device(c, W, H, n_strands=1_000_000)
            c.build_accel()
        comm_init_local(ctxs)
        for k in range(PASSES):
            for r in reversed(range(world)):   # senders enqueue their k-th gather before the root
                ctxs[r].render(W, H, SPP, 5, first_sample=k * SPP, tile_size=TILE, tile_rank=r, tile_nranks=world,
                               readback=False)
                ctxs[r].gather_framebuffer(W, H, SPP, 5, TILE, world, r, 0)
        for c in ctxs[1:]:
            c.sync()
        ctxs[0].sync()
        got = ctxs[0].read_framebuffer(W, H)
    finally:
        for c in ctxs:
            c.close()
    # a rank's 8-spp call (1M pixels) runs the path kernel, the whole frame's the
    # wavefront: the same values bit for bit; pixel (860, 2057) turns NaN at
    # sample 16 in both and in the oracle (KIRK's own arithmetic), with a
    # different NaN encoding on each (tests/_util.py)
    assert_parity(got, want, exact=True)
    assert np.isnan(got[860, 2057]).all()
    host = S.config5(W, H, n_strands=1_000_000)
    orc = oracle_ffi.Oracle(host)
    rows = list(range(11, H, 54)) + [860]
    ref = orc.render(W, H, SPP * PASSES, 5, threads=16, rows=(11, H, 54))
    ref = orc.render(W, H, SPP * PASSES, 5, threads=16, rows=(860, 861, 1), out=ref)
    assert_parity(got[rows], ref[rows], exact=True)


def test_local_group_driver_batch_two_ranks():
    """The driver's 2-GPU bench at the metric size, on one GPU: each of 2 ranks
    renders its tiles of 20 fused 8-spp passes with a gather after every pass
    (bench.py at N > 1).  A rank's 20 passes are 166M paths, within 5/4 of the
    2^27 cap, so flush() keeps them one group and enqueue_frames one chunk (5
    k_extend launches, not a 16 + 4 split).  Rank 0's frame equals the single-rank
    frame of the same passes, bit for bit."""
    from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_init_local
    W, H, SPP, PASSES, TILE = 1920, 1080, 8, 20, 64
    ctxs = [HipContext(0) for _ in range(2)]
    try:
        for c in ctxs:
            S.config3_device(c, W, H, n_strands=1_000_000)
            c.build_accel()
        for k in range(PASSES):
            ctxs[0].render(W, H, SPP, 5, first_sample=k * SPP, readback=False, async_=True)
        ctxs[0].sync()
        want = ctxs[0].read_framebuffer(W, H)
        comm_init_local(ctxs)
        for k in range(PASSES):
            for r in (1, 0):
                ctxs[r].render(W, H, SPP, 5, first_sample=k * SPP, tile_size=TILE, tile_rank=r, tile_nranks=2,
                               readback=False, async_=True)
                ctxs[r].gather_framebuffer(W, H, SPP, 5, TILE, 2, r, 0)
        ctxs[1].sync()
        assert ctxs[1].stats()["extend_launches"] == 5
        ctxs[0].sync()
        assert ctxs[0].stats()["extend_launches"] == 5
        got = ctxs[0].read_framebuffer(W, H)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    finally:
        for c in ctxs:
            c.close()


def test_rccl_single_rank_gather_on_one_gpu():
    """The RCCL path on a one-GPU box: a non-blocking communicator of one rank
    (khp_comm_init, ABI 11), rank 0's gather posting an empty receive group
    (ncclGroupStart/End), frames fused around it.  The frame is the untiled one."""
    from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_unique_id
    W, H, SPP = 64, 48, 2
    sd = S.config2(W, H, n_strands=800)
    want = oracle_ffi.Oracle(sd).render(W, H, 2 * SPP, 5, threads=16)
    ctx = HipContext(0)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        ctx.comm_init(1, 0, comm_unique_id(), timeout_ms=30000)
        for k in range(2):
            ctx.render(W, H, SPP, 5, first_sample=k * SPP, tile_size=16, tile_rank=0, tile_nranks=1, readback=False,
                       async_=True)
            ctx.gather_framebuffer(W, H, SPP, 5, 16, 1, 0, 0)
        ctx.sync()
        assert_parity(ctx.read_framebuffer(W, H), want, exact=True)
    finally:
        ctx.close()


def test_rccl_compute_waits_are_not_bounded():
    """the communicator's bound applies to RCCL operations that are
    runnable but not completing, never to compute.  With a one-rank communicator
    and a 1 ms bound, synchronous renders, fused passes with gathers between them
    and reads that each take far longer than 1 ms must all succeed (they used to
    abort the communicator and return KHP_EDEVICE), and the frame is the oracle's."""
    from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_unique_id
    W, H, SPP = 96, 64, 4
    sd = S.config2(W, H, n_strands=2000)
    want = oracle_ffi.Oracle(sd).render(W, H, 3 * SPP, 5, threads=16)
    ctx = HipContext(0)
    try:
        ctx.set_scene(sd)
        ctx.build_accel()
        ctx.comm_init(1, 0, comm_unique_id(), timeout_ms=30000)
        ctx.comm_set_timeout(1)
        ctx.render(W, H, SPP, 5, first_sample=0, tile_size=16, tile_rank=0, tile_nranks=1, readback=False)
        ctx.gather_framebuffer(W, H, SPP, 5, 16, 1, 0, 0)
        for k in (1, 2):
            ctx.render(W, H, SPP, 5, first_sample=k * SPP, tile_size=16, tile_rank=0, tile_nranks=1,
                       readback=False, async_=True)
            ctx.gather_framebuffer(W, H, SPP, 5, 16, 1, 0, 0)
        ctx.sync()
        assert_parity(ctx.read_framebuffer(W, H), want, exact=True)
    finally:
        ctx.close()


_ABORT_THEN_LOCAL = r"""
import os, sys
sys.path.insert(0, %(root)r)
import numpy as np
import torch.distributed as dist
from ba_pathtracing_fur_amd import native as N, scenes as S
from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_init_local, comm_unique_id
rank = int(os.environ["RANK"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%(port)d", rank=rank, world_size=2)
ctx = HipContext(rank)
sd = S.config2(64, 48, n_strands=1500)
ctx.set_scene(sd); ctx.build_accel()
uid = [comm_unique_id() if rank == 0 else None]
dist.broadcast_object_list(uid, src=0)
ctx.comm_init(2, rank, uid[0], timeout_ms=60000)
dist.barrier()
if rank == 1:                       # rank 1 never sends: the root's gather must abort
    dist.barrier()
    ctx.close(); print("ABORT_LOCAL_OK"); sys.exit(0)
ctx.comm_set_timeout(2000)
ctx.render(64, 48, 1, 5, tile_size=16, tile_rank=0, tile_nranks=2, readback=False)
try:
    ctx.gather_framebuffer(64, 48, 1, 5, 16, 2, 0, 0)
    ctx.sync()
    print("UNEXPECTED: gather completed"); sys.exit(1)
except N.KhpError as e:
    assert e.status == N.KHP_EDEVICE, e
dist.barrier()
comm_init_local([ctx])              # a one-member local group: no communicator any more
img = ctx.render(512, 384, 16, 5)   # far longer than the old 2 s bound on an aborted comm
assert img.shape == (384, 512, 3)
ctx.close(); print("ABORT_LOCAL_OK")
"""


def test_rccl_abort_then_local_group_waits_unbounded(tmp_path):
    """after a communicator abort, khp_comm_init_local must clear the
    dead communicator's state, so the context's later waits block normally
    instead of failing after the old bound with "still running after the abort"."""
    if _n_gpus() < 2:
        pytest.skip(f"needs 2 GPUs, this box has {_n_gpus()}")
    src = tmp_path / "abort_local.py"
    src.write_text(_ABORT_THEN_LOCAL % {"root": ROOT, "port": _port()})
    procs = [subprocess.Popen([sys.executable, str(src)], env={**os.environ, "RANK": str(r)},
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0 and "ABORT_LOCAL_OK" in o, (o[-2000:], e[-3000:])


_NO_PEER = r"""
import sys, time
sys.path.insert(0, %(root)r)
from ba_pathtracing_fur_amd import native as N, scenes as S
from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_unique_id
ctx = HipContext(0)
sd = S.config2(32, 24, n_strands=100)
ctx.set_scene(sd); ctx.build_accel()
t0 = time.time()
try:
    ctx.comm_init(2, 0, comm_unique_id(), timeout_ms=3000)   # rank 1 never joins
    print("UNEXPECTED: init succeeded"); sys.exit(1)
except N.KhpError as e:
    dt = time.time() - t0
    assert e.status == N.KHP_EDEVICE, e
    assert "rank 0 of 2" in str(e) and "3000 ms" in str(e), e
    assert dt < 30, dt
try:
    ctx.gather_framebuffer(32, 24, 1, 5, 16, 2, 0, 0)
    print("UNEXPECTED: gather without a communicator"); sys.exit(1)
except N.KhpError as e:
    assert e.status in (N.KHP_ENOTREADY, N.KHP_EINVAL), e
img = ctx.render(32, 24, 1, 5)          # the context is still usable
assert img.shape == (24, 32, 3)
# VERDICT r05 item 5 (ADVICE r04, the two-GPU test_rccl_abort_then_local_group_waits_unbounded
# on one GPU): after the abort, a 1 ms bound and a move into a one-member local group, a
# render that takes far longer than the bound completes normally
from ba_pathtracing_fur_amd.pathtracer import comm_init_local
ctx.comm_set_timeout(1)
t1 = time.time()
big = ctx.render(384, 288, 16, 5)       # ~tens of ms of device work
assert big.shape == (288, 384, 3)
comm_init_local([ctx])
big2 = ctx.render(384, 288, 16, 5, first_sample=16)
assert big2.shape == (288, 384, 3) and time.time() - t1 > 0.002
ctx.close()                             # khp_destroy with the abandoned init thread still blocked in RCCL
# the abandoned helper thread stays blocked inside ncclCommInitRankConfig (RCCL
# 2.27.7 does not return while a peer is missing): it holds only its own job, so a
# new context and a new (one-rank) communicator work beside it, and the process
# exits with it still blocked (this child's exit status is the check)
ctx2 = HipContext(0)
ctx2.set_scene(sd); ctx2.build_accel()
ctx2.comm_init(1, 0, comm_unique_id(), timeout_ms=30000)
ctx2.render(32, 24, 1, 5, tile_size=16, tile_rank=0, tile_nranks=1, readback=False)
ctx2.gather_framebuffer(32, 24, 1, 5, 16, 1, 0, 0)
ctx2.sync()
ctx2.close()
print("NO_PEER_OK %%.1f s" %% dt)
"""


def test_rccl_init_without_peer_fails_with_a_status():
    """A forced RCCL failure: rank 0 of 2 initialises while rank 1 never joins.
    The non-blocking init is polled against the context's timeout and returns
    KHP_EDEVICE naming the rank (it used to block in ncclCommInitRank forever).
    After the abort, with a 1 ms bound and the context moved into a local group,
    renders far longer than the bound complete (the one-GPU form of
    test_rccl_abort_then_local_group_waits_unbounded).  Run in a child process
    with its own time limit, so a regression cannot hang the test run."""
    r = subprocess.run([sys.executable, "-c", _NO_PEER % {"root": ROOT}], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "NO_PEER_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_bounded_waits_count_only_runnable_rccl_time(hip_ctx):
    """ADVICE r05 (comm_op_pending / poll_wait, ADVICE r04's rule): a rank's device
    wait is bounded only by the time its oldest RCCL operation has been runnable
    without completing.  khp_debug_comm_wait brackets a gate kernel (released by
    the host after `release` ms) with an operation's pre/post events: an operation
    whose `pre` is still pending never times out; a runnable one whose `post` does
    not complete fails after the bound; one with no `post` is retired once `pre`
    completes, and the wait on the compute behind it is not bounded."""
    import ctypes
    from ba_pathtracing_fur_amd import native as N
    lib, waited = hip_ctx.lib, ctypes.c_double(0.0)

    def run(scenario, bound, release):
        return lib.khp_debug_comm_wait(hip_ctx.ptr, scenario, bound, release, ctypes.byref(waited))

    assert run(0, 20, 200) == N.KHP_OK and waited.value >= 150, waited.value     # pending pre: no timeout
    st = run(1, 20, 400)                                                          # runnable, not completing
    assert st == N.KHP_EDEVICE and 15 <= waited.value < 300, (st, waited.value)
    assert "not complete" in (lib.khp_last_error() or b"").decode() or "still running" in (
        lib.khp_last_error() or b"").decode()
    assert run(2, 20, 200) == N.KHP_OK and waited.value >= 150, waited.value     # no post: retired at pre
    sd = S.config2(32, 24, n_strands=100)                                         # the context still renders
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    assert hip_ctx.render(32, 24, 1, 5).shape == (24, 32, 3)


def test_local_group_refuses_out_of_order_gathers():
    """khp_comm_init_local's stamped ring slots (ABI 11): a root gather enqueued
    before its sender's returns KHP_ENOTREADY and can be repeated; a sender 64
    gathers ahead of its root gets KHP_ENOTREADY instead of overwriting a slot
    the root has not copied (both used to copy stale pixels silently); the
    frame after the repeated gathers is still the oracle's."""
    from ba_pathtracing_fur_amd import native as N
    from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_init_local
    W, H, SPP, TILE = 48, 32, 1, 16
    sd = S.config2(W, H, n_strands=600)
    want = oracle_ffi.Oracle(sd).render(W, H, SPP, 5, threads=16)
    ctxs = [HipContext(0) for _ in range(2)]
    try:
        for c in ctxs:
            c.set_scene(sd)
            c.build_accel()
        comm_init_local(ctxs)
        for r in (0, 1):
            ctxs[r].render(W, H, SPP, 5, tile_size=TILE, tile_rank=r, tile_nranks=2, readback=False)
        with pytest.raises(N.KhpError) as e:       # root first: its sender has not packed gather 0
            ctxs[0].gather_framebuffer(W, H, SPP, 5, TILE, 2, 0, 0)
        assert e.value.status == N.KHP_ENOTREADY
        ctxs[1].gather_framebuffer(W, H, SPP, 5, TILE, 2, 1, 0)
        ctxs[0].gather_framebuffer(W, H, SPP, 5, TILE, 2, 0, 0)   # repeated: now it finds gather 0
        ctxs[0].sync()
        assert_parity(ctxs[0].read_framebuffer(W, H), want, exact=True)
        for _ in range(64):                        # gathers 1..64 fill the ring; the root takes none
            ctxs[1].gather_framebuffer(W, H, SPP, 5, TILE, 2, 1, 0)
        with pytest.raises(N.KhpError) as e:       # gather 65 would overwrite gather 1's slot
            ctxs[1].gather_framebuffer(W, H, SPP, 5, TILE, 2, 1, 0)
        assert e.value.status == N.KHP_ENOTREADY
        ctxs[0].gather_framebuffer(W, H, SPP, 5, TILE, 2, 0, 0)   # the root takes gather 1
        ctxs[1].gather_framebuffer(W, H, SPP, 5, TILE, 2, 1, 0)   # and slot 1 is free again
        ctxs[1].sync()
        ctxs[0].sync()
        comm_init_local(ctxs)                      # a new group starts from gather 0 on both
        ctxs[1].gather_framebuffer(W, H, SPP, 5, TILE, 2, 1, 0)
        ctxs[0].gather_framebuffer(W, H, SPP, 5, TILE, 2, 0, 0)
        ctxs[0].sync()
        assert_parity(ctxs[0].read_framebuffer(W, H), want, exact=True)
    finally:
        for c in ctxs:
            c.close()


def test_bench_two_ranks_on_one_gpu():
    """`bench.py --gpus 2` end to end with real HIP contexts on ONE GPU: the
    launcher, two bench processes rendering their tiles with libkirk_hip.so,
    asynchronous passes with a gather after each, the synchronous and isolated
    passes, max-over-ranks timing and rank 0's gather check on a second real
    context.  Only the transport is replaced (RCCL refuses two ranks on one GPU):
    tests/_bench_hip_gloo.py moves the product plan's pixels over gloo."""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "1", "--width", "64",
                          "--height", "48", "--spp", "2", "--tile", "16", "--steps", "3", "--warmup", "1",
                          "--sync-check-steps", "1", "--iso-steps", "1", "--gui-steps", "0", "--no-cpu-baseline",
                          "--ctx-factory", "tests/_bench_hip_gloo.py:HipGlooCtx", "--launch-timeout", "200"],
                         cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["value"] > 0
    assert line["gather_check"]["bit_exact"] and line["gather_check"]["passes"] == 1 + 1 + 3 + (1 + 1) + 1
