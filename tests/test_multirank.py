"""Tile sharding across ranks (ba_pathtracing_fur_amd/sharding.py), world_size 2 on gloo, CPU only.

Each rank drives sharding.ShardedFrame exactly as bench.py does.  The GPU
context is replaced by a stand-in that renders this rank's tiles with the
oracle and moves the framebuffer over gloo with the PRODUCT's gather plan
(khp_gather_plan from libkirk_hip.so, the same host function
khp_gather_framebuffer builds its ncclSend/ncclRecv lists with): a sender packs
exactly the pixels its plan lists, the root receives counts[r] pixels from
each sender and scatters them by its own plan.  Rank 0's assembled frame must
equal the single-process frame bit for bit.  The RCCL transport itself runs on
a multi-GPU node (tests/test_multigpu.py).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ba_pathtracing_fur_amd import native
from ba_pathtracing_fur_amd import scenes as S
from ba_pathtracing_fur_amd import sharding

W, H, SPP, DEPTH, TILE = 40, 24, 2, 4, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    return S.config2(W, H, n_strands=200)


class OracleBackedCtx:
    """HipContext-shaped stand-in: oracle renders, gloo moves the owned pixels to root."""

    def __init__(self, scene):
        import oracle_ffi
        self.o = oracle_ffi.Oracle(scene)
        self.fb = np.zeros((H, W, 3), np.float32)
        self.uid = None

    def comm_init(self, nranks, rank, uid):
        self.uid, self.nranks, self.rank = uid, nranks, rank

    def render(self, width, height, spp, depth, seed, first_sample, tile_size, tile_rank, tile_nranks, readback,
               stats, async_=False):
        self.o.render(width, height, spp, depth, seed=seed, first_sample=first_sample, threads=2, out=self.fb,
                      tile_size=tile_size, tile_rank=tile_rank, tile_nranks=tile_nranks)

    def gather_framebuffer(self, width, height, spp, depth, tile, nranks, rank, root):
        counts, pix = native.gather_plan(width, height, tile, nranks, rank, root)
        flat = self.fb.reshape(-1, 3)
        if rank != root:        # k_pack + ncclSend of counts[rank] pixels
            assert int(counts.sum()) == int(counts[rank]) == len(pix)
            dist.send(torch.from_numpy(flat[pix].copy()), dst=root)
            return
        off = 0                 # ncclRecv of counts[r] pixels per sender, then k_unpack
        for r in range(nranks):
            if r == root:
                continue
            n = int(counts[r])
            buf = torch.empty((n, 3), dtype=torch.float32)
            dist.recv(buf, src=r)
            flat[pix[off:off + n]] = buf.numpy()
            off += n
        assert off == len(pix)

    def sync(self):
        pass


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, lr, w = sharding.env_ranks()
    assert (r, lr, w) == (rank, rank, world)
    ctx = OracleBackedCtx(_scene())
    frame = sharding.ShardedFrame(ctx, rank, world, dist, tile=TILE, unique_id=lambda: bytes(range(128)))
    assert ctx.uid == bytes(range(128))                  # root's id reached every rank
    frame.barrier()
    for _ in range(2):   # bench.py's pipelined steps: asynchronous frames + gathers, one sync at the end
        frame.render(W, H, SPP, DEPTH, async_=True)
    frame.sync()
    assert frame.max_over_ranks(float(rank + 1)) == float(world)
    assert frame.sum_over_ranks(1.0) == float(world)
    if rank == 0:
        np.save(os.path.join(out_dir, "frame.npy"), ctx.fb)
    frame.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_frame_equals_single_rank(tmp_path, world):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(tmp_path / "frame.npy")
    import oracle_ffi
    want = oracle_ffi.Oracle(_scene()).render(W, H, SPP, DEPTH, threads=2)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("w,h,t,n", [(40, 24, 8, 2), (1920, 1080, 64, 8), (100, 37, 16, 3), (64, 64, 64, 4)])
def test_tiles_partition_frame(w, h, t, n):
    masks = [sharding.owned_mask(w, h, r, n, t) for r in range(n)]
    total = np.sum(masks, axis=0)
    assert np.all(total == 1)                             # every pixel owned exactly once
    tx, ty = sharding.tile_grid(w, h, t)
    if tx * ty >= n:
        assert all(len(sharding.owned_tiles(w, h, r, n, t)) >= (tx * ty) // n for r in range(n))


def test_load_balance_at_metric_row():
    # 1080p / 64 px tiles = 510 tiles over 8 ranks: at most one tile of imbalance
    sizes = [len(sharding.owned_tiles(1920, 1080, r, 8)) for r in range(8)]
    assert max(sizes) - min(sizes) <= 1 and sum(sizes) == 30 * 17


def test_single_process_needs_no_dist():
    class Rec:
        calls = []

        def render(self, *a, **k):
            self.calls.append(k)

    ctx = Rec()
    f = sharding.ShardedFrame(ctx, 0, 1, None)
    f.render(W, H, SPP, DEPTH)
    assert ctx.calls[0]["tile_nranks"] == 1 and f.max_over_ranks(2.5) == 2.5
    with pytest.raises(ValueError):
        sharding.ShardedFrame(ctx, 0, 2, None)


@pytest.mark.parametrize("nranks", [2, 3, 8])
@pytest.mark.parametrize("w,h,t", [(1920, 1080, 64), (100, 37, 16), (40, 24, 8)])
def test_gather_plan_sender_matches_root(nranks, w, h, t):
    """khp_gather_plan: every sender sends exactly the pixels the root expects
    from it (the round-2 plan had every sender list the ROOT's pixels and send
    0 floats), and the root's lists are the senders' owned tiles."""
    for root in sorted({0, nranks - 1}):
        rc, rpix = native.gather_plan(w, h, t, nranks, root, root)
        assert rc[root] == 0 and int(rc.sum()) == len(rpix)
        off = 0
        for r in range(nranks):
            if r == root:
                continue
            sc, spix = native.gather_plan(w, h, t, nranks, r, root)
            assert int(sc[r]) == int(rc[r]) == len(spix) > 0 or (int(rc[r]) == 0 and len(spix) == 0)
            assert int(sc.sum()) == int(sc[r])                   # a sender lists only itself
            assert np.array_equal(spix, rpix[off:off + len(spix)])
            m = sharding.owned_mask(w, h, r, nranks, t).reshape(-1)
            assert np.array_equal(np.sort(spix), np.flatnonzero(m))  # its own tiles, each pixel once
            off += len(spix)
        # root's own tiles + everything it receives = the whole frame, each pixel once
        own = np.flatnonzero(sharding.owned_mask(w, h, root, nranks, t).reshape(-1))
        allpix = np.concatenate([own, rpix])
        assert len(allpix) == w * h and len(np.unique(allpix)) == w * h


def test_gather_plan_rejects_bad_arguments():
    for args in [(64, 64, 12, 2, 0, 0), (64, 64, 64, 2, 2, 0), (64, 64, 64, 2, 0, 5), (0, 64, 64, 2, 0, 0)]:
        with pytest.raises(native.KhpError):
            native.gather_plan(*args)
