"""Multi-GPU frame sharding: one process per GPU, tiles interleaved over ranks.

SURVEY §8(e): KIRK has no multi-device path; north_star asks for frames
sharded by tile across the GPUs of one node with one small RCCL gather of the
framebuffer over xGMI.  Tile t (64x64 px, row-major over the frame) belongs to
rank t % N, so every rank gets an even, spatially spread share of the hairball
(load balance without a work queue).  Each rank renders only its tiles; rank 0
then receives the other ranks' tiles with one grouped ncclSend/ncclRecv
(khp_gather_framebuffer).  The total frame is fixed, so scaling is "strong".

torch.distributed is the bootstrap channel only (RANK/WORLD_SIZE/MASTER_* from
torchrun; "gloo" carries the 128-byte RCCL unique id and the max-over-ranks
timing); the framebuffer itself moves over RCCL inside libkirk_hip.so.
"""
from __future__ import annotations

import os

import numpy as np

TILE = 64


def env_ranks() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (defaults: single process)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def tile_grid(width: int, height: int, tile: int = TILE) -> tuple[int, int]:
    return (width + tile - 1) // tile, (height + tile - 1) // tile


def owned_tiles(width: int, height: int, rank: int, nranks: int, tile: int = TILE) -> list[int]:
    """Tile ids owned by `rank` (render.hip owned_pixels: tile_id % nranks == rank)."""
    tx, ty = tile_grid(width, height, tile)
    return [t for t in range(tx * ty) if nranks <= 1 or t % nranks == rank]


def owned_mask(width: int, height: int, rank: int, nranks: int, tile: int = TILE) -> np.ndarray:
    """(H, W) bool mask of the pixels `rank` renders."""
    tx, _ = tile_grid(width, height, tile)
    m = np.zeros((height, width), bool)
    for t in owned_tiles(width, height, rank, nranks, tile):
        x0, y0 = (t % tx) * tile, (t // tx) * tile
        m[y0:y0 + tile, x0:x0 + tile] = True
    return m


class ShardedFrame:
    """Renders one frame's share on this rank and gathers the frame on rank 0.

    `ctx` is a pathtracer.HipContext (or anything with its render / comm_init /
    gather_framebuffer methods); `dist` is torch.distributed, already
    initialised, or None for a single process.
    """

    def __init__(self, ctx, rank: int, world: int, dist=None, tile: int = TILE, root: int = 0,
                 unique_id=None, comm_timeout_ms: int | None = None):
        """comm_timeout_ms: khp_comm_set_timeout (ABI 11) -- the RCCL init and every
        later wait of the context fail with KHP_EDEVICE instead of hanging when a
        peer is lost or a gather has no counterpart (library default 120 s)."""
        if world > 1 and dist is None:
            raise ValueError("world_size > 1 needs an initialised torch.distributed")
        self.ctx, self.rank, self.world, self.dist, self.tile, self.root = ctx, rank, world, dist, tile, root
        if world > 1:
            if unique_id is None:
                from .pathtracer import comm_unique_id as unique_id
            obj = [unique_id() if rank == root else None]
            dist.broadcast_object_list(obj, src=root)
            if comm_timeout_ms is None:
                ctx.comm_init(world, rank, obj[0])
            else:
                ctx.comm_init(world, rank, obj[0], timeout_ms=comm_timeout_ms)

    def render(self, width, height, spp, depth, seed=0x4B49524B, first_sample=0, stats=False, gather=True,
               async_=False):
        """One frame (or a progressive slice of samples) of this rank's tiles, framebuffer left in HBM.

        async_=True enqueues the frame and its gather without waiting (frames in
        flight overlap on the device); sync() completes them."""
        self.ctx.render(width, height, spp, depth, seed=seed, first_sample=first_sample, tile_size=self.tile,
                        tile_rank=self.rank, tile_nranks=self.world, readback=False, stats=stats,
                        async_=async_ and not stats)
        if gather and self.world > 1:
            self.ctx.gather_framebuffer(width, height, spp, depth, self.tile, self.world, self.rank, self.root)

    def sync(self):
        self.ctx.sync()

    def barrier(self):
        if self.dist is not None and self.world > 1:
            self.dist.barrier()

    def max_over_ranks(self, x: float) -> float:
        if self.dist is None or self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x: float) -> float:
        if self.dist is None or self.world == 1:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())
