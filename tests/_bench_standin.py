"""HipContext-shaped stand-in for bench.py's multi-rank orchestration on the CPU.

bench.py --ctx-factory tests/_bench_standin.py:OracleBenchCtx makes every rank
use this object instead of libkirk_hip.so's context, so `bench.py --gpus N`
runs its real launcher (torch.distributed.run, one process per rank), gloo
bootstrap, ShardedFrame, asynchronous passes with a gather after each,
max-over-ranks timing and rank 0's gather check on a machine without a GPU.

Rendering is the oracle's (this rank's tiles only); the gather moves exactly
the pixels of the PRODUCT's plan (khp_gather_plan, the host function the RCCL
gather uses) over gloo point-to-point, like tests/test_multirank.py.  Test
infrastructure only: the numbers such a run prints measure nothing.
KHP_STANDIN_CORRUPT=1 flips one pixel of every frame rank 1 sends, so the
gather check must fail.
"""
from __future__ import annotations

import os
import sys

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_ROOT, "oracle"))
import oracle_ffi  # noqa: E402

from ba_pathtracing_fur_amd import native as N  # noqa: E402


class OracleBenchCtx:
    def __init__(self, device=0, host_build=False):
        self.device = device
        self.o = None
        self.fb = None
        self.frames = 0
        self.rank, self.nranks = 0, 1
        lib = N.load_library()          # host-only call: khp_ctx_params defaults
        prm = N.CtxParams()
        lib.khp_ctx_params_defaults(prm)
        self.prm = prm.as_dict()
        self.n_objects = 0

    # scene ------------------------------------------------------------------------------
    def set_scene(self, sd):
        self.o = oracle_ffi.Oracle(sd)
        self.n_objects = sd.n_objects

    def build_accel(self):
        pass

    def params(self):
        return dict(self.prm)

    def set_params(self, **kw):
        old = dict(self.prm)
        self.prm.update({k: int(v) for k, v in kw.items()})
        return old

    def stats(self):
        s = N.Stats().as_dict()
        s.update(n_objects=self.n_objects, frames=max(1, self.frames))
        return s

    # frames -----------------------------------------------------------------------------
    def render(self, width, height, spp, depth, seed=0x4B49524B, first_sample=0, tile_size=64, tile_rank=0,
               tile_nranks=1, out=None, readback=True, stats=False, async_=False):
        if self.fb is None or self.fb.shape != (height, width, 3):
            self.fb = np.zeros((height, width, 3), np.float32)
        self.o.render(width, height, spp, depth, seed=seed, first_sample=first_sample, threads=2, out=self.fb,
                      tile_size=tile_size, tile_rank=tile_rank, tile_nranks=tile_nranks)
        self.frames += 1
        return self.fb.copy() if readback else None

    def sync(self):
        pass

    def read_framebuffer(self, width, height):
        return self.fb.copy()

    def read_rgba8(self, width, height, tonemap=None):
        return oracle_ffi.to_rgba8(self.fb)

    def close(self):
        self.o = None

    # gather over gloo with the product's plan --------------------------------------------------
    def comm_unique_id(self):
        return bytes(range(128))

    def comm_init(self, nranks, rank, uid, timeout_ms=None):
        self.nranks, self.rank = nranks, rank

    def gather_framebuffer(self, width, height, spp, depth, tile, nranks, rank, root=0):
        import torch
        import torch.distributed as dist
        counts, pix = N.gather_plan(width, height, tile, nranks, rank, root)
        flat = self.fb.reshape(-1, 3)
        if rank != root:
            buf = flat[pix].copy()
            if os.environ.get("KHP_STANDIN_CORRUPT") == "1" and rank == 1 and len(buf):
                buf[0, 0] += 1.0
            dist.send(torch.from_numpy(buf), dst=root)
            return
        off = 0
        for r in range(nranks):
            if r == root:
                continue
            n = int(counts[r])
            buf = torch.empty((n, 3), dtype=torch.float32)
            dist.recv(buf, src=r)
            flat[pix[off:off + n]] = buf.numpy()
            off += n
