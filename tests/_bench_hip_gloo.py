"""HipContext with a gloo framebuffer gather, for `bench.py --gpus N` on ONE GPU.

bench.py --ctx-factory tests/_bench_hip_gloo.py:HipGlooCtx: every rank renders its
tiles with the real HIP kernels (libkirk_hip.so) on device 0 -- RCCL refuses two
ranks on one GPU, so the gather alone is replaced: a sender reads its
framebuffer and sends exactly the pixels of the product's plan (khp_gather_plan)
over gloo; the root patches the received pixels into the frame it reads back.
This runs bench.py's whole multi-rank orchestration (real launcher, tile
shards, asynchronous passes, sync steps, the isolated re-run, rank 0's gather
check on a second real context) on a one-GPU box.  Test infrastructure only.
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ba_pathtracing_fur_amd import native as N  # noqa: E402
from ba_pathtracing_fur_amd.pathtracer import HipContext  # noqa: E402


class HipGlooCtx(HipContext):
    def __init__(self, device=0, host_build=False):
        super().__init__(device=0, host_build=host_build)   # every rank on the one GPU
        self.recv = None   # root: pixels received from the senders (flat index -> rgb)
        self.nranks, self.rank = 1, 0

    def comm_unique_id(self):
        return bytes(128)

    def comm_init(self, nranks, rank, uid, timeout_ms=None):
        self.nranks, self.rank = nranks, rank

    def gather_framebuffer(self, width, height, spp, depth, tile_size, nranks, rank, root=0):
        import torch
        import torch.distributed as dist
        counts, pix = N.gather_plan(width, height, tile_size, nranks, rank, root)
        if rank != root:
            self.sync()
            flat = super().read_framebuffer(width, height).reshape(-1, 3)
            dist.send(torch.from_numpy(np.ascontiguousarray(flat[pix])), dst=root)
            return
        if self.recv is None or self.recv[0].shape != (width * height, 3):
            self.recv = (np.zeros((width * height, 3), np.float32), np.zeros(width * height, bool))
        off = 0
        for r in range(nranks):
            if r == root:
                continue
            n = int(counts[r])
            buf = torch.empty((n, 3), dtype=torch.float32)
            dist.recv(buf, src=r)
            self.recv[0][pix[off:off + n]] = buf.numpy()
            self.recv[1][pix[off:off + n]] = True
            off += n

    def read_framebuffer(self, width, height):
        img = super().read_framebuffer(width, height)
        if self.recv is not None and self.recv[0].shape == (width * height, 3):
            flat = img.reshape(-1, 3)
            flat[self.recv[1]] = self.recv[0][self.recv[1]]
        return img
