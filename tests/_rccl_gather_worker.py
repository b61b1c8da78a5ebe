"""Worker of tests/test_multigpu.py (run by torch.distributed.run, one rank per GPU):
renders this rank's tiles of a small config-2 frame as progressive asynchronous
passes with a real RCCL framebuffer gather after each (khp_gather_framebuffer),
and rank 0 saves the assembled framebuffer.  Not collected by pytest."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    W, H, SPP, DEPTH, TILE = int(sys.argv[2]), int(sys.argv[3]), 2, 5, 16
    import torch  # noqa: F401  (HIP runtime before libkirk_hip.so)
    import torch.distributed as dist

    from ba_pathtracing_fur_amd import HipContext, scenes
    from ba_pathtracing_fur_amd.sharding import ShardedFrame, env_ranks

    rank, local_rank, world = env_ranks()
    dist.init_process_group("gloo")
    ctx = HipContext(local_rank)
    ctx.set_scene(scenes.config2(W, H, n_strands=1500))
    ctx.build_accel()
    frame = ShardedFrame(ctx, rank, world, dist, tile=TILE)
    for k in range(3):  # progressive passes, each followed by its gather, one sync at the end
        frame.render(W, H, SPP, DEPTH, first_sample=k * SPP, async_=True)
    frame.sync()
    frame.barrier()
    if rank == 0:
        np.save(os.path.join(out, "frame.npy"), ctx.read_framebuffer(W, H))
    frame.barrier()
    dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
