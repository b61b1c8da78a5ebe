#!/usr/bin/env python3
"""Headline benchmark: Msamples/s at 1080p 8 spp on the 1M-strand hairball.

BASELINE.json metric: "Msamples/s at 1080p 8spp, 1M-strand hairball; achieved
HBM GB/s vs peak".  Workload = config 3's scene (1M strands -> 9M cone frusta
on a 2-triangle plane, 2x2 quad light, sky environment) rendered at
1920x1080, 8 spp, depth 5 (SURVEY §8(d) "Metric row").

One step = one full frame (16.6M camera samples) through the HIP wavefront
core, inputs (scene + BVH) resident in HBM, framebuffer left in HBM.  With
--gpus N (torchrun, one process per GPU) the frame is tile-sharded
(64x64 tiles, tile_id % N) and each step ends with the RCCL framebuffer
gather to rank 0; total work is fixed, so scaling is "strong".

Steps are pipelined (default): each frame is enqueued asynchronously
(KHP_RENDER_ASYNC) and up to two frames run on the device at once, so one
frame's chain of 2 x depth persistent launches -- each ending only when its
slowest ray does -- overlaps the other frame's work; frames still complete and
accumulate in order, and the timed region ends with khp_sync + a barrier.
--sync-steps waits for every frame before starting the next.

The JSON line also carries:
  roofline     -- the extend (closest-hit) kernel: algorithmic bytes
                  (28 B ray + 32 B per visited node + 32 B per
                  primitive test + 16 B hit, visit counts from an instrumented
                  frame) of all timed launches / the time during which at
                  least one of them was running (union of their HIP-event
                  intervals), against 8 TB/s HBM.  Without overlap
                  (--sync-steps) that is bytes per launch / average launch
                  time; avg_launch_ms and achieved_per_launch give the
                  per-launch view (launch durations include the time the
                  other frame's kernels shared the chip);
  cpu_baseline -- the C restatement (oracle/) timed on this host's cores on a
                  bounded sample of the same frame: progressive full-frame
                  samples 0, 1, ... until --cpu-seconds or the workload's spp.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--strands", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sync-steps", action="store_true",
                    help="wait for each frame before the next (no frame pipelining)")
    ap.add_argument("--host-scene", action="store_true",
                    help="generate + flatten + build on the host (the pre-(f)1/(f)2 path) instead of in HBM")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(sd, args, budget_s):
    """Oracle timed on the host cores over a bounded sample of the same frame."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle_ffi  # test infrastructure: only bench's cpu_baseline leg uses it

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    t0 = time.time()
    o = oracle_ffi.Oracle(sd)
    build_s = time.time() - t0
    W, H = args.width, args.height
    frame = W * H
    # progressive full frames (sample k of the same seeds) until the budget is spent or the
    # workload's spp is reached; if one frame alone would blow the budget, every k-th row instead
    step = max(1, H // 8)
    t0 = time.time()
    o.render(W, H, 1, args.depth, threads=threads, rows=(0, H, step))
    pilot = time.time() - t0
    est_frame_s = pilot * H / len(range(0, H, step))
    if est_frame_s <= budget_s:
        out = None
        spp_cpu = 0
        t0 = time.time()
        while spp_cpu < args.spp and time.time() - t0 < budget_s:
            out = o.render(W, H, 1, args.depth, first_sample=spp_cpu, threads=threads, out=out)
            spp_cpu += 1
        dt = time.time() - t0
        samples = frame * spp_cpu
        what = f"full {W}x{H} frame x {spp_cpu} of {args.spp} spp"
    else:
        n_rows = int(max(1, budget_s / est_frame_s * H))
        step = max(1, H // n_rows)
        rows = len(range(0, H, step))
        t0 = time.time()
        o.render(W, H, 1, args.depth, threads=threads, rows=(0, H, step))
        dt = time.time() - t0
        samples = rows * W
        what = f"{rows} of {H} rows (every {step}th) x {W} px x 1 spp"
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{what} of the same frame = {samples} samples in {dt:.1f} s ({threads} threads, "
                      f"CPU restatement oracle/, -O3 x86-64-v3, same seeds); throughput is spp-linear; "
                      f"oracle BVH build {build_s:.1f} s excluded"}


def pmc_traffic(frames_per_launch: float):
    """HBM bytes per k_extend launch from the committed PMC profile, scaled to
    this run's frames per launch (the profile records how many fused frames
    its launches carried), or None."""
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "pmc_extend_*.json")))
    if not files:
        return None
    try:
        with open(files[-1]) as f:
            d = json.load(f)
        return int(d["bytes_per_launch"] / d.get("frames_per_launch", 1) * frames_per_launch)
    except Exception:
        return None


def main():
    args = parse()
    sys.path.insert(0, HERE)
    from ba_pathtracing_fur_amd.sharding import ShardedFrame, env_ranks

    rank, local_rank, world = env_ranks()
    dist = None
    if world > 1:
        import torch  # noqa: F401  (load torch's HIP runtime before libkirk_hip.so)
        import torch.distributed as dist

        dist.init_process_group("gloo")   # bootstrap only: the framebuffer moves over RCCL
    from ba_pathtracing_fur_amd import HipContext, scenes

    W, H, spp, depth = args.width, args.height, args.spp, args.depth
    ctx = HipContext(device=local_rank, host_build=args.host_scene)
    t0 = time.time()
    if args.host_scene:
        sd = scenes.config3(W, H, n_strands=args.strands)
        gen_s = time.time() - t0
        t0 = time.time()
        ctx.set_scene(sd)
    else:  # hairball generated and flattened in HBM
        sd = scenes.config3_device(ctx, W, H, n_strands=args.strands)
        gen_s = time.time() - t0
        t0 = time.time()
    ctx.build_accel()
    build_s = time.time() - t0
    st0 = ctx.stats()
    n_objects = st0["n_objects"]
    setup = {"path": "host" if args.host_scene else "device", "gen_s": round(gen_s, 4),
             "flatten_ms": round(st0["flatten_ms"], 2), "bvh_ms": round(st0["bvh_ms"], 2),
             "bvh_kernel_ms": round(st0["bvh_kernel_ms"], 2), "layout_ms": round(st0["layout_ms"], 2),
             "upload_ms": round(st0["upload_ms"], 2), "build_accel_s": round(build_s, 4)}
    if rank == 0:
        log(f"scene: {n_objects} objects, gen+flatten {gen_s:.3f}s, BVH+layout {build_s:.3f}s "
            f"({setup}), depth {st0['bvh_depth']}, nodes {st0['n_nodes']}, HBM {st0['device_bytes'] / 1e9:.2f} GB")
    frame = ShardedFrame(ctx, rank, world, dist, tile=args.tile)
    ext_ms_acc = []

    pipelined = not args.sync_steps

    def step(stats=False):
        # pipelined (default): the frame and its gather are enqueued and the next
        # step starts at once, so consecutive frames overlap on the device (each
        # frame alone is a chain of 2 x depth persistent launches that each wait
        # for their slowest ray); frames still complete and accumulate in order.
        frame.render(W, H, spp, depth, stats=stats, async_=pipelined and not stats)

    for _ in range(args.warmup):
        step()
    frame.sync()
    # one instrumented frame (outside the timed region): exact visit counts
    step(stats=True)
    cnt = ctx.stats()

    frame.sync()
    frame.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        if not pipelined:
            s = ctx.stats()
            ext_ms_acc.append((s["extend_ms"], s["extend_launches"], s["extend_busy_ms"]))
    frame.sync()   # every frame and gather of the timed region is complete
    frame.barrier()
    elapsed = frame.max_over_ranks(time.perf_counter() - t0)
    last = ctx.stats()   # pipelined: sums over the timed frames (khp_sync report)
    if pipelined:
        ext_ms, ext_launches, busy_ms = last["extend_ms"], last["extend_launches"], last["extend_busy_ms"]
        nfr = max(1, last["frames"])
    else:
        ext_ms = sum(a for a, _, _ in ext_ms_acc)
        ext_launches = sum(b for _, b, _ in ext_ms_acc)
        busy_ms = sum(c for _, _, c in ext_ms_acc)
        nfr = 1
    samples_per_step = W * H * spp
    value = args.steps * samples_per_step / elapsed / 1e6
    # roofline of the extend kernel (this rank's launches)
    rays = cnt["extend_rays"]
    alg_bytes_frame = 44 * rays + 32 * (cnt["node_visits"] + cnt["prim_tests"])
    launches_frame = max(1, cnt["extend_launches"])
    avg_launch_ms = ext_ms / max(1, ext_launches)
    # timed launches may carry several fused frames (KHP_FUSE_FRAMES): bytes per
    # timed launch = the frames' algorithmic bytes / the launches they took
    frames_timed = nfr if pipelined else args.steps
    bytes_per_launch = alg_bytes_frame * frames_timed / max(1, ext_launches) if ext_launches else \
        alg_bytes_frame / launches_frame
    per_launch = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    # Pipelined frames run two frames' launches side by side, so a launch's own
    # duration also counts time the chip spent on the other frame.  `achieved`
    # divides the algorithmic bytes of every timed k_extend launch by the time
    # during which at least one of them was running (union of their HIP-event
    # intervals, khp_stats.extend_busy_ms); without overlap (--sync-steps) the
    # union is the sum of the launch durations and this is bytes/launch over
    # the average launch duration.
    achieved = (bytes_per_launch * ext_launches) / (busy_ms * 1e-3) / 1e9 if busy_ms > 0 else 0.0
    traffic = pmc_traffic(frames_timed * launches_frame / max(1, ext_launches))
    out = {
        "metric": "Msamples/s at 1080p 8spp, 1M-strand hairball; achieved HBM GB/s vs peak",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: seeded hairball (khp_gen_hairball[_device], seed 0x4B49524B), scene built in-process",
        "config": {
            "workload": f"config3 scene at the metric row: {args.strands} strands ({n_objects - 2} cone frusta) "
                        f"on a 2-tri plane + 2x2 quad light, {W}x{H}, {spp} spp, depth {depth}",
            "width": W, "height": H, "spp": spp, "depth": depth, "strands": args.strands,
            "objects": n_objects, "parallelism": f"tile-sharded {args.tile}px tiles x{world}, RCCL gather",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_extend (closest-hit BVH2 traversal)",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "bytes_per_launch": int(bytes_per_launch),
            "avg_launch_ms": round(avg_launch_ms, 4),
            "achieved_per_launch": round(per_launch, 1),
            "frames_per_launch": round(frames_timed * launches_frame / max(1, ext_launches), 3),
            "alg_bytes_per_frame": int(alg_bytes_frame),
            "extend_busy_ms_per_frame": round(busy_ms / max(1, nfr if pipelined else args.steps), 3),
            "achieved_def": "algorithmic bytes of all timed k_extend launches / union of their HIP-event "
                            "intervals (= bytes per launch / avg launch duration when launches do not overlap)",
            "per_ray": {"nodes": round(cnt["node_visits"] / max(1, rays), 2),
                        "prims": round(cnt["prim_tests"] / max(1, rays), 2)},
        },
        "frame": {
            "extend_rays": rays, "shadow_rays": cnt["shadow_rays"],
            "extend_ms": round(last["extend_ms"] / nfr, 3), "shade_ms": round(last["shade_ms"] / nfr, 3),
            "shadow_ms": round(last["shadow_ms"] / nfr, 3), "other_ms": round(last["other_ms"] / nfr, 3),
            "device_ms": round(last["render_ms"] / nfr, 3),
            "shadow_nodes_per_ray": round(cnt["shadow_node_visits"] / max(1, cnt["shadow_rays"]), 2),
            "stack_spills_per_ray": round(cnt["stack_spills"] / max(1, rays + cnt["shadow_rays"]), 4),
            "pruned_pops_per_ray": round(cnt["extend_pruned_pops"] / max(1, rays), 3),
            "shadow_pruned_pops_per_ray": round(cnt["shadow_pruned_pops"] / max(1, cnt["shadow_rays"]), 3),
            "subframes": last.get("subframes"),
            "pipelined": pipelined, "fused_frames": min(args.steps, int(os.environ.get("KHP_FUSE_FRAMES", "32"))) if pipelined else 1,
            "build_s": round(build_s, 3),
            "setup": setup,
            "per_bounce": [
                {"bounce": b, "rays": cnt["bounce_rays"][b],
                 "nodes_per_ray": round(cnt["bounce_nodes"][b] / max(1, cnt["bounce_rays"][b]), 2),
                 "prims_per_ray": round(cnt["bounce_prims"][b] / max(1, cnt["bounce_rays"][b]), 2),
                 "extend_ms": round(last["bounce_extend_ms"][b] / nfr, 3),
                 "shadow_rays": cnt["bounce_shadow_rays"][b],
                 "shadow_nodes_per_ray": round(cnt["bounce_shadow_nodes"][b] / max(1, cnt["bounce_shadow_rays"][b]), 2),
                 "shadow_ms": round(last["bounce_shadow_ms"][b] / nfr, 3),
                 "wave_iters": cnt["bounce_wave_iters"][b],
                 "lane_use": round(cnt["bounce_lanes_busy"][b] / max(1, 64 * cnt["bounce_wave_iters"][b]), 3),
                 "shadow_lane_use": round(cnt["bounce_shadow_lanes_busy"][b] / max(1, 64 * cnt["bounce_shadow_wave_iters"][b]), 3)}
                for b in range(min(depth, 16))],
        },
    }
    if rank == 0:
        # output stage, outside the timed region: the device
        # 8-bit conversion and Tonemapper::map, wall time including the D2H copy of
        # W*H*4 bytes (kernel durations: profiles/*_kernel_stats.csv)
        from ba_pathtracing_fur_amd import native as N
        tm = N.Tonemap.defaults(gamma=2.2)
        o = {}
        for key, t in (("rgba8_ms", None), ("tonemap_rgba8_ms", tm)):
            ctx.read_rgba8(W, H, t)
            t1 = time.perf_counter()
            for _ in range(5):
                ctx.read_rgba8(W, H, t)
            o[key] = round((time.perf_counter() - t1) / 5 * 1e3, 3)
        o["bytes_per_pixel"] = {"rgba8": 16, "tonemap": 40}
        out["output_stage"] = o
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            # the oracle reads host arrays: the same scene generated on the host
            host_sd = sd if args.host_scene else scenes.config3(W, H, n_strands=args.strands)
            out["cpu_baseline"] = cpu_baseline(host_sd, args, args.cpu_seconds)
        except Exception as e:  # reported, never silently replaced
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        frame.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
