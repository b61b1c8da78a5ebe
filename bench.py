#!/usr/bin/env python3
"""Headline benchmark: Msamples/s at 1080p 8 spp on the 1M-strand hairball.

BASELINE.json metric: "Msamples/s at 1080p 8spp, 1M-strand hairball; achieved
HBM GB/s vs peak".  Default workload (--config metric) = config 3's scene (1M
strands -> 9M cone frusta on a 2-triangle plane, 2x2 quad light, sky
environment) at 1920x1080, 8 spp, depth 5 (SURVEY §8(d) "Metric row").  The
other BASELINE configs run with --config 1 | 2 | 3 | 5 (their own scene, size
and spp).

One step = one progressive pass of KIRK's PathTracer::render loop
(CPU_PathTracer.cpp:17-52) over the whole frame: step k renders samples
[k*spp, (k+1)*spp) of every pixel and folds them into the running mean, so
every step traces new samples.  Inputs (scene + BVH) are resident in HBM, the
framebuffer stays in HBM.  Steps are enqueued asynchronously (KHP_RENDER_ASYNC)
and consecutive passes with equal parameters are fused into one wavefront
(khp_ctx_params.fuse_frames, default 32); the timed region ends with khp_sync +
a barrier, so every pass is complete.  `sync_steps` in the JSON line is the
same workload with a host wait after every pass (KIRK's synchronous call):
one untimed call starts the series, then 12 calls are timed (with render-ahead
a call renders its pass and the next three as one batch and the three later calls
only accumulate, so 12 calls are 3 whole batches).

--gpus N: one process per GPU.  Under torchrun (WORLD_SIZE set) each rank
renders the 64x64 tiles t with t % N == rank and every step ends with the RCCL
framebuffer gather to rank 0; total work is fixed, so scaling is "strong".
Without WORLD_SIZE, `python bench.py --gpus N` starts those N ranks itself
(torch.distributed.run as a child process, before this process touches a GPU)
and exits with its status.

The JSON line also carries:
  roofline     -- the extend (closest-hit) kernel: algorithmic bytes
                  (28 B ray + 32 B per visited node + 32 B per
                  primitive test + 16 B hit, visit counts from an instrumented
                  pass) of all timed launches / the time during which at
                  least one of them was running (union of their HIP-event
                  intervals), against 8 TB/s HBM; roofline.shadow is the same
                  for the any-hit kernel (28 B + 32 B per node/prim + 4 B)
                  over its overlapped launches;
  isolated     -- both traversal kernels' own rates: the same fused passes
                  re-run with khp_ctx_params.serial_stages = 1 (no kernel
                  overlaps another), algorithmic bytes / kernel time;
  cpu_baseline -- the C restatement (oracle/) timed on the host cores this
                  process may use, on a bounded sample of the same frame.
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "Msamples/s at 1080p 8spp, 1M-strand hairball; achieved HBM GB/s vs peak"

# BASELINE.json configs: scene builder, width, height, spp, default steps/warmup
CONFIGS = {
    "metric": dict(scene="config3", width=1920, height=1080, spp=8, strands=1_000_000, steps=32, warmup=16,
                   what="config 3 scene at the metric row: 1M-strand hairball on a diffuse plane + 2x2 area light"),
    "1": dict(scene="config1", width=256, height=256, spp=4, strands=0, steps=64, warmup=16,
              what="config 1: Cornell box + 1 Lambert icosphere (5,120 tris)"),
    "2": dict(scene="config2", width=1920, height=1080, spp=8, strands=10_000, steps=32, warmup=16,
              what="config 2: Cornell box + 10k-strand procedural hairball (90k cones), Marschner fur"),
    "3": dict(scene="config3", width=1920, height=1080, spp=16, strands=1_000_000, steps=32, warmup=16,
              what="config 3: 1M-strand hairball on a diffuse plane + 2x2 area light, 16 spp"),
    "5": dict(scene="config5", width=3840, height=2160, spp=32, strands=1_000_000, steps=4, warmup=2,
              what="config 5: 1M-strand hairball + 500k-tri torus + glass icosphere (20,480 tris), 4K"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="metric", choices=sorted(CONFIGS))
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--strands", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--tile", type=int, default=64)
    ap.add_argument("--sync-check-steps", type=int, default=12,
                    help="passes timed with a host wait after each (the sync_steps field; 0: skip), after one "
                         "untimed call that starts the series")
    ap.add_argument("--fuse", type=int, default=None, help="khp_ctx_params.fuse_frames (default: the library's)")
    ap.add_argument("--chunk-paths", type=int, default=None, help="khp_ctx_params.chunk_paths")
    ap.add_argument("--frames-in-flight", type=int, default=None, help="khp_ctx_params.frames_in_flight")
    ap.add_argument("--gui-steps", type=int, default=12,
                    help="KIRK GUI calls timed: 1 spp per synchronous render + 8-bit texture read (0: skip)")
    ap.add_argument("--iso-steps", type=int, default=8,
                    help="fused passes re-run with serial_stages=1 for the isolated per-kernel rooflines (0: skip)")
    ap.add_argument("--shade-order", type=int, default=None, help="khp_ctx_params.shade_order (1: hits sorted by shading class)")
    ap.add_argument("--path-order", type=int, default=None,
                    help="khp_ctx_params.path_order (0: frame-major fused chunks, 1: pixel-major, 2: pixel-major heavy-first)")
    ap.add_argument("--wide-from", type=int, default=None,
                    help="khp_ctx_params.wide_from (first bounce on two-level node records; >= depth: never)")
    ap.add_argument("--ray-sort-from", type=int, default=None,
                    help="khp_ctx_params.ray_sort_from (first bounce whose rays are regrouped by origin cell; "
                         "0: automatic, >= depth: never)")
    ap.add_argument("--render-ahead", type=int, default=None,
                    help="khp_ctx_params.render_ahead (later calls of a synchronous series rendered ahead, 0..3)")
    ap.add_argument("--lds-nodes", type=int, default=None,
                    help="khp_ctx_params.lds_nodes (0 or 7: the tree's top records staged in LDS)")
    ap.add_argument("--heavy-iters", type=int, default=None,
                    help="khp_ctx_params.heavy_iters (longest-first queue threshold, traversal iterations)")
    ap.add_argument("--bdpt", default=None, metavar="PATHS,VERTICES",
                    help="light-path variant (khp_bdpt_params, SURVEY §8(f)4): not the metric's estimator")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-scene", action="store_true",
                    help="generate + flatten + build on the host (the pre-(f)1/(f)2 path) instead of in HBM")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="--gpus N without torchrun: seconds the N ranks may take before they are killed "
                         "(exit status 124)")
    ap.add_argument("--comm-timeout-ms", type=int, default=60000,
                    help="N > 1: khp_comm_set_timeout -- a lost peer or a gather without its counterpart fails "
                         "the rank (KHP_EDEVICE) after this long instead of hanging")
    ap.add_argument("--no-gather-check", action="store_true",
                    help="N > 1: skip rank 0's re-render of the untiled frame compared with the gathered one")
    ap.add_argument("--ctx-factory", default=None, metavar="FILE.py:CALLABLE",
                    help="test hook: build each rank's context with CALLABLE(device=, host_build=) from FILE.py "
                         "instead of libkirk_hip.so (tests/_bench_standin.py runs the multi-rank orchestration "
                         "on a CPU); the line is then marked as a stand-in run and measures nothing")
    a = ap.parse_args()
    cfg = CONFIGS[a.config]
    for k in ("steps", "warmup", "strands", "width", "height", "spp"):
        if getattr(a, k) is None:
            setattr(a, k, cfg[k])
    return a


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without torchrun: run N ranks as a child process group
    (no GPU has been touched in this process) and return their exit status.
    torch.distributed.run ends every rank when one fails; if the ranks together
    take longer than --launch-timeout, the whole group is killed and the status
    is 124 (a hang never outlives the bench)."""
    import signal
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log("bench: launching", " ".join(cmd))
    proc = subprocess.Popen(cmd, start_new_session=True)
    try:
        rc = proc.wait(timeout=args.launch_timeout)
    except subprocess.TimeoutExpired:
        log(f"bench: the {args.gpus} ranks did not finish within {args.launch_timeout:.0f} s; killing them")
        for sig, grace in ((signal.SIGTERM, 15), (signal.SIGKILL, 15)):
            try:
                os.killpg(proc.pid, sig)
            except ProcessLookupError:
                break
            try:
                proc.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        return 124
    if rc != 0:
        log(f"bench: the ranks exited with status {rc}")
    return rc if rc >= 0 else 128 - rc


def make_context(args, local_rank):
    """The rank's khp_ctx (pathtracer.HipContext on GPU local_rank), or the
    --ctx-factory stand-in."""
    if args.ctx_factory is None:
        from ba_pathtracing_fur_amd import HipContext
        return HipContext(device=local_rank, host_build=args.host_scene)
    import importlib.util
    path, name = args.ctx_factory.rsplit(":", 1)
    path = path if os.path.isabs(path) else os.path.join(HERE, path)
    spec = importlib.util.spec_from_file_location("bench_ctx_factory", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return getattr(mod, name)(device=local_rank, host_build=args.host_scene)


def gather_check(args, passes, gathered, scenes):
    """N > 1, rank 0: re-render the same `passes` progressive passes of the whole
    (untiled) frame on a second context of this GPU and compare them with the
    frame the ranks' tiles and RCCL gathers assembled.  Bit for bit: the counter
    RNG is keyed by pixel and sample, so tile ownership must not change a value
    (SURVEY §8(e), config 4)."""
    W, H, spp, depth = args.width, args.height, args.spp, args.depth
    t0 = time.perf_counter()
    ref_ctx = make_context(args, int(os.environ.get("LOCAL_RANK", "0")))
    try:
        build_scene(ref_ctx, args, scenes)
        ref_ctx.build_accel()
        for k in range(passes):
            ref_ctx.render(W, H, spp, depth, first_sample=k * spp, readback=False, async_=True)
        ref_ctx.sync()
        ref = ref_ctx.read_framebuffer(W, H)
    finally:
        ref_ctx.close()
    import numpy as np
    a, b = gathered.view(np.uint32), ref.view(np.uint32)
    bad = np.any(a != b, axis=-1)
    out = {"passes": passes, "pixels": W * H, "bit_exact": bool(not bad.any()), "mismatched_pixels": int(bad.sum()),
           "ms": round((time.perf_counter() - t0) * 1e3, 1),
           "def": "rank 0's gathered frame (every rank's tiles, one gather per pass) vs the same passes of the "
                  "untiled frame re-rendered on rank 0's GPU; float bits compared"}
    if bad.any():
        ys, xs = np.nonzero(bad)
        out["first_mismatch"] = {"x": int(xs[0]), "y": int(ys[0]), "gathered": gathered[ys[0], xs[0]].tolist(),
                                 "untiled": ref[ys[0], xs[0]].tolist()}
    return out


def available_cores() -> tuple[int, str]:
    """Host cores this process may use: the CPU affinity set, capped by a cgroup
    CPU quota when one is set (cpu.max), and where the figure came from."""
    n = len(os.sched_getaffinity(0))
    src = "sched_getaffinity"
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            q = max(1, math.floor(int(quota) / int(period)))
            if q < n:
                n, src = q, "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    return n, src


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(sd, args, budget_s):
    """Oracle timed on the host cores over a bounded sample of the same frame."""
    sys.path.insert(0, os.path.join(HERE, "oracle"))
    import oracle_ffi  # test infrastructure: only bench's cpu_baseline leg uses it

    threads, cores_src = available_cores()
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
            "cpu": cpu_model(), "cores_from": cores_src,
            "sample": f"{what} of the same frame = {samples} samples in {dt:.1f} s ({threads} threads = every "
                      f"core this process may use, {cpu_model()}; CPU restatement oracle/, -O3 x86-64-v3, same "
                      f"seeds); throughput is spp-linear; oracle BVH build {build_s:.1f} s excluded"}


def _pmc_profile(config: str, frames_per_launch: float | None = None):
    """The committed PMC profile of k_extend for this workload (tools/summarize_prof.py):
    among the newest round's profiles, the one whose launches carried the number of
    fused frames nearest this run's (since round 6 the driver's 20 passes: 20 per
    launch; the default 32: 16), else the newest.  Returns (file name, contents) or
    (None, None)."""
    def tag_order(f):   # r05p < r05z < r05aa: a round's tags run a..z, then aa, ab, ...
        t = os.path.basename(f)[len("pmc_extend_"):].split(".")[0].split("_")[0]
        return (t[:3], len(t), t, f)
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "pmc_extend_*.json")), key=tag_order)
    files = [f for f in files if ("_cfg" not in f) == (config == "metric") and
             (config == "metric" or f"_cfg{config}_" in f)]
    loaded = []
    for f in files:
        try:
            with open(f) as fh:
                loaded.append((os.path.basename(f), json.load(fh)))
        except Exception:
            continue
    if not loaded:
        return None, None
    rnd = lambda name: name[len("pmc_extend_"):len("pmc_extend_") + 3]   # "r04"
    newest = max(rnd(n) for n, _ in loaded)
    cands = [(n, d) for n, d in loaded if rnd(n) == newest]
    if frames_per_launch is not None:
        return min(cands, key=lambda nd: (abs(nd[1].get("frames_per_launch", 1) - frames_per_launch),
                                          -cands.index(nd)))
    return cands[-1]


def pmc_traffic(frames_per_launch: float, config: str):
    """HBM bytes per k_extend launch from the committed PMC profile of this
    workload, scaled to this run's frames per launch (the profile records how
    many fused frames its launches carried), or None."""
    name, d = _pmc_profile(config, frames_per_launch)
    try:
        return int(d["bytes_per_launch"] / d.get("frames_per_launch", 1) * frames_per_launch) if d else None
    except Exception:
        return None


def pmc_per_bounce(config: str, frames_per_launch: float | None = None):
    """Per-bounce measured / algorithmic read bytes of k_extend from the same
    committed PMC profile (tools/summarize_prof.py), or None."""
    name, d = _pmc_profile(config, frames_per_launch)
    if d and d.get("per_bounce"):
        return name, d["per_bounce"]
    return None, None


def build_scene(ctx, args, scenes):
    """The configured scene, in HBM.  The hairball of configs 3/5/metric is
    generated and flattened on the device unless --host-scene."""
    name = CONFIGS[args.config]["scene"]
    W, H = args.width, args.height
    if args.host_scene or name in ("config1", "config2"):
        kw = {} if name == "config1" else {"n_strands": args.strands}
        sd = scenes.build_config(name, width=W, height=H, **kw)
        ctx.set_scene(sd)
        return sd, "host"
    if name == "config3":
        return scenes.config3_device(ctx, W, H, n_strands=args.strands), "device"
    return scenes.config5_device(ctx, W, H, n_strands=args.strands), "device"


def host_scene_for_oracle(sd, args, scenes):
    name = CONFIGS[args.config]["scene"]
    if args.host_scene or name in ("config1", "config2"):
        return sd
    kw = {"n_strands": args.strands}
    return scenes.build_config(name, width=args.width, height=args.height, **kw)


def main():
    args = parse()
    sys.path.insert(0, HERE)
    from ba_pathtracing_fur_amd.sharding import ShardedFrame, env_ranks

    rank, local_rank, world = env_ranks()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if world != args.gpus:
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; the line reports the {world} ranks that ran")
    dist = None
    if world > 1:
        import torch  # noqa: F401  (load torch's HIP runtime before libkirk_hip.so)
        import torch.distributed as dist

        dist.init_process_group("gloo")   # bootstrap only: the framebuffer moves over RCCL
    from ba_pathtracing_fur_amd import scenes

    W, H, spp, depth = args.width, args.height, args.spp, args.depth
    ctx = make_context(args, local_rank)
    t0 = time.time()
    sd, path = build_scene(ctx, args, scenes)
    gen_s = time.time() - t0
    t0 = time.time()
    ctx.build_accel()
    build_s = time.time() - t0
    st0 = ctx.stats()
    n_objects = st0["n_objects"]
    setup = {"path": path, "gen_s": round(gen_s, 4),
             "flatten_ms": round(st0["flatten_ms"], 2), "bvh_ms": round(st0["bvh_ms"], 2),
             "bvh_kernel_ms": round(st0["bvh_kernel_ms"], 2), "layout_ms": round(st0["layout_ms"], 2),
             "upload_ms": round(st0["upload_ms"], 2), "build_accel_s": round(build_s, 4)}
    if rank == 0:
        log(f"scene: {n_objects} objects, gen+flatten {gen_s:.3f}s, BVH+layout {build_s:.3f}s "
            f"({setup}), depth {st0['bvh_depth']}, nodes {st0['n_nodes']}, HBM {st0['device_bytes'] / 1e9:.2f} GB")
    frame = ShardedFrame(ctx, rank, world, dist, tile=args.tile, unique_id=getattr(ctx, "comm_unique_id", None),
                         comm_timeout_ms=args.comm_timeout_ms if world > 1 else None)
    knobs = {k: v for k, v in (("fuse_frames", args.fuse), ("chunk_paths", args.chunk_paths),
                               ("frames_in_flight", args.frames_in_flight), ("shade_order", args.shade_order),
                               ("heavy_iters", args.heavy_iters), ("path_order", args.path_order),
                               ("wide_from", args.wide_from), ("ray_sort_from", args.ray_sort_from),
                               ("lds_nodes", args.lds_nodes), ("render_ahead", args.render_ahead))
             if v is not None}
    if knobs:
        ctx.set_params(**knobs)
    params = ctx.params()
    if args.bdpt:
        ns, nv = (int(x) for x in args.bdpt.split(","))
        ctx.set_bdpt(enabled=1, light_paths=ns, vertices=nv)
        params["bdpt"] = {"light_paths": ns, "vertices": nv}
    k = 0  # progressive pass counter: pass k renders samples [k*spp, (k+1)*spp)

    def step(stats=False, async_=True):
        nonlocal k
        frame.render(W, H, spp, depth, first_sample=k * spp, stats=stats, async_=async_ and not stats)
        k += 1

    for _ in range(args.warmup):
        step()
    frame.sync()
    # one instrumented pass (outside the timed region): exact visit counts
    step(stats=True)
    cnt = ctx.stats()

    frame.sync()
    frame.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    frame.sync()   # every pass and gather of the timed region is complete
    frame.barrier()
    elapsed = frame.max_over_ranks(time.perf_counter() - t0)
    last = ctx.stats()   # sums over the timed passes (khp_sync report)
    ext_ms, ext_launches, busy_ms = last["extend_ms"], last["extend_launches"], last["extend_busy_ms"]
    nfr = max(1, last["frames"])
    samples_per_step = W * H * spp
    value = args.steps * samples_per_step / elapsed / 1e6

    # the same workload with a host wait after every pass (no fusion, no overlap)
    sync_line = None
    if args.sync_check_steps > 0:
        step(async_=False)   # the series' first call (untimed): render-ahead starts with the second
        frame.sync()
        frame.barrier()
        calls, ahead = [], []
        t1 = time.perf_counter()
        for _ in range(args.sync_check_steps):
            tc = time.perf_counter()
            step(async_=False)
            ahead.append(ctx.stats()["ahead_finished"])   # before khp_sync opens a new report
            frame.sync()
            calls.append(round((time.perf_counter() - tc) * 1e3, 3))
        frame.barrier()
        sync_el = frame.max_over_ranks(time.perf_counter() - t1)
        sync_line = {"value": round(args.sync_check_steps * samples_per_step / sync_el / 1e6, 3),
                     "ms_per_step": round(sync_el / args.sync_check_steps * 1e3, 3), "steps": args.sync_check_steps,
                     "call_ms": calls, "paths_finished_ahead": ahead,
                     "def": "one synchronous khp_render per pass (+ gather), consecutive first_sample, after one "
                            "untimed call; synchronous renders run the path kernel up to 14 x 2^20 paths per call "
                            f"and the wavefront above (khp_ctx_params.path_kernel = {params['path_kernel']}, "
                            f"0 = automatic), render_ahead = {params.get('render_ahead', 0)} (a wavefront call "
                            "that continues the series renders its pass and the next render_ahead passes as one "
                            "fused batch; those calls only accumulate: call_ms, paths_finished_ahead)"}

    # KIRK's GUI pattern (CPU_PathTracer.cpp:17-52): every
    # render() call adds ONE sample to every pixel synchronously and the viewer
    # then reads the 8-bit texture (drawTexture -> Texture::setPixel)
    gui_line = None
    if args.gui_steps > 0 and rank == 0 and world == 1:
        for g in range(2):   # the series' first calls (render-ahead fills up), untimed
            ctx.render(W, H, 1, depth, first_sample=k * spp + g, readback=False)
            ctx.read_rgba8(W, H)
        calls, ahead = [], []
        t1 = time.perf_counter()
        for g in range(args.gui_steps):
            tc = time.perf_counter()
            ctx.render(W, H, 1, depth, first_sample=k * spp + 2 + g, readback=False)
            ctx.read_rgba8(W, H)
            calls.append(round((time.perf_counter() - tc) * 1e3, 3))
            st_g = ctx.stats()
            ahead.append(st_g["ahead_finished"])
        gui_el = time.perf_counter() - t1
        gui_line = {"value": round(args.gui_steps * W * H / gui_el / 1e6, 3),
                    "ms_per_call": round(gui_el / args.gui_steps * 1e3, 3), "calls": args.gui_steps,
                    "call_ms": calls, "paths_finished_ahead": ahead,
                    "def": "KIRK GUI render() calls: one synchronous khp_render of 1 spp + khp_read_rgba8 "
                           "(8-bit texture to the host) per call, consecutive first_sample; synchronous renders run "
                           f"the path kernel (khp_ctx_params.path_kernel = {params['path_kernel']}, 0 = automatic) "
                           f"with render_ahead = {params.get('render_ahead', 0)} (a call's drain starts the paths of "
                           "the next calls; each call returns when its own paths end; call_ms: each call, "
                           "paths_finished_ahead: its paths found finished by earlier calls)"}
        k += (args.gui_steps + 2 + spp - 1) // spp   # those samples belong to the pass slots after the last timed one
        # the same calls pipelined (ABI 8): render() enqueues its 1-spp pass and an
        # asynchronous texture read, the viewer shows textures as they complete;
        # consecutive passes fuse, each texture is taken between two accumulates
        import numpy as np
        n_async = max(args.gui_steps, 32)
        bufs = [np.zeros((H, W, 4), np.uint8) for _ in range(4)]
        s0 = k * spp
        frame.sync()
        t1 = time.perf_counter()
        for g in range(n_async):
            ctx.render(W, H, 1, depth, first_sample=s0 + g, async_=True)
            ctx.read_rgba8_async(bufs[g % 4])   # a viewer's rotating textures
        ctx.sync()
        ga_el = time.perf_counter() - t1
        k += (n_async + spp - 1) // spp
        gui_line["pipelined"] = {"value": round(n_async * W * H / ga_el / 1e6, 3),
                                 "ms_per_call": round(ga_el / n_async * 1e3, 3), "calls": n_async,
                                 "def": "the same calls with KHP_RENDER_ASYNC + khp_read_rgba8_async (ABI 8): "
                                        "1-spp passes fused, every pass's 8-bit texture delivered"}

    # the same fused passes with the shadow stage on the extend stream (serial_stages):
    # no two kernels overlap, so each kernel's HIP-event time is its own -- the
    # isolated per-kernel rooflines (k_shadow's overlapped launch time above also
    # counts the co-running k_extend's share of the chip)
    iso_st = None
    if args.iso_steps > 0:
        old_prm = ctx.set_params(serial_stages=1)
        for _ in range(args.iso_steps):
            step()
        frame.sync()
        iso_st = ctx.stats()
        ctx.set_params(**old_prm)

    # roofline of the extend kernel (this rank's launches)
    rays = cnt["extend_rays"]
    alg_bytes_frame = 44 * rays + 32 * (cnt["node_visits"] + cnt["prim_tests"])
    launches_frame = max(1, cnt["extend_launches"])
    avg_launch_ms = ext_ms / max(1, ext_launches)
    # timed launches carry several fused passes: bytes per timed launch = the
    # passes' algorithmic bytes / the launches they took
    bytes_per_launch = alg_bytes_frame * nfr / max(1, ext_launches)
    per_launch = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    achieved = (bytes_per_launch * ext_launches) / (busy_ms * 1e-3) / 1e9 if busy_ms > 0 else 0.0
    frames_per_launch = nfr * launches_frame / max(1, ext_launches)
    traffic = None if args.bdpt else pmc_traffic(frames_per_launch, args.config)  # profiles are of the default estimator
    # per bounce: this run's algorithmic rate (exact visit counts, HIP-event launch
    # times) next to the measured/algorithmic read ratio of the committed profile
    prof_name, prof_pb = (None, None) if args.bdpt else pmc_per_bounce(args.config, frames_per_launch)
    per_bounce_rl = []
    for b in range(min(depth, 16)):
        r_b = cnt["bounce_rays"][b]
        if not r_b:
            continue
        alg_b = 44 * r_b + 32 * (cnt["bounce_nodes"][b] + cnt["bounce_prims"][b])
        ms_b = last["bounce_extend_ms"][b] / nfr
        row = {"bounce": b, "alg_GB_per_frame": round(alg_b / 1e9, 3), "ms_per_frame": round(ms_b, 3),
               "alg_TBps": round(alg_b / (ms_b * 1e-3) / 1e12, 3) if ms_b > 0 else None}
        pr = next((x for x in (prof_pb or []) if x["bounce"] == b), None)
        if pr:
            row["profile_read_over_alg"] = pr["measured_over_alg"]
            row["profile_read_TBps"] = pr["measured_TBps"]
        per_bounce_rl.append(row)
    # the any-hit kernel (k_shadow alone; the finish is a separate streaming kernel)
    sh_rays = cnt["shadow_rays"]
    sh_bytes_frame = 32 * sh_rays + 32 * (cnt["shadow_node_visits"] + cnt["shadow_prim_tests"])
    sh_ms = last["shadow_ms"] - last["shadow_finish_ms"]
    sh_launches = max(1, last["shadow_launches"])
    sh_bytes_per_launch = sh_bytes_frame * nfr / sh_launches
    sh_avg_ms = sh_ms / sh_launches
    sh_achieved = sh_bytes_per_launch / (sh_avg_ms * 1e-3) / 1e9 if sh_avg_ms > 0 else 0.0
    isolated = None
    if iso_st is not None:
        nfi = max(1, iso_st["frames"])
        e_ms, s_ms = iso_st["extend_ms"], iso_st["shadow_ms"] - iso_st["shadow_finish_ms"]

        def _rl(bytes_frame, ms, launches):
            a = bytes_frame * nfi / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            return {"ms_per_frame": round(ms / nfi, 3), "launches": launches, "achieved": round(a, 1),
                    "frac": round(a / HBM_PEAK_GBPS, 4)}
        isolated = {
            "frames": nfi, "def": "the same fused progressive passes with khp_ctx_params.serial_stages = 1 "
                                  "(one stream: no kernel overlaps another); algorithmic bytes / kernel time",
            "device_ms_per_frame": round(iso_st["render_ms"] / nfi, 3),
            "k_extend": _rl(alg_bytes_frame, e_ms, iso_st["extend_launches"]),
            "k_shadow": _rl(sh_bytes_frame, s_ms, iso_st["shadow_launches"]),
            "k_shade_ms_per_frame": round(iso_st["shade_ms"] / nfi, 3),
            "k_shadow_finish_ms_per_frame": round(iso_st["shadow_finish_ms"] / nfi, 3),
        }
        isolated["k_shadow"]["records_per_s"] = round(
            (cnt["shadow_node_visits"] + cnt["shadow_prim_tests"]) * nfi / max(1e-9, s_ms * 1e-3), 1)
        isolated["k_extend"]["records_per_s"] = round(
            (cnt["node_visits"] + cnt["prim_tests"]) * nfi / max(1e-9, e_ms * 1e-3), 1)
    # N > 1: rank 0's gathered frame against the untiled frame of the same passes
    check = None
    if world > 1 and not args.no_gather_check:
        frame.sync()
        if rank == 0:
            check = gather_check(args, k, ctx.read_framebuffer(W, H), scenes)
            log(f"bench: gather check over {k} passes: {'bit-exact' if check['bit_exact'] else 'MISMATCH'} "
                f"({check['mismatched_pixels']} pixels differ)")
        frame.barrier()
    cfg = CONFIGS[args.config]
    out = {
        "metric": METRIC if args.config == "metric" else f"Msamples/s, {cfg['what']}, {W}x{H} {spp}spp",
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
        "data": "synthetic: seeded hairball (khp_gen_hairball[_device], seed 0x4B49524B), scene built in-process; "
                "step k = progressive pass k (samples k*spp .. (k+1)*spp-1)",
        "config": {
            "workload": f"{cfg['what']} ({n_objects} objects), {W}x{H}, {spp} spp, depth {depth}, progressive passes"
                        + (f", light-path variant {args.bdpt}" if args.bdpt else ""),
            "config": args.config, "width": W, "height": H, "spp": spp, "depth": depth, "strands": args.strands,
            "objects": n_objects, "parallelism": f"tile-sharded {args.tile}px tiles x{world}, RCCL gather",
        },
        "gather_check": check,
        "sync_steps": sync_line,
        "gui_steps": gui_line,
        "isolated": isolated,
        "roofline": {
            "bound": "hbm",
            "kernel": "k_extend (closest-hit traversal: bounce-0, 64-B and two-level instances together)",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "bytes_per_launch": int(bytes_per_launch),
            "avg_launch_ms": round(avg_launch_ms, 4),
            "achieved_per_launch": round(per_launch, 1),
            "frames_per_launch": round(frames_per_launch, 3),
            "alg_bytes_per_frame": int(alg_bytes_frame),
            "extend_busy_ms_per_frame": round(busy_ms / nfr, 3),
            "achieved_def": "algorithmic bytes of all timed k_extend launches / union of their HIP-event "
                            "intervals (= bytes per launch / avg launch duration when launches do not overlap)",
            "per_ray": {"nodes": round(cnt["node_visits"] / max(1, rays), 2),
                        "prims": round(cnt["prim_tests"] / max(1, rays), 2)},
            "per_bounce": per_bounce_rl,
            "per_bounce_def": "alg = SURVEY §8(d) bytes of the bounce's exact visit counts; ms = the bounce's "
                              "k_extend launches (HIP events) per frame; profile_read_* = 2 x FETCH_SIZE of "
                              f"the bounce's launches in {prof_name} (L2 misses, Infinity-Cache hits included)",
            "shadow": {
                "kernel": "k_shadow (any-hit BVH2 traversal)",
                "achieved_def": "algorithmic bytes per launch / average launch duration of the overlapped "
                                "launches, which share the chip with the next bounce's k_extend; the "
                                "kernel's own rate is isolated.k_shadow",
                "achieved": round(sh_achieved, 1), "frac": round(sh_achieved / HBM_PEAK_GBPS, 4),
                "bytes_per_launch": int(sh_bytes_per_launch), "avg_launch_ms": round(sh_avg_ms, 4),
                "alg_bytes_per_frame": int(sh_bytes_frame),
                "per_ray": {"nodes": round(cnt["shadow_node_visits"] / max(1, sh_rays), 2),
                            "prims": round(cnt["shadow_prim_tests"] / max(1, sh_rays), 2)},
                "records_per_s": round((cnt["shadow_node_visits"] + cnt["shadow_prim_tests"]) * nfr /
                                       max(1e-9, sh_ms * 1e-3), 1),
            },
        },
        "frame": {
            "extend_rays": rays, "shadow_rays": sh_rays,
            "extend_ms": round(last["extend_ms"] / nfr, 3), "shade_ms": round(last["shade_ms"] / nfr, 3),
            "shadow_ms": round(last["shadow_ms"] / nfr, 3),
            "shadow_finish_ms": round(last["shadow_finish_ms"] / nfr, 3),
            "other_ms": round(last["other_ms"] / nfr, 3),
            "device_ms": round(last["render_ms"] / nfr, 3),
            "extend_records_per_s": round((cnt["node_visits"] + cnt["prim_tests"]) * nfr / max(1e-9, ext_ms * 1e-3), 1),
            "stack_spills_per_ray": round(cnt["stack_spills"] / max(1, rays + sh_rays), 4),
            "pruned_pops_per_ray": round(cnt["extend_pruned_pops"] / max(1, rays), 3),
            "shadow_pruned_pops_per_ray": round(cnt["shadow_pruned_pops"] / max(1, sh_rays), 3),
            "fused_frames": min(args.steps, params["fuse_frames"]), "params": params,
            "build_s": round(build_s, 3),
            "setup": setup,
            "per_bounce": [
                {"bounce": b, "rays": cnt["bounce_rays"][b],
                 "nodes_per_ray": round(cnt["bounce_nodes"][b] / max(1, cnt["bounce_rays"][b]), 2),
                 "prims_per_ray": round(cnt["bounce_prims"][b] / max(1, cnt["bounce_rays"][b]), 2),
                 "extend_ms": round(last["bounce_extend_ms"][b] / nfr, 3),
                 "shadow_rays": cnt["bounce_shadow_rays"][b],
                 "shadow_nodes_per_ray": round(cnt["bounce_shadow_nodes"][b] / max(1, cnt["bounce_shadow_rays"][b]), 2),
                 "shadow_prims_per_ray": round(cnt["bounce_shadow_prims"][b] / max(1, cnt["bounce_shadow_rays"][b]), 2),
                 "shadow_ms": round(last["bounce_shadow_ms"][b] / nfr, 3),
                 "wave_iters": cnt["bounce_wave_iters"][b],
                 "lane_use": round(cnt["bounce_lanes_busy"][b] / max(1, 64 * cnt["bounce_wave_iters"][b]), 3),
                 "shadow_lane_use": round(cnt["bounce_shadow_lanes_busy"][b] /
                                          max(1, 64 * cnt["bounce_shadow_wave_iters"][b]), 3)}
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
            out["cpu_baseline"] = cpu_baseline(host_scene_for_oracle(sd, args, scenes), args, args.cpu_seconds)
        except Exception as e:  # reported, never silently replaced
            out["cpu_baseline"] = {"error": repr(e)}
    if args.ctx_factory is not None:
        out["data"] = f"STAND-IN RUN ({args.ctx_factory}): orchestration test, the numbers measure nothing"
        out["config"]["ctx_factory"] = args.ctx_factory
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        frame.barrier()
        dist.destroy_process_group()
    ctx.close()
    if check is not None and not check["bit_exact"]:
        log("bench: the gathered frame differs from the untiled frame; exiting with status 3")
        sys.exit(3)


if __name__ == "__main__":
    main()
