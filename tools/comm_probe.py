"""RCCL init with a peer that never joins (dev probe, GPU box): where does it block?
Run with KHP_LIB=variants/libkirk_commtrace.so (built with -DKHP_COMM_TRACE) under a timeout."""
import faulthandler
import os
import sys
import time

faulthandler.dump_traceback_later(40, exit=True)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ba_pathtracing_fur_amd import native as N, scenes as S  # noqa: E402
from ba_pathtracing_fur_amd.pathtracer import HipContext, comm_unique_id  # noqa: E402

ctx = HipContext(0)
ctx.set_scene(S.config2(32, 24, n_strands=100))
ctx.build_accel()
uid = comm_unique_id()
print("unique id made", flush=True)
t0 = time.time()
try:
    ctx.comm_init(2, 0, uid, timeout_ms=3000)
    print("init returned OK (unexpected)", flush=True)
except N.KhpError as e:
    print(f"init failed after {time.time() - t0:.1f} s: {e}", flush=True)
ctx.close()
print("closed", flush=True)
