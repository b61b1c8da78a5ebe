"""`bench.py --gpus 2` end to end on the CPU: the real launcher (launch_ranks ->
torch.distributed.run -> one bench.py process per rank), the gloo bootstrap,
ShardedFrame's asynchronous passes with a gather after each, max-over-ranks
timing and rank 0's gather check, with each rank's context replaced by the
oracle-backed stand-in (tests/_bench_standin.py, bench.py --ctx-factory).  The
RCCL transport itself needs >= 2 GPUs (tests/test_multigpu.py)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--config", "1", "--width", "40", "--height", "24", "--spp", "1", "--depth", "3", "--tile", "8",
        "--steps", "3", "--warmup", "1", "--sync-check-steps", "1", "--iso-steps", "1", "--gui-steps", "0",
        "--ctx-factory", "tests/_bench_standin.py:OracleBenchCtx", "--launch-timeout", "240"]


def _run(gpus, env_extra=None):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), *ARGS], cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=300)


def _line(stdout):
    return json.loads([ln for ln in stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("gpus", [2, 3])
def test_bench_gpus_n_orchestration(gpus):
    r = _run(gpus)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == gpus and line["value"] > 0 and line["steps"] == 3
    assert line["config"]["ctx_factory"].endswith("OracleBenchCtx") and line["data"].startswith("STAND-IN")
    chk = line["gather_check"]
    # warmup + instrumented pass + timed + (series start + sync-check) + isolated passes, all gathered
    assert chk["passes"] == 1 + 1 + 3 + (1 + 1) + 1 and chk["pixels"] == 40 * 24
    assert chk["bit_exact"] and chk["mismatched_pixels"] == 0


def test_bench_gather_check_fails_loudly():
    """A sender whose pixels arrive altered: the line reports the mismatch and the
    bench exits non-zero (status 3 from the rank, passed on by the launcher)."""
    r = _run(2, {"KHP_STANDIN_CORRUPT": "1"})
    assert r.returncode != 0
    line = _line(r.stdout)
    assert line["gather_check"]["bit_exact"] is False and line["gather_check"]["mismatched_pixels"] > 0
    assert "MISMATCH" in r.stderr


def test_launcher_timeout_kills_the_ranks(tmp_path):
    """launch_ranks: ranks that outlive --launch-timeout are killed, status 124."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_lt", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    stamp = tmp_path / "alive"
    script = tmp_path / "sleeper.py"
    script.write_text(f"import time, pathlib\npathlib.Path({str(stamp)!r}).write_text('x')\ntime.sleep(120)\n")

    class A:
        gpus, launch_timeout = 2, 20.0
    old = sys.argv
    sys.argv = [str(script)]
    try:
        bench.__file__ = str(script)   # the launcher starts this file per rank
        rc = bench.launch_ranks(A())
    finally:
        sys.argv = old
    assert rc == 124 and stamp.exists()
