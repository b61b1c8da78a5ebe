"""bench.py host logic on the CPU: the workload each --config names (BASELINE.json
configs), the scheduling knobs it forwards to khp_ctx_params, and the host-core
count the cpu_baseline leg reports.  No GPU and no library call."""
import importlib.util
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _parse(bench, monkeypatch, *argv):
    monkeypatch.setattr(sys, "argv", ["bench.py", *argv])
    return bench.parse()


def test_metric_row_is_baseline_metric(bench, monkeypatch):
    """Default run = BASELINE.json's metric: 1080p, 8 spp, 1M strands, one GPU."""
    metric = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
    assert "1080p 8spp" in metric and "1M-strand" in metric
    a = _parse(bench, monkeypatch)
    assert (a.config, a.gpus, a.width, a.height, a.spp, a.strands, a.depth) == ("metric", 1, 1920, 1080, 8, 1_000_000, 5)
    assert a.steps > 0 and a.warmup > 0


@pytest.mark.parametrize("cfg,wh,spp,strands", [("1", (256, 256), 4, 0), ("2", (1920, 1080), 8, 10_000),
                                                ("3", (1920, 1080), 16, 1_000_000),
                                                ("5", (3840, 2160), 32, 1_000_000)])
def test_config_rows(bench, monkeypatch, cfg, wh, spp, strands):
    """--config N gives BASELINE.json configs[N-1]'s resolution, spp and strand count."""
    text = json.load(open(os.path.join(ROOT, "BASELINE.json")))["configs"][int(cfg) - 1]
    a = _parse(bench, monkeypatch, "--config", cfg)
    assert (a.width, a.height, a.spp, a.strands) == (*wh, spp, strands)
    assert f"{spp}spp" in text.replace(" ", "")


def test_explicit_sizes_override_config(bench, monkeypatch):
    a = _parse(bench, monkeypatch, "--config", "2", "--width", "64", "--height", "48", "--spp", "2", "--steps", "3")
    assert (a.width, a.height, a.spp, a.steps, a.strands) == (64, 48, 2, 3, 10_000)


def test_scheduling_knobs_parse(bench, monkeypatch):
    """Knobs map onto khp_ctx_params fields (they change scheduling, never frames)."""
    a = _parse(bench, monkeypatch, "--fuse", "16", "--frames-in-flight", "2", "--chunk-paths", "4096",
               "--shade-order", "1", "--heavy-iters", "80", "--ray-sort-from", "3")
    assert (a.fuse, a.frames_in_flight, a.chunk_paths, a.shade_order, a.heavy_iters, a.ray_sort_from) == \
        (16, 2, 4096, 1, 80, 3)
    b = _parse(bench, monkeypatch)
    assert (b.fuse, b.frames_in_flight, b.chunk_paths, b.shade_order, b.heavy_iters, b.ray_sort_from) == (None,) * 6


def test_available_cores(bench):
    n, src = bench.available_cores()
    assert 1 <= n <= len(os.sched_getaffinity(0))
    assert src in ("sched_getaffinity", "cgroup cpu.max quota")


def test_traffic_profile_matches_the_launch_shape(bench, tmp_path, monkeypatch):
    """`roofline.traffic` comes from the newest round's committed PMC profile
    whose launches carried the nearest number of fused frames, scaled to the
    run's frames per launch; config profiles are kept apart from the metric's."""
    prof = tmp_path / "profiles"
    prof.mkdir()
    def put(name, bytes_per_launch, fpl):
        (prof / f"pmc_extend_{name}.json").write_text(json.dumps(
            {"bytes_per_launch": bytes_per_launch, "frames_per_launch": fpl, "per_bounce": [{"bounce": 0}]}))
    put("r03s", 999, 10.0)          # an older round, even with the exact shape, is not taken
    put("r04a", 800, 8.0)
    put("r04b", 1000, 10.0)
    put("r04c_cfg5_", 50, 1.0)
    monkeypatch.setattr(bench, "HERE", str(tmp_path))
    assert bench._pmc_profile("metric", 10.0)[0] == "pmc_extend_r04b.json"
    assert bench._pmc_profile("metric", 8.0)[0] == "pmc_extend_r04a.json"
    assert bench.pmc_traffic(10.0, "metric") == 1000 and bench.pmc_traffic(8.0, "metric") == 800
    assert bench._pmc_profile("metric", 9.0)[0] == "pmc_extend_r04b.json"   # a tie goes to the newer profile
    assert bench._pmc_profile("5", 1.0)[0] == "pmc_extend_r04c_cfg5_.json"
    assert bench._pmc_profile("2", 1.0) == (None, None)
    assert bench.pmc_per_bounce("metric", 8.0)[0] == "pmc_extend_r04a.json"
