"""Committed golden fixtures (tests/golden/*.npz, made by make_golden.py).

CPU: the oracle must reproduce every stored frame and probe-ray result bit for
bit from the stored inputs (pins the oracle against drift).  GPU: the product
(libkirk_hip.so through the C-ABI) must reproduce them too.
"""
import glob
import os

import numpy as np
import pytest

from _util import assert_parity
from ba_pathtracing_fur_amd import scenes as S

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = sorted(glob.glob(os.path.join(HERE, "*.npz")))
IDS = [os.path.basename(f)[:-4] for f in FIXTURES]


def load(path):
    a = np.load(path, allow_pickle=False)
    return S.SceneData.from_arrays(a), a


def test_fixtures_present():
    assert len(FIXTURES) >= 5


@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_oracle_reproduces_fixture(path):
    import oracle_ffi
    sd, a = load(path)
    w, h, spp, depth, seed = (int(x) for x in a["params"])
    o = oracle_ffi.Oracle(sd)
    img = o.render(w, h, spp, depth, seed=seed, threads=4)
    assert np.array_equal(img.view(np.uint32), a["image"].view(np.uint32))
    t, obj, uv, nodes, prims = o.trace_closest(a["ray_orig"], a["ray_dir"])
    assert np.array_equal(obj, a["hit_obj"]) and np.array_equal(t.view(np.uint32), a["hit_t"].view(np.uint32))
    assert np.array_equal(uv.view(np.uint32), a["hit_uv"].view(np.uint32))
    assert [nodes, prims] == a["visits"].tolist()
    assert np.array_equal(o.trace_any(a["ray_orig"], a["ray_dir"], a["ray_tmax"]), a["hit_any"])


@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_fixture_scene_round_trip(path):
    sd, a = load(path)
    back = sd.to_arrays()
    for k in ("tri_v", "tri_n", "tri_mat", "cone_base_r0", "cone_apex_r1", "cone_mat", "materials", "lights",
              "camera", "env"):
        assert np.array_equal(np.asarray(back[k]), a[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_product_reproduces_fixture(path, hip_ctx):
    sd, a = load(path)
    w, h, spp, depth, seed = (int(x) for x in a["params"])
    hip_ctx.set_scene(sd)
    hip_ctx.build_accel()
    img = hip_ctx.render(w, h, spp, depth, seed=seed)
    assert_parity(img, a["image"], exact=True)
    t, obj, uv = hip_ctx.trace_closest(a["ray_orig"], a["ray_dir"])
    assert np.array_equal(obj, a["hit_obj"]) and np.array_equal(t.view(np.uint32), a["hit_t"].view(np.uint32))
    assert np.array_equal(uv.view(np.uint32), a["hit_uv"].view(np.uint32))
    assert np.array_equal(hip_ctx.trace_any(a["ray_orig"], a["ray_dir"], a["ray_tmax"]), a["hit_any"])
