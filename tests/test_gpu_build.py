"""Device BVH build (bvh_build.hip) vs the host build (scene.cpp).

The traversal order, and with it every closest hit, depends on the exact tree,
so the bar is identity: the same nodes in the same DFS preorder, the same
boxes bit for bit, the same leaf ranges and the same leaf-ordered object ids
as BVH::addBaseDataStructure restated on the host (CPU_BVH.cpp:16-44, 95-138,
357-552), which tests/test_host_build.py pins against the oracle.
"""
import numpy as np
import pytest

from ba_pathtracing_fur_amd import native as N
from ba_pathtracing_fur_amd import scenes as S
from ba_pathtracing_fur_amd.pathtracer import HipContext

pytestmark = pytest.mark.gpu


def _same_tree(dev: dict, host: dict):
    assert dev["depth"] == host["depth"]
    assert len(dev["boxes"]) == len(host["boxes"])
    assert np.array_equal(dev["count"], host["count"])
    assert np.array_equal(dev["first"], host["first"])
    assert np.array_equal(dev["ids"], host["ids"])
    assert np.array_equal(dev["boxes"].view(np.uint32), host["boxes"].view(np.uint32))


def _device_tree(sd, layout=False):
    ctx = HipContext(0)
    ctx.set_scene(sd)
    ctx.build_accel()
    t = ctx.read_bvh()
    st = ctx.stats()
    if layout:
        t["layout"] = ctx.read_layout()
    ctx.close()
    assert st["bvh_on_device"] == 1
    return t, st


def _host_layout(sd):
    ctx = HipContext(0, host_build=True)
    ctx.set_scene(sd)
    ctx.build_accel()
    lay = ctx.read_layout()
    ctx.close()
    return lay


def _base(n_tris=0):
    sd = S.SceneData(name="build_case")
    sd.add_material(S.material())
    sd.cam = S.camera((0, 0, 3), (0, 0, -1), (0, 1, 0), 16, 16)
    return sd


def _tris(sd, centers, size=0.01, planar=False):
    c = np.asarray(centers, np.float32)
    off = np.array([[0, 0, 0], [size, 0, 0], [0, size, 0 if planar else size]], np.float32)
    v = c[:, None, :] + off[None]
    n = np.broadcast_to(np.float32([0, 0, 1]), v.shape).copy()
    sd.add_triangles(v, n, 0)
    return sd


def _random_scene(n, seed):
    rng = np.random.default_rng(seed)
    return _tris(_base(), rng.uniform(-1, 1, (n, 3)))


CASES = {
    "one": lambda: _random_scene(1, 1),
    "two": lambda: _random_scene(2, 2),
    "three": lambda: _random_scene(3, 3),
    "small_256": lambda: _random_scene(256, 4),
    "just_level_257": lambda: _random_scene(257, 5),
    "random_50k": lambda: _random_scene(50_000, 6),
    # every centroid on one plane: the root's centroid box is flat -> one leaf of everything
    "planar_root_leaf": lambda: _tris(_base(), np.c_[np.random.default_rng(7).uniform(-1, 1, (3000, 2)),
                                                       np.zeros(3000)], planar=True),
    # a flat cluster inside a 3-D one: a large leaf made by the level phase
    "flat_cluster": lambda: _tris(_tris(_base(), np.random.default_rng(8).uniform(-1, 1, (20_000, 3))),
                                  np.c_[np.random.default_rng(9).uniform(2, 3, (1500, 2)), np.full(1500, 0.5)],
                                  planar=True),
    # many duplicated centroids (bins with everything in one place)
    "duplicates": lambda: _tris(_base(), np.repeat(np.random.default_rng(10).uniform(-1, 1, (700, 3)), 9, 0)),
    "config1": lambda: S.config1(32, 32),
    "config2": lambda: S.config2(32, 32, n_strands=2000),
    "config3_20k": lambda: S.config3(32, 32, n_strands=20_000),
    "config5_small": lambda: S.config5(32, 32, n_strands=5000, torus_grid=60, glass_subdiv=3),
    "zoo": lambda: S.zoo(32, 32),
}


@pytest.mark.parametrize("name", list(CASES))
def test_device_build_equals_host_build(name):
    sd = CASES[name]()
    dev, st = _device_tree(sd, layout=True)
    host = N.host_build(sd)
    _same_tree(dev, host)
    assert st["n_nodes"] == len(host["boxes"])
    # make_device_layout on the device: the same traversal records, bit for bit
    hl, dl = _host_layout(sd), dev["layout"]
    for k in ("nodes", "aux"):
        assert np.array_equal(dl[k], hl[k]), k
    assert np.array_equal(dl["prims"].view(np.uint32), hl["prims"].view(np.uint32))


def test_device_build_full_size():
    """The metric-row scene (1M strands, 9,000,002 objects)."""
    sd = S.config3(64, 36, n_strands=1_000_000)
    dev, st = _device_tree(sd, layout=True)
    host = N.host_build(sd)
    _same_tree(dev, host)
    hl, dl = _host_layout(sd), dev["layout"]
    for k in ("nodes", "aux"):
        assert np.array_equal(dl[k], hl[k]), k
    assert np.array_equal(dl["prims"].view(np.uint32), hl["prims"].view(np.uint32))
    print(f"device BVH build: {st['bvh_ms']:.1f} ms wall ({st['bvh_kernel_ms']:.1f} ms kernels), "
          f"layout {st['layout_ms']:.1f} ms, flatten {st['flatten_ms']:.1f} ms")


def test_host_build_flag():
    sd = S.config2(32, 32, n_strands=500)
    ctx = HipContext(0, host_build=True)
    ctx.set_scene(sd)
    ctx.build_accel()
    assert ctx.stats()["bvh_on_device"] == 0
    _same_tree(ctx.read_bvh(), N.host_build(sd))
    ctx.close()
