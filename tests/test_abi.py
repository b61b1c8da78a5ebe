"""The C-ABI drop-in boundary (include/kirk_hip.h): library loads, exports what the
header declares, registries mirror KIRK's factories, errors are loud.  CPU only:
no compute calls need a GPU here (khp_create is checked to *fail* without one).
"""
import ctypes
import os
import re
import subprocess
import sys

import pytest

from ba_pathtracing_fur_amd import native as N
from ba_pathtracing_fur_amd import scenes as S
from ba_pathtracing_fur_amd.pathtracer import BsdfFactory, ShaderFactory

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kirk_hip.h")


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(khp_[a-z_0-9]+)\s*\(", txt)))


def test_header_and_python_list_agree():
    assert header_functions() == sorted(N.EXPORTED)


def test_library_exports_every_symbol():
    out = subprocess.check_output(["nm", "-D", "--defined-only", N.LIB_PATH], text=True)
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing
    lib = N.load_library()
    for f in header_functions():
        assert getattr(lib, f) is not None


def test_library_is_gfx950_code_object():
    # the embedded offload bundle names its target; the build is gfx950-only
    # (host-side strings of rocPRIM's arch table name other targets; only the
    # offload-bundle target ids say which code objects are embedded)
    import re
    blob = open(N.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_abi_version():
    """The library, the header and the ctypes mirror agree (load_library refuses a
    library of another ABI: its structs would be read with the wrong layout)."""
    m = re.search(r"#define KHP_ABI_VERSION (\d+)", open(HEADER).read())
    assert N.load_library().khp_abi_version() == int(m.group(1)) == N.ABI_VERSION


def test_comm_timeout_needs_a_context_and_a_bound():
    lib = N.load_library()
    assert lib.khp_comm_set_timeout(None, 1000) == N.KHP_EINVAL
    assert b"timeout" in lib.khp_last_error()


def test_bsdf_registry_matches_kirk_factory_names():
    # BsdfFactory::getBsdf / CPU_Scene.cpp name strings (SURVEY §2 "BSDF zoo")
    lib = N.load_library()
    for i, name in enumerate(N.BSDF_NAMES):
        assert lib.khp_bsdf_kind_from_name(name.encode()) == i
        assert lib.khp_bsdf_name(i).decode() == name
        assert BsdfFactory.get_bsdf(name) == i
    assert lib.khp_bsdf_kind_from_name(b"NoSuchBSDF") == -1
    assert lib.khp_bsdf_name(99) is None
    with pytest.raises(ValueError):
        BsdfFactory.get_bsdf("NoSuchBSDF")


def test_shader_registry():
    lib = N.load_library()
    for i, name in enumerate(N.SHADER_NAMES):
        assert lib.khp_shader_kind_from_name(name.encode()) == i
        assert ShaderFactory.get_shader(name) == i
    assert lib.khp_shader_kind_from_name(b"x") == -1


def test_struct_layouts_match_header_sizes():
    # sizes implied by the header's plain-C structs (no padding surprises across the boundary)
    assert ctypes.sizeof(N.Material) == 4 * (2 + 12 + 2)
    assert ctypes.sizeof(N.Light) == 4 * (1 + 3 + 3 + 3 + 2 + 1 + 3 + 2)
    assert ctypes.sizeof(N.RenderParams) == 40
    assert ctypes.sizeof(N.Camera) == 4 * 13


def test_null_and_invalid_arguments():
    lib = N.load_library()
    assert lib.khp_host_build(None, None, None, None, None, None, None, None, None) == N.KHP_EINVAL
    assert b"null" in lib.khp_last_error()
    assert lib.khp_fibers_to_cones(1, 1, None, None, None, None) == N.KHP_EINVAL     # < 2 vertices
    sd = S.config1(8, 8)
    d = sd.desc()
    d.tri_mat[0] = 10_000                                                              # material out of range
    nn, dep = ctypes.c_uint32(), ctypes.c_uint32()
    assert lib.khp_host_build(ctypes.byref(d), ctypes.byref(nn), ctypes.byref(dep), None, None, None, None, None,
                              None) == N.KHP_EINVAL
    assert b"material" in lib.khp_last_error()


def test_create_fails_loudly_without_gpu():
    import torch  # noqa: F401  (device probing only)
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by tests/test_gpu_*.py")
    lib = N.load_library()
    ctx = ctypes.c_void_p()
    assert lib.khp_create(ctypes.byref(ctx), 0, 0) == N.KHP_EDEVICE
    assert not ctx.value
    from ba_pathtracing_fur_amd.pathtracer import HipContext
    with pytest.raises(N.KhpError):
        HipContext()


def test_missing_library_is_an_error(tmp_path):
    with pytest.raises(RuntimeError, match="not built"):
        N.load_library(str(tmp_path / "libkirk_hip.so"))


def test_product_does_not_link_the_oracle():
    out = subprocess.check_output(["ldd", N.LIB_PATH], text=True)
    assert "kirk_oracle" not in out
    import ba_pathtracing_fur_amd.pathtracer as pt
    import ba_pathtracing_fur_amd.native as nat
    src = "".join(open(m.__file__).read() for m in (pt, nat, S))
    assert "import oracle" not in src and "oracle_ffi" not in src


def test_package_exports_and_leaves_hw_queues_alone():
    """Importing the package changes no process setting: GPU_MAX_HW_QUEUES is set
    only by an explicit set_hw_queues() call of the host program."""
    code = ("import os, sys; sys.path.insert(0, %r); os.environ.pop('GPU_MAX_HW_QUEUES', None); "
            "import ba_pathtracing_fur_amd as P; [getattr(P, n) for n in P.__all__]; "
            "assert 'GPU_MAX_HW_QUEUES' not in os.environ; P.set_hw_queues(8); "
            "assert os.environ['GPU_MAX_HW_QUEUES'] == '8'") % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call([sys.executable, "-c", code])


def test_ctx_params_struct_matches_header():
    """khp_ctx_params defaults (no device needed) and the ctypes layout."""
    lib = N.load_library()
    prm = N.CtxParams()
    lib.khp_ctx_params_defaults(prm)
    assert prm.as_dict() == {"fuse_frames": 32, "frames_in_flight": 1, "chunk_paths": 0, "heavy_iters": 0xFFFFFFFF,
                             "dump_bounce": -1, "trace_kernels": 0, "shade_order": 0, "serial_stages": 0, "path_order": 1,
                             "wide_from": 2, "path_kernel": 0, "ray_sort_from": 0, "lds_nodes": 0,
                             "render_ahead": 3, "path_from": 0}
    assert ctypes.sizeof(N.CtxParams) == 64  # 15 fields: 8 + 8 + 12 x 4 bytes
