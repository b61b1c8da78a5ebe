"""The documented numeric definitions (DESIGN.md "kmath") against float64 references.

KIRK calls libm / MSVC CRT (sin, cos, atan2, acos, exp, sinh, _j0); both the
oracle and the kernels use the kmath restatements instead, so they must be
within a few float ulps of the true functions over the ranges the hot path
uses.  Parity between oracle and product is then bit-exact by construction.
"""
import numpy as np
import pytest

import oracle_ffi

L = oracle_ffi.load()


def ulp_err(got, want):
    got = np.float32(got)
    want = np.float64(want)
    sp = np.spacing(np.float32(abs(want))) if want != 0 else np.float32(1e-45)
    return abs(np.float64(got) - want) / np.float64(sp)


@pytest.mark.parametrize("fn,ref,lo,hi,tol", [
    ("ko_sinf", np.sin, -12.0, 12.0, 2.0),
    ("ko_cosf", np.cos, -12.0, 12.0, 2.0),
    ("ko_asinf", np.arcsin, -1.0, 1.0, 3.0),
    ("ko_acosf", np.arccos, -1.0, 1.0, 3.0),
    ("ko_expf", np.exp, -80.0, 80.0, 2.0),
    ("ko_sinhf", np.sinh, -6.0, 6.0, 3.0),
])
def test_unary_ulp(fn, ref, lo, hi, tol):
    f = getattr(L, fn)
    xs = np.linspace(lo, hi, 4001, dtype=np.float32)
    worst = max(ulp_err(f(float(x)), ref(np.float64(x))) for x in xs)
    assert worst <= tol, (fn, worst)


def test_sin_cos_absolute():
    xs = np.linspace(-12, 12, 20001, dtype=np.float32)
    s = np.array([L.ko_sinf(float(x)) for x in xs])
    c = np.array([L.ko_cosf(float(x)) for x in xs])
    assert np.max(np.abs(s - np.sin(xs.astype(np.float64)))) < 2.5e-7
    assert np.max(np.abs(c - np.cos(xs.astype(np.float64)))) < 2.5e-7


def test_atan2_quadrants():
    rng = np.random.default_rng(1)
    ys = rng.normal(size=4000).astype(np.float32)
    xs = rng.normal(size=4000).astype(np.float32)
    got = np.array([L.ko_atan2f(float(y), float(x)) for y, x in zip(ys, xs)])
    want = np.arctan2(ys.astype(np.float64), xs.astype(np.float64))
    assert np.max(np.abs(got - want)) < 5e-7
    # Cephes special cases
    assert L.ko_atan2f(0.0, 0.0) == 0.0
    assert L.ko_atan2f(1.0, 0.0) == np.float32(np.pi / 2)
    assert L.ko_atan2f(-1.0, 0.0) == -np.float32(np.pi / 2)
    assert L.ko_atan2f(0.0, -1.0) == np.float32(np.pi)


def test_exp_limits():
    assert L.ko_expf(100.0) == float("inf")
    assert L.ko_expf(-200.0) == 0.0
    assert L.ko_expf(0.0) == 1.0
    # subnormal range goes through the documented two-step ldexp
    assert 0.0 < L.ko_expf(-100.0) < 1e-40


def test_acos_domain():
    assert np.isnan(L.ko_acosf(1.0000001))
    assert L.ko_acosf(1.0) == 0.0


def test_j0_series():
    sp = pytest.importorskip("scipy.special")
    xs = np.linspace(-6.0, 6.0, 241)
    got = np.array([L.ko_j0(float(x)) for x in xs])
    assert np.max(np.abs(got - sp.j0(xs))) < 1e-12


def test_rng_known_values():
    # lowbias32-chain counter RNG (DESIGN.md "RNG"); pinned values
    vals = [L.ko_rand_u32(0x4B49524B, p, s, d) for p, s, d in [(0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1),
                                                                 (123456, 7, 19)]]
    assert len(set(vals)) == 5
    import json, os
    here = os.path.join(os.path.dirname(__file__), "golden", "rng_values.json")
    assert vals == json.load(open(here))["values"]


def test_rng_uniformity():
    u = np.array([L.ko_rand_u32(1, i, 0, 2) >> 8 for i in range(20000)], np.float64) / 2**24
    assert abs(u.mean() - 0.5) < 0.01
    assert abs(u.var() - 1 / 12) < 0.005


def _ulp64(got, want):
    if want == 0.0:
        return 0.0 if got == 0.0 else np.inf
    return abs(got - want) / np.spacing(abs(np.float64(want)))


def test_log_exp_pow_double_ulp():
    """The output stage's log / exp / pow (ko_*_d == kmath k_*_d) within 2 ulp of float64."""
    rng = np.random.default_rng(4)
    xs = np.concatenate([np.exp(rng.uniform(-700, 700, 3000)), rng.uniform(1e-6, 10, 3000), [2.3e-5, 1.0, 0.5, 2.0],
                         [5e-324, 2.2250738585072014e-308 / 3]])
    assert max(_ulp64(L.ko_log_d(float(x)), np.log(x)) for x in xs) <= 2.0
    es = np.concatenate([rng.uniform(-740, 709, 3000), rng.uniform(-1, 1, 3000), [0.0, 1.0, -1.0]])
    assert max(_ulp64(L.ko_exp_d(float(x)), np.exp(x)) for x in es if np.exp(x) > 2.2250738585072014e-308) <= 2.0
    ps = [(float(a), float(b)) for a, b in zip(rng.uniform(1e-4, 50, 2000), rng.uniform(-4, 4, 2000))]
    assert max(_ulp64(L.ko_pow_d(a, b), np.power(a, b)) for a, b in ps) <= 64.0   # |y log x| < 40: ~40 ulp worst
    for a, b in ps[:500]:   # the float overload (powf) is the double result rounded: within 1 float ulp
        assert ulp_err(np.float32(L.ko_pow_d(float(np.float32(a)), float(np.float32(b)))),
                       np.power(np.float64(np.float32(a)), np.float64(np.float32(b)))) <= 1.0


def test_pow_special_cases_c99():
    inf, nan = float("inf"), float("nan")
    cases = [((nan, 0.0), 1.0), ((1.0, nan), 1.0), ((0.0, -1.0), inf), ((-0.0, -1.0), -inf), ((-0.0, 3.0), -0.0),
             ((0.0, 0.5), 0.0), ((-1.0, inf), 1.0), ((0.5, -inf), inf), ((2.0, -inf), 0.0), ((0.5, inf), 0.0),
             ((-inf, -3.0), -0.0), ((-inf, 3.0), -inf), ((-inf, 2.0), inf), ((inf, -0.5), 0.0), ((-2.0, 3.0), -8.0),
             ((-2.0, 2.0), 4.0), ((-8.0, 1.0 / 3.0), nan), ((2.0, 10.0), 1024.0)]
    for (x, y), want in cases:
        # exp(y log x) is within a few double ulp; the float overloads the output stage uses round it exactly
        got = float(np.float32(L.ko_pow_d(x, y)))
        if np.isnan(want):
            assert np.isnan(got), (x, y)
        else:
            assert got == want and np.signbit(got) == np.signbit(want), (x, y, got)
    assert L.ko_log_d(0.0) == -inf and np.isnan(L.ko_log_d(-1.0)) and L.ko_log_d(inf) == inf
    assert L.ko_exp_d(1000.0) == inf and L.ko_exp_d(-1000.0) == 0.0 and L.ko_exp_d(0.0) == 1.0
