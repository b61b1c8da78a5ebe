"""Shared test helpers: image comparison with KIRK's NaN semantics."""
import numpy as np

# Parity bar (BASELINE.json north_star): per-pixel L2 of the fp32 RGB radiance
# <= 1e-3 against the CPU reference on identical seeds.  The HIP core and the
# oracle share every float operation, so in practice the frames are identical
# bit for bit; the tolerance below is the contract, bit-exactness is checked too.
PIXEL_L2_TOL = 1e-3


def compare_images(a: np.ndarray, b: np.ndarray):
    """Returns dict(bitexact, mask_equal, max_l2, mean_l2, n_div, n_nonfinite).

    KIRK's Marschner lobe divides by sqrt(1 - sin^2(gamma)) which is 0 for
    grazing hits (Bsdf.cpp:715), so some pixels are legitimately inf/NaN; both
    sides must agree on exactly which, and L2 is measured on the finite rest.
    """
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    # NaNs compare by position, not encoding: an invalid operation yields
    # 0xFFC00000 on x86 (the oracle, and KIRK's own build) and 0x7FC00000 on
    # gfx950, and the sign of a propagated NaN follows operand order; no output
    # byte depends on it (Texture::toByte and the tonemapper map every NaN
    # alike).  Every non-NaN value must match bit for bit, and the NaNs must sit
    # in the same channels.
    na, nb = np.isnan(a), np.isnan(b)
    ua, ub = a.view(np.uint32).copy(), b.view(np.uint32).copy()
    ua[na] = 0x7FC00000
    ub[nb] = 0x7FC00000
    bitexact = np.array_equal(na, nb) and np.array_equal(ua, ub)
    fa = np.isfinite(a).all(-1)
    fb = np.isfinite(b).all(-1)
    mask_equal = np.array_equal(fa, fb)
    both = fa & fb
    d = np.linalg.norm(a[both] - b[both], axis=-1) if both.any() else np.zeros(1, np.float32)   # mask first
    return {"bitexact": bitexact, "mask_equal": mask_equal, "max_l2": float(d.max(initial=0.0)),
            "mean_l2": float(d.mean()) if d.size else 0.0, "n_div": int((d > PIXEL_L2_TOL).sum()),
            "n_nonfinite": int((~fa).sum())}


def assert_parity(a, b, exact=True):
    r = compare_images(a, b)
    assert r["mask_equal"], r
    assert r["max_l2"] <= PIXEL_L2_TOL, r
    if exact:
        assert r["bitexact"], r
    return r
