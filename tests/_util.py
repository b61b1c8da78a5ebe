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
    bitexact = np.array_equal(a.view(np.uint32), b.view(np.uint32))
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
