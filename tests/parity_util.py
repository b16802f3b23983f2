"""Shared comparison helpers of the parity tests (HIP path vs the CPU oracle).

Stress-like fields (xi, sigma and the partial stresses) are ill-conditioned
where the last step changed T by almost nothing: ``1 - E(xi, lambda)`` cancels
 and xi itself is a difference of two nearly equal shift
factors, so there the reference's own value is rounding noise.  The dofs are
therefore split by the oracle's last temperature change:

* well-conditioned dofs (|T - T_prev| > ``thresh``): relative L2 error <= tol
  (1e-6, the north-star tolerance);
* the rest: not dropped, but bounded in absolute terms,
  max |got - want| <= abs_tol * max |want|;

and the fraction of well-conditioned dofs is reported (and, where the test
asks for it, required to be at least ``min_frac``).  NaN positions (xi == 0,
quirk Q5) must coincide on the well-conditioned dofs.  Elsewhere xi == 0 is
decided by rounding: where T - T_prev is ~1e-14 K on one side and exactly 0 on
the other, one side holds 0/0 = NaN and the other a finite value of the same
rounding noise, so NaN mismatches there are counted and reported, not failed.
"""
from __future__ import annotations

import numpy as np


def relerr(a, b, mask=None, scale=None):
    """relative L2 error; NaN positions must coincide.  ``mask`` restricts the
    comparison, ``scale`` (optional) replaces ||b|| in the denominator."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if mask is not None:
        a, b = a[mask], b[mask]
    na, nb = np.isnan(a), np.isnan(b)
    assert np.array_equal(na, nb), f"NaN pattern differs: {na.sum()} vs {nb.sum()}"
    a, b = a[~na], b[~nb]
    den = np.linalg.norm(b) if scale is None else scale
    if not den:
        return float(np.linalg.norm(a - b))
    return float(np.linalg.norm(a - b) / den)


def cond_mask(T_now, T_prev, src_map=None, thresh=1e-6):
    """Per-dof well-conditioned mask of the T space (|T - T_prev| > thresh) and,
    with ``src_map`` (sigma dof -> T dof), of the sigma space."""
    mT = np.abs(np.asarray(T_now) - np.asarray(T_prev)) > thresh
    mS = mT if src_map is None else mT[src_map]
    return mT, mS


def check_field(name, got, want, dof_mask, bs=1, tol=1e-6, abs_tol=1e-6, min_frac=None, scale=None):
    """Assert the split comparison described in the module docstring; returns a
    record {name, frac, rel, abs_rest} for reporting."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)
    assert got.shape == want.shape, (name, got.shape, want.shape)
    m = np.repeat(np.asarray(dof_mask, dtype=bool), bs)
    ng, nw = np.isnan(got), np.isnan(want)
    assert np.array_equal(ng[m], nw[m]), f"{name}: NaN pattern differs on well-conditioned dofs"
    nan_mismatch = int((ng != nw).sum())
    frac = float(m.mean()) if m.size else 1.0
    rel = relerr(got, want, m, scale) if m.any() else 0.0
    fin = ~nw
    wmax = float(np.abs(want[fin]).max()) if fin.any() else 0.0
    rest = (~m) & fin & ~ng
    abs_rest = float(np.abs(got[rest] - want[rest]).max()) if rest.any() else 0.0
    rec = {"name": name, "frac": frac, "rel": rel, "abs_rest": abs_rest, "max": wmax, "nan_mismatch": nan_mismatch}
    print(f"[parity] {name}: compared {frac:.1%} of dofs at rel {rel:.2e} (tol {tol:g}); "
          f"rest max abs {abs_rest:.2e} (bound {abs_tol:g} x {wmax:.3e}); "
          f"xi = 0 NaN mismatches on ill-conditioned dofs: {nan_mismatch}")
    assert rel < tol, rec
    assert abs_rest <= abs_tol * wmax + 1e-300, rec
    if min_frac is not None:
        assert frac >= min_frac, rec
    return rec
