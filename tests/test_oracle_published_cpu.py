"""The restated MATLAB built-ins the Krusell-Smith rows depend on, checked against scipy's
published implementations of the same algorithms (scipy 1.15 is importable
here; MATLAB is not, so this anchors the restatement, it does not pin MATLAB itself).

* `griddedInterpolant(..., 'pchip')` (Krusell_Smith_VFI.m:133, :189) — np_oracle.pchip_slopes /
  pchip_eval against scipy.interpolate.PchipInterpolator (the same Fritsch–Butland interior rule
  and the same three-point end rule; the two evaluate the harmonic mean in different
  association orders, so agreement is to rounding).
* `fminbnd` (Krusell_Smith_VFI.m:164) — np_oracle.fminbnd (MATLAB constants: TolX 1e-4,
  seps = sqrt(eps), MaxFunEvals = MaxIter = 500) against scipy's bounded Brent minimiser
  (`scipy.optimize.minimize_scalar(method='bounded')`, a line-by-line translation of the same
  FMM routine).  scipy hard-codes sqrt(2.2e-16) where MATLAB uses sqrt(eps) = sqrt(2^-52); the
  tolerance constants are otherwise passed as MATLAB's, so the minimisers agree to TolX.

Sizes are the KS reference grid (k = 100 points, linspace^7 spacing with a first gap of
~1.1e-11, Krusell_Smith_VFI.m:16) and the scaling size's first columns.  Parity unpinned
against MATLAB; these are the published algorithms the restatement follows.
"""
import math

import numpy as np
import pytest

from oracle import np_oracle as no

scipy_interp = pytest.importorskip("scipy.interpolate")
scipy_opt = pytest.importorskip("scipy.optimize")


def _ks_columns():
    p, k_grid, K_grid, P, V0, B = no.ks_setup()
    rng = np.random.default_rng(3)
    cols = [V0[:, 0, 0], V0[:, 2, 3],                    # the script's initial value :98
            np.log(k_grid + 1.0) * 40 - 90,               # smooth concave, V-like range
            np.cumsum(rng.random(k_grid.size)),           # monotone, rough
            np.sin(k_grid / 37.0) * 10 + rng.standard_normal(k_grid.size) * 0.1]  # sign changes
    return k_grid, cols


def test_pchip_slopes_match_scipy():
    k_grid, cols = _ks_columns()
    for y in cols:
        d = no.pchip_slopes(k_grid, y)
        ds = scipy_interp.PchipInterpolator(k_grid, y).derivative()(k_grid)
        assert np.array_equal(d == 0, ds == 0)  # the same sign-change / end-rule zeros
        m = ds != 0
        assert np.max(np.abs(d[m] - ds[m]) / np.abs(ds[m])) <= 1e-15  # measured: <= 3.5e-16


def test_pchip_eval_matches_scipy():
    k_grid, cols = _ks_columns()
    rng = np.random.default_rng(5)
    xq = np.concatenate([k_grid, rng.uniform(k_grid[0], k_grid[-1], 400),
                         k_grid[:5] + 3e-12])  # the 1.1e-11-wide first segments
    for y in cols:
        d = no.pchip_slopes(k_grid, y)
        ours = np.array([no.pchip_eval(k_grid, y, d, q) for q in xq])
        ref = scipy_interp.PchipInterpolator(k_grid, y)(xq)
        tol = 1e-12 * (np.abs(y).max() + 1)
        assert np.max(np.abs(ours - ref)) <= tol


@pytest.mark.parametrize("k_i,K_i,s_i", [(0, 0, 0), (17, 1, 1), (55, 2, 2), (99, 3, 3), (80, 0, 3)])
def test_fminbnd_matches_scipy_bounded_brent(k_i, K_i, s_i):
    """One policy-improvement node of Krusell_Smith_VFI.m:157-164 on the script's initial value."""
    p, k_grid, K_grid, P, V0, B = no.ks_setup()
    dV = no.ks_slopes(k_grid, V0)
    a = p["alpha"]
    zt = p["z_grid"][0] if s_i < 2 else p["z_grid"][1]
    eps = p["eps_grid"][0] if s_i % 2 == 0 else p["eps_grid"][1]
    K = K_grid[K_i]
    L = p["l_bar"] * (1 - p["ug"] * float(zt == p["z_grid"][0]) - p["ub"] * float(zt == p["z_grid"][1]))
    wt = (1 - a) * zt * math.pow(K, a) * math.pow(L, -a)
    rt = a * zt * math.pow(K, a - 1) * math.pow(L, 1 - a)
    res = (rt + 1 - p["delta"]) * k_grid[k_i] + wt * (eps * p["l_bar"] + (1 - eps) * p["mu"])
    hi = min(res, p["k_max"])
    f = lambda x: -no.ks_bellman(p, k_grid, K_grid, V0, dV, B, P, x, k_i, K_i, s_i)
    x, fx, nf = no.fminbnd(f, p["k_min"], hi)
    r = scipy_opt.minimize_scalar(f, bounds=(p["k_min"], hi), method="bounded",
                                  options={"xatol": 1e-4, "maxiter": 500})
    assert abs(x - r.x) <= 2e-4 * max(1.0, abs(x))        # TolX-level agreement
    assert abs(fx - r.fun) <= 1e-6 * max(1.0, abs(fx))
    assert nf <= 500 and p["k_min"] <= x <= hi


def test_fminbnd_exact_on_quadratic():
    """A case both must solve to TolX: minimum of a parabola inside the bracket."""
    x, fx, nf = no.fminbnd(lambda t: (t - 3.25) ** 2, 0.0, 10.0)
    r = scipy_opt.minimize_scalar(lambda t: (t - 3.25) ** 2, bounds=(0.0, 10.0), method="bounded",
                                  options={"xatol": 1e-4})
    assert abs(x - 3.25) < 1e-4 and abs(r.x - 3.25) < 1e-4
    assert abs(x - r.x) < 1e-4


def test_fminbnd_sweep_agreement():
    """Every 7th k node of all 16 (K, s) slices: the only difference from scipy is its
    sqrt(2.2e-16) for MATLAB's sqrt(eps) in tol1, so most nodes end on the identical point and
    the rest within a tiny fraction of TolX (measured: 187 of 240 identical, max 6.5e-8)."""
    p, k, K, P, V0, B = no.ks_setup()
    dV = no.ks_slopes(k, V0)
    a = p["alpha"]
    diffs = []
    for s_i in range(4):
        for K_i in range(4):
            zt = p["z_grid"][0] if s_i < 2 else p["z_grid"][1]
            eps = p["eps_grid"][0] if s_i % 2 == 0 else p["eps_grid"][1]
            L = p["l_bar"] * (1 - p["ug"] * float(zt == p["z_grid"][0]) - p["ub"] * float(zt == p["z_grid"][1]))
            wt = (1 - a) * zt * K[K_i] ** a * L ** (-a)
            rt = a * zt * K[K_i] ** (a - 1) * L ** (1 - a)
            for k_i in range(0, 100, 7):
                hi = min((rt + 1 - p["delta"]) * k[k_i] + wt * (eps * p["l_bar"]), p["k_max"])
                f = lambda x: -no.ks_bellman(p, k, K, V0, dV, B, P, x, k_i, K_i, s_i)
                x, _, _ = no.fminbnd(f, p["k_min"], hi)
                r = scipy_opt.minimize_scalar(f, bounds=(p["k_min"], hi), method="bounded",
                                              options={"xatol": 1e-4, "maxiter": 500})
                diffs.append(abs(x - r.x))
    diffs = np.array(diffs)
    assert diffs.max() < 1e-6
    assert (diffs == 0).mean() > 0.7
