"""F4 — inequality statistics of the reference's reporting block (Aiyagari_VFI.m:314-410; the
same block closes the three other Aiyagari scripts): Lorenz curve, Gini coefficient and wealth
quintile shares, for the simulated sample (as the scripts do) and for the histogram
stationary distribution (A10; weighted version, no reference code).

Host-side by design: these are O(n log n) passes over at most a few 10^4 numbers after the
solve (SURVEY §8(f) F4 "cheap"), evaluated in the scripts' order — MATLAB `cumsum` is a
sequential prefix sum, which numpy's cumsum reproduces; `sum`/`trapz` reduction order inside
MATLAB is unpinned (ulp-level)."""
from __future__ import annotations

import math

import numpy as np


def matlab_round(x: float) -> int:
    """MATLAB round: half away from zero (Python's round is half-to-even)."""
    return int(math.floor(abs(x) + 0.5)) * (1 if x >= 0 else -1)


def lorenz(x):
    """:317-338 — sorted sample, cumulative share cumsum(sorted)/sum(sorted) and population
    share (1:n)/n."""
    xs = np.sort(np.asarray(x, dtype=np.float64))
    n = xs.size
    cum = np.cumsum(xs) / np.sum(xs)
    pop = np.arange(1, n + 1, dtype=np.float64) / n
    return pop, cum


def trapz(x, y):
    """MATLAB trapz(x, y) for vectors: sum(diff(x) .* (y(1:end-1) + y(2:end)) / 2)."""
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    return float(np.sum(np.diff(x) * (y[:-1] + y[1:]) / 2))


def gini(x):
    """:341-352 — 1 - 2 * trapz(population share, cumulative share) (the scripts' formula;
    it omits the (0, 0) point, so a perfectly equal sample gives 1/n, not 0)."""
    pop, cum = lorenz(x)
    return 1.0 - 2.0 * trapz(pop, cum)


def quintile_shares(x):
    """:375-398 — wealth shares (%) of the five quintiles of the sorted sample, with the
    scripts' index rule q_idx = round(n * 0.2 k) (MATLAB round)."""
    xs = np.sort(np.asarray(x, dtype=np.float64))
    n = xs.size
    q = [0] + [matlab_round(n * f) for f in (0.2, 0.4, 0.6, 0.8)] + [n]
    total = float(np.sum(xs))
    return [float(np.sum(xs[q[i]:q[i + 1]])) / total * 100 for i in range(5)]


def inequality_report(sim_k, sim_c=None, sim_y=None, sim_gy=None, sim_s=None):
    """The disp lines of :354-358 and :400-404 as a dict (variables the caller has)."""
    out = {"gini_wealth": gini(sim_k), "wealth_quintile_shares": quintile_shares(sim_k)}
    for name, v in (("consumption", sim_c), ("net_income", sim_y), ("gross_income", sim_gy),
                    ("savings", sim_s)):
        if v is not None:
            out[f"gini_{name}"] = gini(v)
    return out


# ------------------------------------------------------------------ histogram (A10) version


def lorenz_weighted(values, weights):
    """Lorenz curve of a distribution with mass `weights` at `values` (e.g. the histogram
    λ(z, a) at a_j): points sorted by value (stable), cumulative population and value shares,
    starting at (0, 0)."""
    v = np.asarray(values, np.float64).ravel()
    w = np.asarray(weights, np.float64).ravel()
    o = np.argsort(v, kind="stable")
    v, w = v[o], w[o]
    pop = np.concatenate([[0.0], np.cumsum(w)]) / np.sum(w)
    cum = np.concatenate([[0.0], np.cumsum(w * v)]) / np.sum(w * v)
    return pop, cum


def gini_weighted(values, weights):
    """Gini of a weighted distribution: 1 - 2 * area under its Lorenz curve (trapezoids, from
    (0, 0)); equals the scripts' sample formula in the limit of many equal-weight points."""
    pop, cum = lorenz_weighted(values, weights)
    return 1.0 - 2.0 * trapz(pop, cum)


def quintile_shares_weighted(values, weights):
    """Value shares (%) held by the population quintiles of a weighted distribution; a point
    whose mass straddles a quintile boundary is split at it (linear in population)."""
    pop, cum = lorenz_weighted(values, weights)
    at = np.interp([0.0, 0.2, 0.4, 0.6, 0.8, 1.0], pop, cum)
    return [float(at[i + 1] - at[i]) * 100 for i in range(5)]


def histogram_wealth_stats(lam, a_grid):
    """Gini and quintile shares of wealth under the histogram stationary distribution
    λ (N x Na, mass of (z_i, a_j)), wealth = a_j."""
    lam = np.asarray(lam, np.float64)
    a = np.broadcast_to(np.asarray(a_grid, np.float64)[None, :], lam.shape)
    return {"gini_wealth": gini_weighted(a, lam),
            "wealth_quintile_shares": quintile_shares_weighted(a, lam)}
