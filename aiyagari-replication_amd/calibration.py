"""Host-side calibration (L1 of the reference scripts; not on the GPU hot path).

The kernels take P, s and a_grid as INPUTS, exactly as the reference's inner loops read
them from the workspace; these helpers only build them the way the scripts do.
"""
from __future__ import annotations

import math

import numpy as np


def linspace01(n: int) -> np.ndarray:
    """linspace(0,1,n): endpoints pinned, interior i/(n-1)."""
    if n == 1:
        return np.array([1.0])
    y = np.arange(n, dtype=np.float64) / float(n - 1)
    y[0], y[-1] = 0.0, 1.0
    return y


def _phi(x):
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


def tauchen7(rho: float, sigma_e: float):
    """Aiyagari_VFI.m:18-35: l_grid = (i-4)σe and P(i,j) = ∫ normpdf(x; ρ l_i, σe√(1-ρ²)) over
    the hard-coded interval table (:23, N = 7 only), in closed form."""
    N = 7
    l_grid = np.array([(i - 3) * sigma_e for i in range(N)])
    edges = [-math.inf] + [(k - 2.5) * sigma_e for k in range(6)] + [math.inf]
    sd = sigma_e * math.sqrt(1.0 - rho ** 2)
    P = np.zeros((N, N))
    for i in range(N):
        mu = rho * l_grid[i]
        for j in range(N):
            zl = -math.inf if edges[j] == -math.inf else (edges[j] - mu) / sd
            zh = math.inf if edges[j + 1] == math.inf else (edges[j + 1] - mu) / sd
            if zl > 0:
                up = 0.0 if zh == math.inf else 0.5 * math.erfc(zh / math.sqrt(2.0))
                P[i, j] = 0.5 * math.erfc(zl / math.sqrt(2.0)) - up
            else:
                P[i, j] = (1.0 if zh == math.inf else _phi(zh)) - (0.0 if zl == -math.inf else _phi(zl))
    return l_grid, P


def rouwenhorst(rho: float, sigma_y: float, N: int):
    """Rouwenhorst chain with unconditional std sigma_y (BASELINE config 2)."""
    p = (1.0 + rho) / 2.0
    Pm = np.array([[p, 1 - p], [1 - p, p]])
    for n in range(3, N + 1):
        Z = np.zeros((n, n))
        Z[:-1, :-1] += p * Pm
        Z[:-1, 1:] += (1 - p) * Pm
        Z[1:, :-1] += (1 - p) * Pm
        Z[1:, 1:] += p * Pm
        Z[1:-1, :] /= 2.0
        Pm = Z
    psi = math.sqrt(N - 1) * sigma_y
    return np.linspace(-psi, psi, N), Pm


def stationary(P):
    """Aiyagari_VFI.m:39-42: [P'-I; 1'] \\ [0; 1] (least squares)."""
    N = P.shape[0]
    A = np.vstack([P.T - np.eye(N), np.ones((1, N))])
    b = np.zeros(N + 1)
    b[-1] = 1.0
    return np.linalg.lstsq(A, b, rcond=None)[0]


def wage(r, alpha=0.36, delta=0.08):
    """Aiyagari_VFI.m:67."""
    return (1 - alpha) * (alpha / (r + delta)) ** (alpha / (1 - alpha))


def capital_demand(r, labor, alpha=0.36, delta=0.08):
    """Aiyagari_VFI.m:195."""
    return labor * (alpha / (r + delta)) ** (1 / (1 - alpha))


def asset_grid(Na, alpha, beta, delta, b, s1):
    """Aiyagari_VFI.m:53-58 (quadratic grid on [amin, amax])."""
    wmin = (1 - alpha) * (alpha / ((1 / beta - 1) + delta)) ** (alpha / (1 - alpha))
    amin = min(b, wmin * s1)
    kmax = delta ** (1 / (alpha - 1))
    amax = kmax ** alpha + (1 - delta) * kmax
    x = linspace01(Na)
    return amin + (amax - amin) * (x * x), amin


def aiyagari(Na=400, rho=0.75, sigma_e=0.75, beta=0.96, sigma=5.0, alpha=0.36, delta=0.08,
             b=0.0, shocks="tauchen", N=7):
    """Calibration block shared by the four Aiyagari scripts (Aiyagari_VFI.m:7-63; the labour
    scripts use rho=.6, sigma_e=.2)."""
    if shocks == "tauchen":
        l_grid, P = tauchen7(rho, sigma_e)
    elif shocks == "rouwenhorst":
        l_grid, P = rouwenhorst(rho, sigma_e, N)
    else:
        raise ValueError(shocks)
    pi = stationary(P)
    s = np.exp(l_grid)
    a_grid, amin = asset_grid(Na, alpha, beta, delta, b, s[0])
    return dict(P=P, s=s, labor=float(s @ pi), a_grid=a_grid, amin=amin, beta=beta,
                sigma=sigma, alpha=alpha, delta=delta, N=len(s), Na=Na)


def krusell_smith(k_size=100, K_size=4, K_min=30.0, K_max=50.0, beta=0.99, k_min=0.0001,
                  k_max=1000.0, ug=0.04, ub=0.10):
    """Krusell_Smith_VFI.m:5-55 and :97-98: the individual grid k_grid = x^7 scaling with
    pinned endpoints (:16-17), the aggregate grid K_grid (linspace, :20), the 4x4 transition
    matrix over s = (z, eps) built from the unemployment durations (:33-55), and the initial
    value log(0.1/0.9 k_opt0)/(1-beta) with k_opt0 = 0.9 k (:97-98).  Returns
    (k_grid, K_grid, P, V0) with V0 of shape (k, K, 4) (MATLAB's k x K x S)."""
    x = linspace01(k_size)
    k_grid = (x ** 7) * (k_max - k_min) + k_min
    k_grid[0], k_grid[-1] = k_min, k_max
    K_grid = K_min + (K_max - K_min) * linspace01(K_size)
    pgg = pbb = 1 - 1 / 8
    pgb, pbg = 1 - pgg, 1 - pbb
    p00_gg, p00_bb = 1 - 1 / 1.5, 1 - 1 / 2.5
    p00_gb, p00_bg = 1.25 * p00_bb, 0.75 * p00_gg
    p01_gg, p01_bb, p01_gb, p01_bg = 1 - p00_gg, 1 - p00_bb, 1 - p00_gb, 1 - p00_bg
    p10_gg = (ug - ug * p00_gg) / (1 - ug)
    p10_bb = (ub - ub * p00_bb) / (1 - ub)
    p10_gb = (ub - ug * p00_gb) / (1 - ug)
    p10_bg = (ug - ub * p00_bg) / (1 - ub)
    p11_gg, p11_bb, p11_gb, p11_bg = 1 - p10_gg, 1 - p10_bb, 1 - p10_gb, 1 - p10_bg
    P = np.array([[pgg * p11_gg, pgb * p11_gb, pgg * p10_gg, pgb * p10_gb],
                  [pbg * p11_bg, pbb * p11_bb, pbg * p10_bg, pbb * p10_bb],
                  [pgg * p01_gg, pgb * p01_gb, pgg * p00_gg, pgb * p00_gb],
                  [pbg * p01_bg, pbb * p01_bb, pbg * p00_bg, pbb * p00_bb]])
    k_opt0 = 0.9 * np.repeat(np.repeat(k_grid[:, None, None], K_size, 1), 4, 2)
    V0 = np.log(0.1 / 0.9 * k_opt0) / (1 - beta)
    return k_grid, K_grid, P, V0
