"""A6/A7 — Krusell-Smith VFI pieces through the C ABI (Krusell_Smith_VFI.m:143-204).
value / k_opt are k x K x S arrays exactly as in the script (column-major on the boundary)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, d, i64, ip, lib, ptr

PARAM_ORDER = ("beta", "alpha", "delta", "k_min", "k_max", "ug", "ub", "l_bar", "mu")


def ks_params(beta=0.99, alpha=0.36, delta=0.025, k_min=0.0001, k_max=1000.0, ug=0.04, ub=0.10,
              mu=0.0, z_grid=(1.01, 0.99), eps_grid=(1.0, 0.0), l_bar=None):
    """The 13-double parameter block (Krusell_Smith_VFI.m:5-13)."""
    if l_bar is None:
        l_bar = 1 / (1 - ub)
    return np.array([beta, alpha, delta, k_min, k_max, ug, ub, l_bar, mu, z_grid[0], z_grid[1],
                     eps_grid[0], eps_grid[1]], dtype=np.float64)


def _arrs(k_grid, K_grid, B, P, params):
    return (np.ascontiguousarray(k_grid, np.float64), np.ascontiguousarray(K_grid, np.float64),
            np.ascontiguousarray(B, np.float64), np.asfortranarray(P, dtype=np.float64),
            np.ascontiguousarray(params, np.float64))


def ks_policy_improve(value, k_grid, K_grid, B, P, params):
    """Replaces :149-168 → (k_opt, nfev)."""
    V = np.asfortranarray(value, dtype=np.float64)
    nk, nK, nS = V.shape
    kg, Kg, B, P, prm = _arrs(k_grid, K_grid, B, P, params)
    k_opt = np.empty_like(V, order="F")
    nfev = np.empty(V.shape, np.int32, order="F")
    check(lib().ks_policy_improve(ptr(V), ptr(kg), ptr(Kg), ptr(B), ptr(P), ptr(prm), i64(nk),
                                  i64(nK), ptr(k_opt), ptr(nfev)))
    return k_opt, nfev


def ks_howard(value, k_opt, k_grid, K_grid, B, P, params, steps=50):
    """Replaces :172-192 (Jacobi Howard sweeps with pchip refresh)."""
    V = np.array(value, dtype=np.float64, order="F", copy=True)
    nk, nK, nS = V.shape
    kg, Kg, B, P, prm = _arrs(k_grid, K_grid, B, P, params)
    ko = np.asfortranarray(k_opt, dtype=np.float64)
    check(lib().ks_howard(ptr(V), ptr(ko), ptr(kg), ptr(Kg), ptr(B), ptr(P), ptr(prm), i64(nk),
                          i64(nK), i64(steps)))
    return V


def ks_vfi_solve(value, k_opt, k_grid, K_grid, B, P, params, howard_steps=50, tol=1e-6,
                 max_vfi=10000, n_devices=1, depth=None):
    """Replaces the VFI loop :143-204 for one ALM coefficient vector B.  n_devices > 1: the
    in-process (K, Z)-sliced solve (ks_vfi_solve_sharded), `depth` Howard sweeps per exchange
    (default 4)."""
    V = np.array(value, dtype=np.float64, order="F", copy=True)
    ko = np.array(k_opt, dtype=np.float64, order="F", copy=True)
    nk, nK, nS = V.shape
    kg, Kg, B, P, prm = _arrs(k_grid, K_grid, B, P, params)
    it, rel = C.c_int64(), C.c_double()
    if depth is not None:
        check(lib().ks_vfi_solve_sharded(ptr(V), ptr(ko), ptr(kg), ptr(Kg), ptr(B), ptr(P),
                                         ptr(prm), i64(nk), i64(nK), i64(howard_steps), d(tol),
                                         i64(max_vfi), ip(n_devices), ip(depth), C.byref(it),
                                         C.byref(rel)))
    else:
        check(lib().ks_vfi_solve(ptr(V), ptr(ko), ptr(kg), ptr(Kg), ptr(B), ptr(P), ptr(prm),
                                 i64(nk), i64(nK), i64(howard_steps), d(tol), i64(max_vfi),
                                 ip(n_devices), C.byref(it), C.byref(rel)))
    return dict(value=V, k_opt=ko, iters=it.value, rel_diff=rel.value)


def ks_egm_solve(k_opt, k_grid, K_grid, B, P, params, tol=1e-6, max_iter=10000, jacobi=False):
    """A8 — replaces the EGM loop of Krusell_Smith_EGM.m:130-209 for one ALM vector B
    (Gauss-Seidel over (s, K) as the script).  jacobi=True: the F1 Jacobi variant
    (ks_egm_solve_jacobi — NOT the reference's result, all pairs of a sweep in parallel).
    Returns dict(k_opt, iters, diff)."""
    ko = np.array(k_opt, dtype=np.float64, order="F", copy=True)
    nk, nK, nS = ko.shape
    kg, Kg, B, P, prm = _arrs(k_grid, K_grid, B, P, params)
    it, diff = C.c_int64(), C.c_double()
    fn = lib().ks_egm_solve_jacobi if jacobi else lib().ks_egm_solve
    check(fn(ptr(ko), ptr(kg), ptr(Kg), ptr(B), ptr(P), ptr(prm), i64(nk), i64(nK), d(tol),
             i64(max_iter), C.byref(it), C.byref(diff)))
    return dict(k_opt=ko, iters=it.value, diff=diff.value)
