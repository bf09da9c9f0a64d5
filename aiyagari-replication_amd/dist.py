"""A10 (new component) — stationary distribution by histogram iteration on the GPU."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, d, i64, ip, lib, ptr, stream_handle


def dist_stationary(a_grid, P, policy_idx=None, policy_k=None, lam0=None, tol=1e-12,
                    max_iter=10000, vfi_layout=True):
    """Iterate λ' = Pᵀ·push(λ) to a fixed point.  policy_idx: on-grid (1-based, as idx from
    Aiyagari_VFI.m:79); policy_k: off-grid (EGM) policy, mass split between bracketing nodes.
    Layout N x Na (vfi_layout) or Na x N.  Returns (lambda, K = Σ λ·a, iters, dist)."""
    a = np.ascontiguousarray(a_grid, np.float64)
    P = np.asfortranarray(P, dtype=np.float64)
    pol = policy_idx if policy_idx is not None else policy_k
    shape = np.shape(pol)
    N, Na = shape if vfi_layout else shape[::-1]
    lam = (np.full(shape, 1.0 / (N * Na)) if lam0 is None else np.array(lam0, np.float64))
    lam = np.asfortranarray(lam)
    idx = np.asfortranarray(policy_idx, np.int32) if policy_idx is not None else None
    kp = np.asfortranarray(policy_k, np.float64) if policy_idx is None else None
    K, it, dist = C.c_double(), C.c_int64(), C.c_double()
    check(lib().aiy_dist_stationary(ptr(idx), ptr(kp), ip(1 if vfi_layout else 0), ptr(a), ptr(P),
                                    i64(N), i64(Na), d(tol), i64(max_iter), ptr(lam),
                                    C.byref(K), C.byref(it), C.byref(dist)))
    return lam, K.value, it.value, dist.value


def dist_update_dev(ws, lam, a_grid, P, out, policy_idx=None, policy_k=None, diff=None,
                    stream=None):
    """One histogram push on device ([N][Na] torch tensors; policy_idx 0-based)."""
    check(lib().aiy_dist_update_dev(ws.handle, ptr(lam), ptr(policy_idx), ptr(policy_k),
                                    ptr(a_grid), ptr(P), ptr(out), ptr(diff),
                                    stream_handle(stream)))


def dist_stationary_dev(ws, lam0, a_grid, P, out, policy_idx=None, policy_k=None, tol=1e-12,
                        max_iter=10000, k_supply=None, stream=None):
    """aiy_dist_stationary_dev: the fixed point on device ([N][Na] torch tensors; policy_idx
    0-based).  `out` receives λ; k_supply (optional 1-element device tensor) Σ λ·a.
    Returns (iters, dist)."""
    it, dist = C.c_int64(), C.c_double()
    check(lib().aiy_dist_stationary_dev(ws.handle, ptr(lam0), ptr(policy_idx), ptr(policy_k),
                                        ptr(a_grid), ptr(P), d(tol), i64(max_iter), ptr(out),
                                        ptr(k_supply), C.byref(it), C.byref(dist),
                                        stream_handle(stream)))
    return it.value, dist.value
