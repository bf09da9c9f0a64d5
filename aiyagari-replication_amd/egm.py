"""A4/A5 — EGM steps through the C ABI.

Arrays follow the EGM scripts' layout: policy_c is Na x N (column j = productivity state),
given here as numpy arrays of shape (Na, N) (Fortran order == the device's [N][Na])."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, d, i64, ip, lib, ptr, stream_handle


def _cm(x):
    return np.asfortranarray(x, dtype=np.float64)


def _prep(policy_c, a_grid, s, P):
    pc = np.array(policy_c, dtype=np.float64, order="F", copy=True)
    Na, N = pc.shape
    return (pc, np.ascontiguousarray(a_grid, np.float64), np.ascontiguousarray(s, np.float64),
            _cm(P), N, Na)


def egm_step(policy_c, a_grid, s, P, r, w, beta, sigma, amin):
    """Replaces one pass of Aiyagari_EGM.m:75-107 → (policy_c_next, policy_k, dist)."""
    pc, a, s, P, N, Na = _prep(policy_c, a_grid, s, P)
    out = np.empty((Na, N), order="F"); pk = np.empty((Na, N), order="F"); dist = C.c_double()
    check(lib().aiy_egm_step(ptr(pc), ptr(a), ptr(s), ptr(P), i64(N), i64(Na), d(r), d(w),
                             d(beta), d(sigma), d(amin), ptr(out), ptr(pk), C.byref(dist)))
    return out, pk, dist.value


def egm_solve(policy_c, a_grid, s, P, r, w, beta, sigma, amin, tol=1e-5, max_iter=1000):
    """Replaces Aiyagari_EGM.m:71-110 (while dist > tol && iter < max_iter)."""
    pc, a, s, P, N, Na = _prep(policy_c, a_grid, s, P)
    pk = np.empty((Na, N), order="F"); dist = C.c_double(); it = C.c_int64()
    check(lib().aiy_egm_solve(ptr(pc), ptr(a), ptr(s), ptr(P), i64(N), i64(Na), d(r), d(w),
                              d(beta), d(sigma), d(amin), d(tol), i64(max_iter), ptr(pk),
                              C.byref(dist), C.byref(it)))
    return dict(policy_c=pc, policy_k=pk, dist=dist.value, iters=it.value)


def labor_egm_step(policy_c, a_grid, s, P, r, w, beta, sigma, phi, theta, amin):
    """Replaces one pass of Aiyagari_Endogenous_Labor_EGM.m:68-104."""
    pc, a, s, P, N, Na = _prep(policy_c, a_grid, s, P)
    out = np.empty((Na, N), order="F"); pk = np.empty((Na, N), order="F")
    pl = np.empty((Na, N), order="F"); dist = C.c_double()
    check(lib().aiy_labor_egm_step(ptr(pc), ptr(a), ptr(s), ptr(P), i64(N), i64(Na), d(r), d(w),
                                   d(beta), d(sigma), d(phi), d(theta), d(amin), ptr(out),
                                   ptr(pk), ptr(pl), C.byref(dist)))
    return out, pk, pl, dist.value


def labor_egm_solve(policy_c, a_grid, s, P, r, w, beta, sigma, phi, theta, amin, tol=1e-5,
                    max_iter=1000):
    """Replaces Aiyagari_Endogenous_Labor_EGM.m:64-107."""
    pc, a, s, P, N, Na = _prep(policy_c, a_grid, s, P)
    pk = np.empty((Na, N), order="F"); pl = np.empty((Na, N), order="F")
    dist = C.c_double(); it = C.c_int64()
    check(lib().aiy_labor_egm_solve(ptr(pc), ptr(a), ptr(s), ptr(P), i64(N), i64(Na), d(r),
                                    d(w), d(beta), d(sigma), d(phi), d(theta), d(amin), d(tol),
                                    i64(max_iter), ptr(pk), ptr(pl), C.byref(dist),
                                    C.byref(it)))
    return dict(policy_c=pc, policy_k=pk, policy_l=pl, dist=dist.value, iters=it.value)


def egm_step_dev(ws, policy_c, a_grid, s, P, r, w, beta, sigma, amin, out, policy_k,
                 labor=False, phi=1.0, theta=1.0, policy_l=None, diff=None, stream=None):
    """Device tier (torch tensors [N][Na])."""
    check(lib().aiy_egm_step_dev(ws.handle, ptr(policy_c), ptr(a_grid), ptr(s), ptr(P), d(r),
                                 d(w), d(beta), d(sigma), d(amin), ip(1 if labor else 0), d(phi),
                                 d(theta), ptr(out), ptr(policy_k), ptr(policy_l), ptr(diff),
                                 stream_handle(stream)))


def egm_solve_dev(ws, policy_c, a_grid, s, P, r, w, beta, sigma, amin, tol, max_iter, policy_k,
                  labor=False, phi=1.0, theta=1.0, policy_l=None, stream=None):
    """aiy_egm_solve_dev: the solve loop on device (torch tensors [N][Na]); policy_c is
    updated in place.  Returns (iters, dist)."""
    it, dist = C.c_int64(), C.c_double()
    check(lib().aiy_egm_solve_dev(ws.handle, ptr(policy_c), ptr(a_grid), ptr(s), ptr(P), d(r),
                                  d(w), d(beta), d(sigma), d(amin), ip(1 if labor else 0),
                                  d(phi), d(theta), d(tol), i64(max_iter), ptr(policy_k),
                                  ptr(policy_l), C.byref(it), C.byref(dist),
                                  stream_handle(stream)))
    return it.value, dist.value
