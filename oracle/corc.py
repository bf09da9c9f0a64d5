"""ctypes wrapper over oracle/liborc.so (the C restatement).  TEST INFRASTRUCTURE ONLY —
used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
Parity against MATLAB: unpinned (see oracle/aiy_oracle.h)."""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB = None

_d = C.c_double
_i64 = C.c_int64
_P = C.c_void_p


def lib():
    global _LIB
    if _LIB is None:
        path = _HERE / "liborc.so"
        if not path.exists():
            raise RuntimeError(f"{path} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = C.CDLL(str(path))
        for name in ("orc_vfi_sweep", "orc_vfi_solve", "orc_labor_vfi_sweep", "orc_labor_vfi_solve",
                     "orc_egm_step", "orc_egm_solve", "orc_labor_egm_step", "orc_labor_egm_solve",
                     "orc_sim_capital", "orc_dist_update_ongrid", "orc_dist_update_lottery",
                     "orc_ks_policy_improve", "orc_ks_howard", "orc_ks_egm_solve", "orc_num_threads",
                     "orc_ks_egm_solve_jacobi",
                     "orc_dist_stationary"):
            getattr(L, name).restype = C.c_int
        L.orc_ks_bellman.restype = _d
        L.orc_pchip_eval.restype = _d
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(_P)


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def num_threads(n=0):
    return lib().orc_num_threads(C.c_int(n))


# ---------------------------------------------------------------- A1/A2
def vfi_sweep(v_old, a_grid, s, P, r, w, beta, sigma):
    v_old, a_grid, s, P = map(f64, (v_old, a_grid, s, P))
    N, Na = v_old.shape
    v_new = np.empty((N, Na)); pk = np.empty((N, Na)); pc = np.empty((N, Na))
    idx = np.empty((N, Na), np.int32)
    rc = lib().orc_vfi_sweep(_i64(N), _i64(Na), _p(v_old), _p(a_grid), _p(s), _p(P), _d(r), _d(w),
                             _d(beta), _d(sigma), _p(v_new), _p(idx), _p(pk), _p(pc))
    assert rc == 0
    return v_new, idx, pk, pc


def vfi_solve(v_old, a_grid, s, P, r, w, beta, sigma, tol=1e-5, max_iter=1000):
    v_old = f64(v_old).copy()
    a_grid, s, P = map(f64, (a_grid, s, P))
    N, Na = v_old.shape
    v_new = np.empty((N, Na)); pk = np.empty((N, Na)); pc = np.empty((N, Na))
    idx = np.empty((N, Na), np.int32)
    it = _i64(0)
    rc = lib().orc_vfi_solve(_i64(N), _i64(Na), _p(v_old), _p(a_grid), _p(s), _p(P), _d(r), _d(w),
                             _d(beta), _d(sigma), _d(tol), _i64(max_iter), _p(v_new), _p(idx),
                             _p(pk), _p(pc), C.byref(it))
    assert rc == 0
    return dict(v_new=v_new, v_old=v_old, idx=idx, policy_k=pk, policy_c=pc, iters=it.value)


# ---------------------------------------------------------------- A3
def labor_vfi_sweep(v_old, a_grid, s, P, L, r, w, beta, sigma, psi, eta, v_new=None, pol=None):
    v_old, a_grid, s, P, L = map(f64, (v_old, a_grid, s, P, L))
    N, Na = v_old.shape
    v_new = np.zeros((N, Na)) if v_new is None else f64(v_new).copy()
    if pol is None:
        pol = (np.zeros((N, Na)), np.zeros((N, Na)), np.zeros((N, Na)), np.zeros((N, Na), np.int32))
    pk, pl, pc, lin = (f64(pol[0]).copy(), f64(pol[1]).copy(), f64(pol[2]).copy(),
                       np.ascontiguousarray(pol[3], np.int32).copy())
    rc = lib().orc_labor_vfi_sweep(_i64(N), _i64(Na), _i64(L.size), _p(v_old), _p(a_grid), _p(s),
                                   _p(P), _p(L), _d(r), _d(w), _d(beta), _d(sigma), _d(psi),
                                   _d(eta), _p(v_new), _p(pk), _p(pl), _p(pc), _p(lin))
    assert rc == 0
    return v_new, (pk, pl, pc, lin)


def labor_vfi_solve(v_old, a_grid, s, P, L, r, w, beta, sigma, psi, eta, tol=1e-5, max_iter=1000):
    v_old = f64(v_old).copy()
    a_grid, s, P, L = map(f64, (a_grid, s, P, L))
    N, Na = v_old.shape
    v_new = np.zeros((N, Na)); pk = np.zeros((N, Na)); pl = np.zeros((N, Na)); pc = np.zeros((N, Na))
    lin = np.zeros((N, Na), np.int32)
    it = _i64(0)
    rc = lib().orc_labor_vfi_solve(_i64(N), _i64(Na), _i64(L.size), _p(v_old), _p(a_grid), _p(s),
                                   _p(P), _p(L), _d(r), _d(w), _d(beta), _d(sigma), _d(psi),
                                   _d(eta), _d(tol), _i64(max_iter), _p(v_new), _p(pk), _p(pl),
                                   _p(pc), _p(lin), C.byref(it))
    assert rc == 0
    return dict(v_new=v_new, v_old=v_old, policy_k=pk, policy_l=pl, policy_c=pc, lin=lin,
                iters=it.value)


# ---------------------------------------------------------------- A4/A5 (arrays [N][Na])
def egm_step(pc, a_grid, s, P, r, w, beta, sigma, amin):
    pc, a_grid, s, P = map(f64, (pc, a_grid, s, P))
    N, Na = pc.shape
    pcn = np.empty((N, Na)); pk = np.empty((N, Na)); dist = _d(0)
    rc = lib().orc_egm_step(_i64(N), _i64(Na), _p(pc), _p(a_grid), _p(s), _p(P), _d(r), _d(w),
                            _d(beta), _d(sigma), _d(amin), _p(pcn), _p(pk), C.byref(dist))
    assert rc == 0
    return pcn, pk, dist.value


def egm_solve(pc, a_grid, s, P, r, w, beta, sigma, amin, tol=1e-5, max_iter=1000):
    pc = f64(pc).copy()
    a_grid, s, P = map(f64, (a_grid, s, P))
    N, Na = pc.shape
    pk = np.zeros((N, Na)); dist = _d(0); it = _i64(0)
    rc = lib().orc_egm_solve(_i64(N), _i64(Na), _p(pc), _p(a_grid), _p(s), _p(P), _d(r), _d(w),
                             _d(beta), _d(sigma), _d(amin), _d(tol), _i64(max_iter), _p(pk),
                             C.byref(dist), C.byref(it))
    assert rc == 0
    return dict(policy_c=pc, policy_k=pk, dist=dist.value, iters=it.value)


def labor_egm_step(pc, a_grid, s, P, r, w, beta, sigma, phi, theta, amin):
    pc, a_grid, s, P = map(f64, (pc, a_grid, s, P))
    N, Na = pc.shape
    pcn = np.empty((N, Na)); pk = np.empty((N, Na)); pl = np.empty((N, Na)); dist = _d(0)
    rc = lib().orc_labor_egm_step(_i64(N), _i64(Na), _p(pc), _p(a_grid), _p(s), _p(P), _d(r),
                                  _d(w), _d(beta), _d(sigma), _d(phi), _d(theta), _d(amin),
                                  _p(pcn), _p(pk), _p(pl), C.byref(dist))
    assert rc == 0
    return pcn, pk, pl, dist.value


def labor_egm_solve(pc, a_grid, s, P, r, w, beta, sigma, phi, theta, amin, tol=1e-5,
                    max_iter=1000):
    pc = f64(pc).copy()
    a_grid, s, P = map(f64, (a_grid, s, P))
    N, Na = pc.shape
    pk = np.zeros((N, Na)); pl = np.zeros((N, Na)); dist = _d(0); it = _i64(0)
    rc = lib().orc_labor_egm_solve(_i64(N), _i64(Na), _p(pc), _p(a_grid), _p(s), _p(P), _d(r),
                                   _d(w), _d(beta), _d(sigma), _d(phi), _d(theta), _d(amin),
                                   _d(tol), _i64(max_iter), _p(pk), _p(pl), C.byref(dist),
                                   C.byref(it))
    assert rc == 0
    return dict(policy_c=pc, policy_k=pk, policy_l=pl, dist=dist.value, iters=it.value)


# ---------------------------------------------------------------- A9
def sim_capital(policy, a_grid, P, z1, k1, uniforms, layout="vfi", return_path=False):
    """policy: [N][Na] array of policy_k rows (both layouts are [N][Na] in this wrapper)."""
    policy, a_grid, P, U = map(f64, (policy, a_grid, P, uniforms))
    N, Na = policy.shape
    T = U.size + 1
    mean = _d(0)
    path = np.empty(T) if return_path else None
    rc = lib().orc_sim_capital(_i64(N), _i64(Na), _p(policy), _i64(Na), _i64(1), _p(a_grid), _p(P),
                               _i64(z1), _d(k1), _i64(T), _p(U), C.byref(mean),
                               _p(path) if path is not None else None)
    if rc != 0:
        raise ValueError(f"orc_sim_capital failed rc={rc}")
    return (mean.value, path) if return_path else mean.value


# ---------------------------------------------------------------- A10
def dist_update_ongrid(lam, idx, P):
    lam, P = f64(lam), f64(P)
    idx = np.ascontiguousarray(idx, np.int32)
    N, Na = lam.shape
    out = np.empty((N, Na))
    assert lib().orc_dist_update_ongrid(_i64(N), _i64(Na), _p(lam), _p(idx), _p(P), _p(out)) == 0
    return out


def dist_update_lottery(lam, kp, a_grid, P):
    lam, kp, a_grid, P = map(f64, (lam, kp, a_grid, P))
    N, Na = lam.shape
    out = np.empty((N, Na))
    assert lib().orc_dist_update_lottery(_i64(N), _i64(Na), _p(lam), _p(kp), _p(a_grid), _p(P),
                                         _p(out)) == 0
    return out


def dist_stationary(lam, a_grid, P, idx=None, kp=None, tol=1e-12, max_iter=10000):
    lam = f64(lam).copy()
    a_grid, P = f64(a_grid), f64(P)
    N, Na = lam.shape
    K, it, dist = _d(0), _i64(0), _d(0)
    idx_p = _p(np.ascontiguousarray(idx, np.int32)) if idx is not None else None
    if idx is not None:
        idx_arr = np.ascontiguousarray(idx, np.int32); idx_p = _p(idx_arr)
    kp_arr = f64(kp) if kp is not None else None
    rc = lib().orc_dist_stationary(_i64(N), _i64(Na), idx_p, _p(kp_arr) if kp_arr is not None else None,
                                   _p(a_grid), _p(P), _d(tol), _i64(max_iter), _p(lam), C.byref(K),
                                   C.byref(it), C.byref(dist))
    assert rc == 0
    return lam, K.value, it.value, dist.value


# ---------------------------------------------------------------- A6/A7
class KSParams(C.Structure):
    _fields_ = [("beta", _d), ("alpha", _d), ("delta", _d), ("k_min", _d), ("k_max", _d),
                ("ug", _d), ("ub", _d), ("l_bar", _d), ("mu", _d), ("z_grid", _d * 2),
                ("eps_grid", _d * 2)]


def ks_params(**kw):
    p = KSParams()
    for k, v in kw.items():
        if k in ("z_grid", "eps_grid"):
            getattr(p, k)[0], getattr(p, k)[1] = v
        else:
            setattr(p, k, v)
    return p


def ks_policy_improve(p, k_grid, K_grid, V, B, P):
    k_grid, K_grid, B, P = map(f64, (k_grid, K_grid, B, P))
    V = np.asfortranarray(V, dtype=np.float64)  # k x K x S column-major
    nk, nK, nS = V.shape
    k_opt = np.empty((nk, nK, nS), order="F")
    nfev = np.empty((nk, nK, nS), np.int32, order="F")
    rc = lib().orc_ks_policy_improve(C.byref(p), _i64(nk), _i64(nK), _p(k_grid), _p(K_grid),
                                     V.ctypes.data_as(_P), _p(B), _p(P), None,
                                     k_opt.ctypes.data_as(_P), nfev.ctypes.data_as(_P))
    assert rc == 0
    return k_opt, nfev


def ks_howard(p, k_grid, K_grid, V, k_opt, B, P, steps):
    k_grid, K_grid, B, P = map(f64, (k_grid, K_grid, B, P))
    V = np.array(V, dtype=np.float64, order="F", copy=True)
    k_opt = np.asfortranarray(k_opt, dtype=np.float64)
    nk, nK, nS = V.shape
    rc = lib().orc_ks_howard(C.byref(p), _i64(nk), _i64(nK), _p(k_grid), _p(K_grid),
                             V.ctypes.data_as(_P), k_opt.ctypes.data_as(_P), _p(B), _p(P),
                             _i64(steps))
    assert rc == 0
    return V


def ks_vfi_solve(p, k_grid, K_grid, V, k_opt, B, P, howard=50, tol=1e-6, max_vfi=10000):
    """Krusell_Smith_VFI.m:143-204 with the C pieces (improve every 5th iteration)."""
    V = np.array(V, dtype=np.float64, order="F", copy=True)
    k_opt = np.array(k_opt, dtype=np.float64, order="F", copy=True)
    rel = float("nan")
    it = 0
    for it in range(1, max_vfi + 1):
        V_old = V.copy(order="F")
        if (it - 1) % 5 == 0:
            k_opt, _ = ks_policy_improve(p, k_grid, K_grid, V, B, P)
        V = ks_howard(p, k_grid, K_grid, V, k_opt, B, P, howard)
        d = np.abs(V - V_old) / (np.abs(V_old) + 1e-10)
        rel = float(np.nanmax(d)) if not np.all(np.isnan(d)) else float("nan")
        if rel < tol:
            break
    return dict(value=V, k_opt=k_opt, iters=it, rel_diff=rel)


# ---------------------------------------------------------------- A8
def ks_egm_solve(p, k_grid, K_grid, B, P, k_opt, tol=1e-6, max_iter=10000, jacobi=False):
    """Krusell_Smith_EGM.m:130-209 (C restatement).  P is MATLAB's 4x4 (row s_i)."""
    k_grid, K_grid, B = map(f64, (k_grid, K_grid, B))
    Pr = np.ascontiguousarray(P, dtype=np.float64)
    ko = np.array(k_opt, dtype=np.float64, order="F", copy=True)
    nk, nK, _ = ko.shape
    it, diff = C.c_int64(), C.c_double()
    rc = (lib().orc_ks_egm_solve_jacobi if jacobi else lib().orc_ks_egm_solve)(C.byref(p), _i64(nk), _i64(nK), _p(k_grid), _p(K_grid), _p(B),
                                _p(Pr), _d(tol), _i64(max_iter), ko.ctypes.data_as(_P),
                                C.byref(it), C.byref(diff))
    if rc:
        raise ValueError(f"orc_ks_egm_solve rc={rc}")
    return dict(k_opt=ko, iters=it.value, diff=diff.value)
