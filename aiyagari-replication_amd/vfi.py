"""A1/A2 — Aiyagari VFI through the C ABI.

Host-tier wrappers mirror the MATLAB loop they replace (same inputs/outputs, MATLAB layout
semantics: arrays are (N, Na) with v[i, j] == v_old(i+1, j+1); indices returned 1-based like
`idx` in Aiyagari_VFI.m:79).  The device tier (`Workspace`) keeps everything in HBM.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, d, i64, ip, lib, ptr, stream_handle, vp


def _f(a):
    """MATLAB column-major view of an (N, Na) array (Fortran order, float64)."""
    return np.asfortranarray(a, dtype=np.float64)


def vfi_sweep(v_old, a_grid, s, P, r, w, beta, sigma):
    """Replaces Aiyagari_VFI.m:68-83: one Bellman sweep.
    Returns (v_new, policy_k, policy_c, idx) with idx 1-based."""
    v_old = _f(v_old)
    N, Na = v_old.shape
    a_grid, s = np.ascontiguousarray(a_grid, np.float64), np.ascontiguousarray(s, np.float64)
    P = _f(P)
    v_new = np.empty((N, Na), order="F"); pk = np.empty((N, Na), order="F")
    pc = np.empty((N, Na), order="F"); idx = np.empty((N, Na), np.int32, order="F")
    check(lib().aiy_vfi_sweep(ptr(v_old), ptr(a_grid), ptr(s), ptr(P), i64(N), i64(Na), d(r),
                              d(w), d(beta), d(sigma), ptr(v_new), ptr(pk), ptr(pc), ptr(idx)))
    return v_new, pk, pc, idx


def vfi_solve(v_old, a_grid, s, P, r, w, beta, sigma, tol=1e-5, max_iter=1000):
    """Replaces Aiyagari_VFI.m:65-90 (break before v_old = v_new: both are returned)."""
    v_old = np.array(v_old, dtype=np.float64, order="F", copy=True)
    N, Na = v_old.shape
    a_grid, s = np.ascontiguousarray(a_grid, np.float64), np.ascontiguousarray(s, np.float64)
    P = _f(P)
    v_new = np.empty((N, Na), order="F"); pk = np.empty((N, Na), order="F")
    pc = np.empty((N, Na), order="F"); idx = np.empty((N, Na), np.int32, order="F")
    it = C.c_int64(0)
    check(lib().aiy_vfi_solve(ptr(v_old), ptr(a_grid), ptr(s), ptr(P), i64(N), i64(Na), d(r),
                              d(w), d(beta), d(sigma), d(tol), i64(max_iter), ptr(v_new),
                              ptr(pk), ptr(pc), ptr(idx), C.byref(it)))
    return dict(v_new=v_new, v_old=v_old, policy_k=pk, policy_c=pc, idx=idx, iters=it.value)


class Workspace:
    """Device-tier handle (aiy_ws): per-shape scratch reused across sweeps.  Arrays are torch
    tensors on the current device, layout [N][Na] (z-major)."""

    def __init__(self, N: int, Na: int, Nl: int = 1):
        self.N, self.Na, self.Nl = N, Na, Nl
        h = vp()
        check(lib().aiy_ws_create(i64(N), i64(Na), i64(Nl), C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().aiy_ws_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_timing(self, on: bool, count: bool = False, trace: bool = False):
        """on: HIP-event timing of the dominant kernel; count: work counters (slows it);
        trace: per-work-item records of the tree sweep (see trace())."""
        check(lib().aiy_ws_set_timing(self._h, ip((1 if on else 0) | (2 if count else 0)
                                                  | (4 if trace else 0))))

    def trace(self):
        """Records of the last tree sweep: int64 array (items, 16) = start, end (100 MHz clock),
        XCD id, superblock tests, block tests, candidates, exact evaluations, block id, then
        wave-0 shader cycles in startup+superblock tests, block tests, fine screens, exact."""
        items = self.N * ((self.Na + 7) // 8)  # (the small-grid sweep: a record per block)
        cap = max(self.N * ((self.Na + 15) // 16), (items + 7) // 8 * 8 * 16)
        out = np.zeros((cap, 16), np.int64)
        n = C.c_int64(0)
        check(lib().aiy_ws_trace(self._h, out.ctypes.data_as(C.c_void_p), i64(cap), C.byref(n)))
        out = out[:n.value]
        return out[out[:, 1] > 0]  # items the last sweep's geometry wrote

    def trace_wide(self):
        """Records of the last small-grid sweep (bellman_wide_kernels.hip): int64 array
        (blocks, 64) = entry / end wall clock, XCD, wave 0's phase marks (cycles since entry:
        table, barrier, bar, screen, all waves, published, outputs), exact evaluations, tests,
        votes, last-arriver flag, tile, total; then per wave w at 16 + 2w: its bar and screen
        ends."""
        items = self.N * ((self.Na + 7) // 8)
        cap = (items + 7) // 8 * 8 * 16 * 4
        out = np.zeros((cap, 16), np.int64)
        n = C.c_int64(0)
        check(lib().aiy_ws_trace(self._h, out.ctypes.data_as(C.c_void_p), i64(cap), C.byref(n)))
        out = out[:n.value - n.value % 4].reshape(-1, 64)
        return out[out[:, 1] > 0]

    def timing(self):
        ms, n, hits = C.c_double(0), C.c_int64(0), C.c_int64(0)
        check(lib().aiy_ws_timing(self._h, C.byref(ms), C.byref(n), C.byref(hits)))
        return ms.value, n.value, hits.value

    def counters(self):
        """Per-state work counters of the screened sweep since set_timing(count=True):
        (exact evaluations, superblock tests, block tests, candidates screened)."""
        out = (C.c_int64 * 4)()
        check(lib().aiy_ws_counters(self._h, out))
        return tuple(int(x) for x in out)

    def invalidate(self):
        """Drop the cached feasibility table (after overwriting a_grid/s/L in place)."""
        check(lib().aiy_ws_invalidate(self._h))

    def set_variant(self, variant: int):
        """Screen-kernel geometry (tuning; results identical), see aiy_ws_set_variant."""
        check(lib().aiy_ws_set_variant(self._h, ip(variant)))

    def set_speculation(self, max_batch: int):
        """Sweeps a solve enqueues between reads of max|dv| (0/1 = one sync per sweep);
        results do not depend on it, see aiy_ws_set_speculation."""
        check(lib().aiy_ws_set_speculation(self._h, ip(max_batch)))

    def set_wide(self, max_na: int = -1, splits: int = 0, waves: int = 0, states: int = 0):
        """The small-grid one-launch sweep (aiy_ws_set_wide): used at Na <= max_na (-1: the
        default bound, 0: never) with `splits` workgroups of `waves` waves per tile of `states`
        states (0: by size).  Results do not depend on it."""
        check(lib().aiy_ws_set_wide(self._h, ip(max_na), ip(splits), ip(waves), ip(states)))

    def set_cu_exclusive(self, on: bool = True):
        """Small-grid sweep workgroups reserve whole CUs (aiy_ws_set_cu_exclusive): for solves
        running concurrently on other streams.  Results do not depend on it."""
        check(lib().aiy_ws_set_cu_exclusive(self._h, ip(int(bool(on)))))

    def set_sim(self, mode: int = -1):
        """A9 chains on this workspace (aiy_ws_set_sim): -1 by size (the speculative-segment
        chain, spread over 16 workgroups, for long chains), 0 the serial kernels, 1 the
        speculative chain in one workgroup wherever it applies, 2 the spread variant wherever it
        applies.  Results do not depend on it."""
        check(lib().aiy_ws_set_sim(self._h, ip(int(mode))))

    def set_search(self, coarse_stride=0, k_chunk=1024):
        check(lib().aiy_ws_set_search(self._h, ip(coarse_stride), ip(k_chunk)))

    def vfi_sweep(self, v_old, a_grid, s, P, r, w, beta, sigma, v_new, idx, policy_k=None,
                  policy_c=None, hint=None, mode=0, diff=None, stream=None):
        """A1 on device (asynchronous on the current torch stream)."""
        check(lib().aiy_vfi_sweep_dev(self._h, ptr(v_old), ptr(a_grid), ptr(s), ptr(P), d(r),
                                      d(w), d(beta), d(sigma), ptr(hint), ip(mode), ptr(v_new),
                                      ptr(idx), ptr(policy_k), ptr(policy_c), ptr(diff),
                                      stream_handle(stream)))

    def vfi_sweeps(self, v_a, v_b, a_grid, s, P, r, w, beta, sigma, nsweeps, idx,
                   policy_k=None, policy_c=None, hint=None, mode=0, diff=None, stream=None):
        """nsweeps A1 sweeps on device, ping-pong from v_a (v_new ends in v_b when nsweeps is
        odd); sweep 1's hint is `hint`, later sweeps use idx.  See aiy_vfi_sweeps_dev."""
        check(lib().aiy_vfi_sweeps_dev(self._h, ptr(v_a), ptr(v_b), ptr(a_grid), ptr(s), ptr(P),
                                       d(r), d(w), d(beta), d(sigma), ptr(hint), i64(nsweeps),
                                       ip(mode), ptr(idx), ptr(policy_k), ptr(policy_c),
                                       ptr(diff), stream_handle(stream)))

    def vfi_solve(self, v_a, v_b, a_grid, s, P, r, w, beta, sigma, tol, max_iter, idx,
                  policy_k=None, policy_c=None, mode=0, stream=None):
        """A2 on device; returns (iters, which) with which = 0 if v_a holds v_new else 1."""
        it, which = C.c_int64(0), C.c_int(0)
        check(lib().aiy_vfi_solve_dev(self._h, ptr(v_a), ptr(v_b), ptr(a_grid), ptr(s), ptr(P),
                                      d(r), d(w), d(beta), d(sigma), d(tol), i64(max_iter),
                                      ip(mode), ptr(idx), ptr(policy_k), ptr(policy_c),
                                      C.byref(it), C.byref(which), stream_handle(stream)))
        return it.value, which.value


def solve_batch_dev(ws, r, w, v_a, v_b, a_grid, s, P, beta, sigma, tol, max_iter, idx,
                    policy_k=None, policy_c=None, use_hint=False, stream=None):
    """Config 4 on device (aiy_vfi_solve_batch_dev): C = len(r) rates solved together; v_a/v_b,
    idx and the policies are [C][N][Na] tensors.  Returns (iters, which) as lists: candidate c
    holds v_new in v_b[c] if which[c] else v_a[c] (its v_old in the other)."""
    r = np.ascontiguousarray(r, np.float64)
    w = np.ascontiguousarray(w, np.float64)
    C = r.size
    it = np.zeros(C, np.int64)
    which = np.zeros(C, np.int32)
    check(lib().aiy_vfi_solve_batch_dev(ws.handle, i64(C), ptr(r), ptr(w), ptr(v_a), ptr(v_b),
                                        ptr(a_grid), ptr(s), ptr(P), d(beta), d(sigma), d(tol),
                                        i64(max_iter), ip(1 if use_hint else 0), ptr(idx),
                                        ptr(policy_k), ptr(policy_c), ptr(it), ptr(which),
                                        stream_handle(stream)))
    return [int(x) for x in it], [int(x) for x in which]


# ------------------------------------------------------------------------------------ A3
def _labor_call(fn, v_old, a_grid, s, P, labor_choice, r, w, beta, sigma, psi, eta, extra,
                v_new=None, pol=None):
    v_old = np.array(v_old, dtype=np.float64, order="F", copy=True)
    N, Na = v_old.shape
    L = np.ascontiguousarray(labor_choice, np.float64)
    a_grid, s = np.ascontiguousarray(a_grid, np.float64), np.ascontiguousarray(s, np.float64)
    P = _f(P)
    v_new = np.zeros((N, Na), order="F") if v_new is None else np.array(v_new, np.float64, order="F")
    if pol is None:
        pol = (np.zeros((N, Na)), np.zeros((N, Na)), np.zeros((N, Na)), np.ones((N, Na), np.int32))
    pk, pl, pc = (np.array(p, np.float64, order="F") for p in pol[:3])
    lin = np.array(pol[3], np.int32, order="F")
    out = fn(ptr(v_old), ptr(a_grid), ptr(s), ptr(P), ptr(L), i64(N), i64(Na), i64(L.size), d(r),
             d(w), d(beta), d(sigma), d(psi), d(eta), *extra(v_new, pk, pl, pc, lin))
    check(out)
    return v_old, v_new, pk, pl, pc, lin


def labor_vfi_sweep(v_old, a_grid, s, P, labor_choice, r, w, beta, sigma, psi, eta,
                    v_new=None, policies=None):
    """Replaces Aiyagari_Endogenous_Labor_VFI.m:69-112.  v_new/policies are in/out (states
    without a feasible (l, a') keep them, :85).  Returns v_new, policy_k, policy_l, policy_c,
    lin (1-based column-major index into the Nl x Na choice matrix)."""
    _, v_new, pk, pl, pc, lin = _labor_call(
        lib().aiy_labor_vfi_sweep, v_old, a_grid, s, P, labor_choice, r, w, beta, sigma, psi,
        eta, lambda vn, pk, pl, pc, lin: (ptr(vn), ptr(pk), ptr(pl), ptr(pc), ptr(lin)),
        v_new, policies)
    return v_new, pk, pl, pc, lin


def labor_vfi_solve(v_old, a_grid, s, P, labor_choice, r, w, beta, sigma, psi, eta, tol=1e-5,
                    max_iter=1000, v_new=None, policies=None):
    """Replaces Aiyagari_Endogenous_Labor_VFI.m:64-122."""
    it = C.c_int64(0)

    def extra(vn, pk, pl, pc, lin):
        return (d(tol), i64(max_iter), ptr(vn), ptr(pk), ptr(pl), ptr(pc), ptr(lin), C.byref(it))

    v_old_out, v_new, pk, pl, pc, lin = _labor_call(
        lambda *a: lib().aiy_labor_vfi_solve(*a), v_old, a_grid, s, P, labor_choice, r, w, beta,
        sigma, psi, eta, extra, v_new, policies)
    return dict(v_new=v_new, v_old=v_old_out, policy_k=pk, policy_l=pl, policy_c=pc, lin=lin,
                iters=it.value)


def _ws_labor_sweep(self, v_old, a_grid, s, P, labor_choice, r, w, beta, sigma, psi, eta, v_new,
                    lin, policy_k=None, policy_l=None, policy_c=None, hint=None, diff=None,
                    stream=None):
    """A3 on device; v_new and the policies are in/out."""
    check(lib().aiy_labor_vfi_sweep_dev(self._h, ptr(v_old), ptr(a_grid), ptr(s), ptr(P),
                                        ptr(labor_choice), d(r), d(w), d(beta), d(sigma),
                                        d(psi), d(eta), ptr(hint), ptr(v_new), ptr(lin),
                                        ptr(policy_k), ptr(policy_l), ptr(policy_c), ptr(diff),
                                        stream_handle(stream)))


Workspace.labor_vfi_sweep = _ws_labor_sweep


def _ws_labor_sweeps(self, v_a, v_b, a_grid, s, P, labor_choice, r, w, beta, sigma, psi, eta,
                     nsweeps, lin, policy_k=None, policy_l=None, policy_c=None, hint=None,
                     diff=None, stream=None):
    """nsweeps A3 sweeps on device from one C call (aiy_labor_vfi_sweeps_dev): ping-pong from
    v_a (v_new ends in v_b when nsweeps is odd), sweep 1's hint `hint`, later ones lin."""
    check(lib().aiy_labor_vfi_sweeps_dev(self._h, ptr(v_a), ptr(v_b), ptr(a_grid), ptr(s), ptr(P),
                                         ptr(labor_choice), d(r), d(w), d(beta), d(sigma), d(psi),
                                         d(eta), ptr(hint), i64(nsweeps), ptr(lin), ptr(policy_k),
                                         ptr(policy_l), ptr(policy_c), ptr(diff),
                                         stream_handle(stream)))


Workspace.labor_vfi_sweeps = _ws_labor_sweeps
