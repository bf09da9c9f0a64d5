"""A9 — Monte-Carlo capital supply through the C ABI (Aiyagari_VFI.m:104-129)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, d, i64, ip, lib, ptr, stream_handle


def sim_capital(policy_k, a_grid, P, z1, k1, uniforms, vfi_layout=True, return_path=False):
    """Replaces the simulation block: z_t = find(rand < cumsum(P(z_{t-1},:)),1),
    k_t = interp1(a_grid, policy_k(z_t,:), k_{t-1}, 'linear', 'extrap'); returns mean(sim_k).
    policy_k is N x Na (VFI scripts, vfi_layout=True) or Na x N (EGM scripts); z1 is 1-based
    (sim_z(1)); uniforms are the T-1 draws of `rand` (MATLAB's stream)."""
    pol = np.asfortranarray(policy_k, dtype=np.float64)
    N, Na = pol.shape if vfi_layout else pol.shape[::-1]
    a = np.ascontiguousarray(a_grid, np.float64)
    P = np.asfortranarray(P, dtype=np.float64)
    U = np.ascontiguousarray(uniforms, np.float64)
    T = U.size + 1
    out = C.c_double()
    path = np.empty(T) if return_path else None
    zpath = np.empty(T, np.int32) if return_path else None
    check(lib().aiy_sim_capital(ptr(pol), ip(1 if vfi_layout else 0), ptr(a), ptr(P), i64(N),
                                i64(Na), i64(z1), d(k1), i64(T), ptr(U), C.byref(out),
                                ptr(path), ptr(zpath)))
    if return_path:
        return out.value, path, zpath
    return out.value


def sim_capital_dev(ws, policy_rows, a_grid, P, z1, k1, uniforms, k_supply, status, sim_k=None,
                    sim_z=None, stream=None):
    """Device tier: policy_rows [N][Na], z1 0-based, outputs are device tensors."""
    T = int(uniforms.numel()) + 1
    check(lib().aiy_sim_capital_dev(ws.handle, ptr(policy_rows), ptr(a_grid), ptr(P), i64(z1),
                                    d(k1), i64(T), ptr(uniforms), ptr(k_supply), ptr(sim_k),
                                    ptr(sim_z), ptr(status), stream_handle(stream)))
