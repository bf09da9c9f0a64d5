"""F3 / F2 — the Krusell-Smith shock panel (Krusell_Smith_VFI.m:57-94) and the agent-panel
capital simulation (:206-248) through the C ABI, plus the script's outer ALM loop
(:138-296) driven from the host: VFI solve (A6/A7 on the GPU) -> panel simulation (GPU) ->
OLS of the law of motion (host, 4 numbers) -> damped B update.

The uniforms are MATLAB's `rand` stream in the script's draw order; `matlab_rand` gives the
fresh-session stream (MT19937 seed 5489, 53-bit doubles — numpy's RandomState implements the
same generator)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._capi import check, i64, lib, ptr, stream_handle


def shock_draws(T: int, population: int) -> int:
    """Uniforms consumed by :57-94: T-1 aggregate, `population` initial, (T-1)*population."""
    return (T - 1) + population + (T - 1) * population


def matlab_rand(n: int, seed: int = 5489) -> np.ndarray:
    """A fresh MATLAB session's first n `rand` values (mt19937ar, genrand_res53)."""
    return np.random.RandomState(seed).random_sample(n)


def ks_shocks(T, population, uniforms, params):
    """Replaces :57-94.  Returns zi_shock (T,) in {0 good, 1 bad} (after :68) and epsi_shock
    (T, population) in {1 employed, 2 unemployed}, as the script holds them."""
    U = np.ascontiguousarray(uniforms, np.float64)
    if U.size != shock_draws(T, population):
        raise ValueError(f"need {shock_draws(T, population)} uniforms, got {U.size}")
    prm = np.ascontiguousarray(params, np.float64)
    zi = np.empty(T)
    eps = np.empty((T, population), order="F")
    check(lib().ks_shocks(i64(T), i64(population), ptr(U), ptr(prm), ptr(zi), ptr(eps)))
    return zi, eps


def ks_simulate_capital(k_opt, k_grid, K_grid, zi_shock, epsi_shock, k_population):
    """Replaces :206-248.  k_opt k x K x 4; returns (K_ts (T,), k_population (pop,))."""
    ko = np.asfortranarray(k_opt, dtype=np.float64)
    nk, nK, nS = ko.shape
    if nS != 4:
        raise ValueError("k_opt must be k x K x 4")
    kg = np.ascontiguousarray(k_grid, np.float64)
    Kg = np.ascontiguousarray(K_grid, np.float64)
    zi = np.ascontiguousarray(zi_shock, np.float64)
    eps = np.asfortranarray(epsi_shock, dtype=np.float64)
    T, pop = eps.shape
    kp = np.array(k_population, dtype=np.float64, copy=True)
    K_ts = np.empty(T)
    check(lib().ks_simulate_capital(ptr(ko), ptr(kg), ptr(Kg), i64(nk), i64(nK), ptr(zi),
                                    ptr(eps), i64(T), i64(pop), ptr(kp), ptr(K_ts)))
    return K_ts, kp


# ------------------------------------------------------------------ device tier


def ks_shocks_dev(uniforms, params, T, population, stream=None):
    """Device tier: uniforms a cuda float64 tensor; returns (zi int8 [T], eps int8 [T][pop])."""
    import torch
    dev = uniforms.device
    if uniforms.numel() != shock_draws(T, population):
        raise ValueError("uniforms has the wrong length")
    prm = np.ascontiguousarray(params, np.float64)
    zi = torch.empty(T, dtype=torch.int8, device=dev)
    eps = torch.empty((T, population), dtype=torch.int8, device=dev)
    check(lib().ks_shocks_dev(i64(T), i64(population), ptr(uniforms), ptr(prm), ptr(zi),
                              ptr(eps), stream_handle(stream)))
    return zi, eps


class PanelSim:
    """Device-resident panel simulation: k_opt [S][K][k] (k x K x S column-major), grids,
    shocks and the population stay in HBM across calls (the population persists across ALM
    iterations, Krusell_Smith_VFI.m:101)."""

    def __init__(self, k_grid, K_grid, zi, eps, k_population):
        import torch
        self.k_grid, self.K_grid, self.zi, self.eps = k_grid, K_grid, zi, eps
        self.k_pop = k_population
        self.T, self.pop = eps.shape
        lib().ks_panel_scratch_bytes.restype = C.c_int64
        nb = int(lib().ks_panel_scratch_bytes(i64(self.pop)))
        self.scratch = torch.empty(nb // 8, dtype=torch.float64, device=k_population.device)
        self.K_ts = torch.empty(self.T, dtype=torch.float64, device=k_population.device)

    def __call__(self, k_opt, stream=None):
        """One run of :206-248 with policy k_opt (device [S][K][k]); returns K_ts (device)."""
        nS, nK, nk = k_opt.shape
        check(lib().ks_simulate_capital_dev(i64(nk), i64(nK), ptr(self.k_grid), ptr(self.K_grid),
                                            ptr(k_opt), i64(self.T), i64(self.pop), ptr(self.zi),
                                            ptr(self.eps), ptr(self.k_pop), ptr(self.K_ts),
                                            ptr(self.scratch), stream_handle(stream)))
        return self.K_ts


# ------------------------------------------------------------------ ALM loop (host)


def alm_regress(K_ts, zi_shock, T_discard=100):
    """Krusell_Smith_VFI.m:252-285: OLS of log K(t+1) on [1, log K(t)] per aggregate state,
    t = T_discard..T-1.  Host-side (4 coefficients; SURVEY C13 is out of the kernel scope).
    Returns (B_new, R2_good, R2_bad)."""
    K_ts = np.asarray(K_ts, np.float64)
    zi = np.asarray(zi_shock)
    ts = np.arange(T_discard - 1, K_ts.size - 1)
    B = np.zeros(4)
    R2 = [0.0, 0.0]
    for g in (0, 1):
        sel = ts[zi[ts] == g]
        if sel.size == 0:
            continue
        X = np.stack([np.ones(sel.size), np.log(K_ts[sel])], 1)
        Y = np.log(K_ts[sel + 1])
        Q, R = np.linalg.qr(X)
        b = np.linalg.solve(R, Q.T @ Y)
        B[2 * g:2 * g + 2] = b
        res = Y - X @ b
        R2[g] = 1 - np.sum(res ** 2) / np.sum((Y - Y.mean()) ** 2)
    return B, R2[0], R2[1]


def krusell_smith_vfi(k_size=100, K_size=4, T=1100, population=10000, max_iter_B=100, tol_B=1e-6,
                      update_B=0.3, howard_steps=50, tol_vfi=1e-6, max_vfi=10000, T_discard=100,
                      uniforms=None, n_devices=1, log=None):
    """Krusell_Smith_VFI.m:4-296 end to end on the GPU kernels: shocks (F3), then per ALM
    iteration the VFI solve (A6/A7), the panel simulation (F2) and the host regression/update.
    Returns dict(B, B_history, R2, K_ts, value, k_opt, vfi_iters)."""
    from . import calibration
    from .ks import ks_params, ks_vfi_solve
    prm = ks_params()
    kg, Kg, P, V0 = calibration.krusell_smith(k_size=k_size, K_size=K_size)
    U = matlab_rand(shock_draws(T, population)) if uniforms is None else uniforms
    zi, eps = ks_shocks(T, population, U, prm)
    value = V0
    k_opt = 0.9 * np.repeat(np.repeat(kg[:, None, None], K_size, 1), 4, 2)    # :97
    B = np.array([0.0, 1.0, 0.0, 1.0])                                          # :99
    k_pop = np.full(population, Kg[0])                                          # :101
    hist, R2, K_ts, vfi_iters = [], (0.0, 0.0), None, []
    for it in range(max_iter_B):
        R = ks_vfi_solve(value, k_opt, kg, Kg, B, P, prm, howard_steps=howard_steps, tol=tol_vfi,
                         max_vfi=max_vfi, n_devices=n_devices)
        value, k_opt = R["value"], R["k_opt"]
        vfi_iters.append(R["iters"])
        K_ts, k_pop = ks_simulate_capital(k_opt, kg, Kg, zi, eps, k_pop)
        B_new, r2g, r2b = alm_regress(K_ts, zi, T_discard)
        R2 = (r2g, r2b)
        diff_B = float(np.max(np.abs(B_new - B)))                              # :286
        hist.append(B_new.copy())
        if log:
            log(f"ALM {it + 1}: B_new={B_new} diff={diff_B:.2e} R2={R2}")
        if diff_B < tol_B:
            break
        B = update_B * B_new + (1 - update_B) * B                                # :295
    return dict(B=B, B_history=hist, R2=R2, K_ts=K_ts, value=value, k_opt=k_opt,
                vfi_iters=vfi_iters, zi=zi)
