"""A11 — the general-equilibrium bisection on r that drives the hot path (host side, like the
reference scripts' L4 loop), for all four Aiyagari scripts:

  aiyagari_vfi          Aiyagari_VFI.m:63-206
  aiyagari_labor_vfi    Aiyagari_Endogenous_Labor_VFI.m:59-256
  aiyagari_egm          Aiyagari_EGM.m:58-253     (w frozen at r = 0.04 inside the loop, :61)
  aiyagari_labor_egm    Aiyagari_Endogenous_Labor_EGM.m:54-251 (same quirk, :55)

Each: initial solve at r = 0.04 → Monte-Carlo capital supply (MATLAB's fresh-session rand
stream: randi(N), randi(Na), then 9,999 draws per simulation) → 10 bisection steps on
[-0.05, 1/beta - 1], warm-starting the solver, restarting the chain from the same (z1, k1).
Every solve and every simulation runs on the GPU through the C ABI.  With supply="histogram"
the Monte-Carlo estimator is replaced by K = Σ λ·a at the stationary histogram (A10, new).
"""
from __future__ import annotations

import math
import time

import numpy as np

from . import calibration as cb
from .dist import dist_stationary
from .egm import egm_solve, labor_egm_solve
from .sim import sim_capital
from .vfi import labor_vfi_solve, vfi_solve


def matlab_rand(n: int, seed: int = 5489) -> np.ndarray:
    """MATLAB's `rand` stream in a fresh session: MT19937 seeded 5489, 53-bit doubles."""
    return np.random.RandomState(seed).random_sample(n)


class _Stream:
    def __init__(self, T, steps):
        self.u = matlab_rand(2 + (T - 1) * (steps + 1))
        self.pos = 0

    def take(self, n):
        out = self.u[self.pos:self.pos + n]
        self.pos += n
        return out


def _bisect(cal, solve_at, supply_of, max_r_iter=10, r_tol=1e-5):
    """Aiyagari_VFI.m:133-206: r_mid each step, K_d = labor (alpha/(r+delta))^(1/(1-alpha))."""
    r_low, r_high = -0.05, 1 / cal["beta"] - 1
    out = dict(r_history=[], k_supply=[], k_demand=[], iters=[])
    r = math.nan
    for _ in range(max_r_iter):
        r_guess = (r_low + r_high) / 2
        r = r_guess
        it = solve_at(r)
        Ks = supply_of()
        Kd = cb.capital_demand(r_guess, cal["labor"], cal["alpha"], cal["delta"])
        out["r_history"].append(r); out["k_supply"].append(Ks); out["k_demand"].append(Kd)
        out["iters"].append(it)
        if abs(Ks - Kd) < r_tol:
            break
        elif Ks > Kd:
            r_high = r_guess
        else:
            r_low = r_guess
    out["r"] = r
    return out


def aiyagari_vfi(Na=400, rho=0.75, sigma_e=0.75, shocks="tauchen", T=10000, tol=1e-5,
                 max_iter=1000, supply="mc", r0=0.04):
    """The whole of Aiyagari_VFI.m's computation (no plots)."""
    t0 = time.perf_counter()
    cal = cb.aiyagari(Na=Na, rho=rho, sigma_e=sigma_e, shocks=shocks)
    a, s, P, N = cal["a_grid"], cal["s"], cal["P"], cal["N"]
    st = _Stream(T, 10)
    z1 = int(math.ceil(N * st.take(1)[0]))                  # randi(N)  (1-based)
    k1 = a[int(math.ceil(Na * st.take(1)[0])) - 1]          # a_grid(randi(grid_size))
    state = {"v_old": np.zeros((N, Na))}

    def solve_at(r):
        R = vfi_solve(state["v_old"], a, s, P, r, cb.wage(r, cal["alpha"], cal["delta"]),
                      cal["beta"], cal["sigma"], tol, max_iter)
        state.update(v_old=R["v_old"], R=R)
        return R["iters"]

    def supply_of():
        R = state["R"]
        if supply == "mc":
            return sim_capital(R["policy_k"], a, P, z1, k1, st.take(T - 1))
        _, K, _, _ = dist_stationary(a, P, policy_idx=R["idx"], tol=1e-13, max_iter=100000)
        return K

    it0 = solve_at(r0)
    supply_of()
    out = _bisect(cal, solve_at, supply_of)
    out["iters"] = [it0] + out["iters"]
    out["wall_s"] = time.perf_counter() - t0
    out["cal"] = cal
    return out


def aiyagari_labor_vfi(Na=400, T=10000, tol=1e-5, max_iter=1000, supply="mc", r0=0.04,
                       labor_choice=None, psi=1.0, eta=2.0):
    """Aiyagari_Endogenous_Labor_VFI.m (rho = .6, sigma_e = .2, 10 labour levels)."""
    t0 = time.perf_counter()
    cal = cb.aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    a, s, P, N = cal["a_grid"], cal["s"], cal["P"], cal["N"]
    L = (0.01 + (1.5 - 0.01) * cb.linspace01(10)) if labor_choice is None else np.asarray(labor_choice)
    st = _Stream(T, 10)
    z1 = int(math.ceil(N * st.take(1)[0]))
    k1 = a[int(math.ceil(Na * st.take(1)[0])) - 1]
    state = {"v_old": np.zeros((N, Na)), "v_new": None, "pol": None}

    def solve_at(r):
        R = labor_vfi_solve(state["v_old"], a, s, P, L, r, cb.wage(r, cal["alpha"], cal["delta"]),
                            cal["beta"], cal["sigma"], psi, eta, tol, max_iter,
                            v_new=state["v_new"], policies=state["pol"])
        state.update(v_old=R["v_old"], v_new=R["v_new"], R=R,
                     pol=(R["policy_k"], R["policy_l"], R["policy_c"], R["lin"]))
        return R["iters"]

    def supply_of():
        R = state["R"]
        if supply == "mc":
            return sim_capital(R["policy_k"], a, P, z1, k1, st.take(T - 1))
        idx = (R["lin"] - 1) // len(L) + 1
        _, K, _, _ = dist_stationary(a, P, policy_idx=idx, tol=1e-13, max_iter=100000)
        return K

    it0 = solve_at(r0)
    supply_of()
    out = _bisect(cal, solve_at, supply_of)
    out["iters"] = [it0] + out["iters"]
    out["wall_s"] = time.perf_counter() - t0
    return out


def _egm_common(labor, Na, T, tol, max_iter, supply, phi=1.0, theta=1.0):
    t0 = time.perf_counter()
    cal = cb.aiyagari(Na=Na, rho=0.6 if labor else 0.75, sigma_e=0.2 if labor else 0.75)
    a, s, P, N = cal["a_grid"], cal["s"], cal["P"], cal["N"]
    r0 = 0.04
    w = cb.wage(r0, cal["alpha"], cal["delta"])  # frozen: the GE loop never updates w (:61)
    pc = np.tile(((1 + r0) * a + w * np.mean(s))[:, None], (1, N))  # :64
    st = _Stream(T, 10)
    z1 = int(math.ceil(N * st.take(1)[0]))
    k1 = a[int(math.ceil(Na * st.take(1)[0])) - 1]
    state = {"pc": pc}

    def solve_at(r):
        if labor:
            R = labor_egm_solve(state["pc"], a, s, P, r, w, cal["beta"], cal["sigma"], phi, theta,
                                cal["amin"], tol, max_iter)
        else:
            R = egm_solve(state["pc"], a, s, P, r, w, cal["beta"], cal["sigma"], cal["amin"], tol,
                          max_iter)
        state.update(pc=R["policy_c"], R=R)
        return R["iters"]

    def supply_of():
        R = state["R"]
        if supply == "mc":
            return sim_capital(R["policy_k"], a, P, z1, k1, st.take(T - 1), vfi_layout=False)
        _, K, _, _ = dist_stationary(a, P, policy_k=R["policy_k"], tol=1e-13, max_iter=100000,
                                     vfi_layout=False)
        return K

    it0 = solve_at(r0)
    supply_of()
    out = _bisect(cal, solve_at, supply_of)
    out["iters"] = [it0] + out["iters"]
    out["wall_s"] = time.perf_counter() - t0
    return out


def aiyagari_egm(Na=400, T=10000, tol=1e-5, max_iter=1000, supply="mc"):
    """Aiyagari_EGM.m."""
    return _egm_common(False, Na, T, tol, max_iter, supply)


def aiyagari_labor_egm(Na=400, T=10000, tol=1e-5, max_iter=1000, supply="mc", phi=1.0,
                       theta=1.0):
    """Aiyagari_Endogenous_Labor_EGM.m."""
    return _egm_common(True, Na, T, tol, max_iter, supply, phi, theta)
