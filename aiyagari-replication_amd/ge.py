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


def aiyagari_vfi_overlapped(Na=400, rho=0.75, sigma_e=0.75, shocks="tauchen", T=10000, tol=1e-5,
                            max_iter=1000, r0=0.04, max_r_iter=10, r_tol=1e-5):
    """Aiyagari_VFI.m's computation (as `aiyagari_vfi`, supply = MC) with the bisection's
    serial Monte-Carlo chain taken off the critical path.  Step j needs K_s(r_j) only to pick
    the next midpoint, and both candidates warm-start from the same v_old(r_j): so while the
    chain for r_j runs (one CU), the solves at both possible next midpoints run beside it on
    their own streams and workspaces (device tier, one host thread each; ctypes drops the GIL),
    and the chain's K_s selects one.  Every solve and chain is the one the sequential loop runs,
    on the same inputs and uniform block, so r_history / k_supply / iters are identical
    (tests/test_ge_gpu.py); the discarded solve is spare GPU work."""
    import concurrent.futures as cf

    import torch

    from .sim import sim_capital_dev
    from .vfi import Workspace

    t0 = time.perf_counter()
    cal = cb.aiyagari(Na=Na, rho=rho, sigma_e=sigma_e, shocks=shocks)
    a, s, P, N = cal["a_grid"], cal["s"], cal["P"], cal["N"]
    st = _Stream(T, max_r_iter)
    z1 = int(math.ceil(N * st.take(1)[0]))
    k1 = float(a[int(math.ceil(Na * st.take(1)[0])) - 1])
    dev = torch.device("cuda", torch.cuda.current_device())
    tt = lambda x: torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=dev)
    a_t, s_t, P_t = tt(a), tt(s), tt(P)
    U = tt(st.u[st.pos:])  # block j (the j-th chain's T-1 draws) = U[j(T-1) : (j+1)(T-1)]

    class _Slot:
        def __init__(self):
            self.ws = Workspace(N, Na)
            self.stream = torch.cuda.Stream(device=dev)
            self.va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
            self.vb = torch.zeros_like(self.va)
            self.idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
            self.pk, self.pc = torch.empty_like(self.va), torch.empty_like(self.va)
            self.v_old = None

        def solve(self, v_init, r):
            with torch.cuda.stream(self.stream):
                self.va.copy_(v_init)
                self.vb.zero_()
                it, which = self.ws.vfi_solve(
                    self.va, self.vb, a_t, s_t, P_t, r, cb.wage(r, cal["alpha"], cal["delta"]),
                    cal["beta"], cal["sigma"], tol, max_iter, self.idx, self.pk, self.pc,
                    stream=self.stream)
                self.stream.synchronize()
            self.v_old = self.vb if which == 0 else self.va
            return it

    sim_ws = Workspace(N, Na)
    sim_stream = torch.cuda.Stream(device=dev)
    k_out = torch.zeros(1, dtype=torch.float64, device=dev)
    k_status = torch.zeros(1, dtype=torch.int32, device=dev)

    def chain(slot, j):
        with torch.cuda.stream(sim_stream):
            sim_capital_dev(sim_ws, slot.pk, a_t, P_t, z1 - 1, k1, U[j * (T - 1):(j + 1) * (T - 1)],
                            k_out, k_status, stream=sim_stream)
            sim_stream.synchronize()
        if int(k_status.item()) != 0:
            raise RuntimeError("find() empty in the capital-supply chain (Aiyagari_VFI.m:106)")
        return float(k_out.item())

    slots = [_Slot(), _Slot(), _Slot()]
    cur = slots[0]
    out = dict(r_history=[], k_supply=[], k_demand=[], iters=[])
    r_low, r_high = -0.05, 1 / cal["beta"] - 1
    with cf.ThreadPoolExecutor(max_workers=3) as pool:
        it0 = cur.solve(torch.zeros((N, Na), dtype=torch.float64, device=dev), r0)
        r = (r_low + r_high) / 2
        # the chain at r0 (its K_s is not used by the bisection) beside the first midpoint
        f_chain = pool.submit(chain, cur, 0)
        nxt = slots[1]
        it = nxt.solve(cur.v_old, r)
        f_chain.result()
        cur, spare = nxt, [slots[0], slots[2]]
        for j in range(1, max_r_iter + 1):
            last = j == max_r_iter
            r_lo_next, r_hi_next = (r_low + r) / 2, (r + r_high) / 2  # Ks > Kd : else
            f_chain = pool.submit(chain, cur, j)
            if not last:
                f_lo = pool.submit(spare[0].solve, cur.v_old, r_lo_next)
                f_hi = pool.submit(spare[1].solve, cur.v_old, r_hi_next)
            Ks = f_chain.result()
            Kd = cb.capital_demand(r, cal["labor"], cal["alpha"], cal["delta"])
            out["r_history"].append(r); out["k_supply"].append(Ks); out["k_demand"].append(Kd)
            out["iters"].append(it)
            if not last:
                it_lo, it_hi = f_lo.result(), f_hi.result()
            if last or abs(Ks - Kd) < r_tol:
                break
            if Ks > Kd:
                r_high = r
                r, it, chosen, other = r_lo_next, it_lo, spare[0], spare[1]
            else:
                r_low = r
                r, it, chosen, other = r_hi_next, it_hi, spare[1], spare[0]
            spare = [cur, other]
            cur = chosen
    out["r"] = out["r_history"][-1]
    out["iters"] = [it0] + out["iters"]
    out["wall_s"] = time.perf_counter() - t0
    out["cal"] = cal
    for sl in slots:
        sl.ws.close()
    sim_ws.close()
    return out
