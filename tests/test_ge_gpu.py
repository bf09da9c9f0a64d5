"""GPU end-to-end for A11 (the GE bisection of each Aiyagari script) with A9 Monte-Carlo supply:
every solve and simulation on the GPU, compared with the same pipeline composed from the C
restatement.  Because every kernel is bit-exact, the bisection trace (r, K_s, K_d, iterations)
must be identical — for the VFI script also to the numpy golden trace."""
import math

import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def test_ge_vfi_matches_golden_trace(pkg, gpu, golden):
    g = golden("a11_ge_vfi_defaults")
    out = pkg.ge.aiyagari_vfi()
    assert out["r_history"] == list(g["r_history"])
    assert out["k_supply"] == list(g["k_supply"])
    assert out["iters"] == list(g["iters"])
    assert out["r"] == float(g["r_final"])


def test_ge_vfi_overlapped_matches_golden_trace(pkg, gpu, golden):
    """The overlapped driver (chain beside both speculative next solves) runs the same solves
    and chains: the trace equals the golden one and the sequential driver's."""
    g = golden("a11_ge_vfi_defaults")
    out = pkg.ge.aiyagari_vfi_overlapped()
    assert out["r_history"] == list(g["r_history"])
    assert out["k_supply"] == list(g["k_supply"])
    assert out["iters"] == list(g["iters"])
    assert out["r"] == float(g["r_final"])
    # a shorter bisection and a tighter grid: still identical to the sequential driver
    kw = dict(Na=300, T=3000)
    seq = pkg.ge.aiyagari_vfi(**kw)
    for la in (1, 2, 3):  # speculation depth (levels solved ahead of the pending chain)
        ovl = pkg.ge.aiyagari_vfi_overlapped(lookahead=la, **kw)
        for key in ("r_history", "k_supply", "k_demand", "iters", "r"):
            assert ovl[key] == seq[key], (la, key)


def _oracle_ge(cal, solve_at_factory, policy_of, vfi_layout, T=10000):
    U = no.matlab_rand_stream(2 + (T - 1) * 11)
    N, Na, a, P = cal["N"], cal["Na"], cal["a_grid"], cal["P"]
    z1 = int(math.ceil(N * U[0])) - 1
    k1 = a[int(math.ceil(Na * U[1])) - 1]
    pos = [2]

    def supply(pol):
        u = U[pos[0]:pos[0] + T - 1]
        pos[0] += T - 1
        return corc.sim_capital(pol if vfi_layout else pol.T, a, P, z1, k1, u)

    solve_at = solve_at_factory(cal)
    it0 = solve_at(0.04)
    supply(policy_of())
    r_low, r_high = -0.05, 1 / cal["beta"] - 1
    hist = dict(r=[], ks=[], iters=[it0])
    for _ in range(10):
        r = (r_low + r_high) / 2
        hist["iters"].append(solve_at(r))
        Ks = supply(policy_of())
        Kd = cal["labor"] * (cal["alpha"] / (r + cal["delta"])) ** (1 / (1 - cal["alpha"]))
        hist["r"].append(r); hist["ks"].append(Ks)
        if abs(Ks - Kd) < 1e-5:
            break
        r_high, r_low = (r, r_low) if Ks > Kd else (r_high, r)
    return hist


@pytest.mark.parametrize("labor", [False, True])
def test_ge_egm_matches_oracle(pkg, gpu, labor):
    out = pkg.ge.aiyagari_labor_egm() if labor else pkg.ge.aiyagari_egm()
    cal = no.calib_aiyagari(rho=0.6 if labor else 0.75, sigma_e=0.2 if labor else 0.75)
    w = no.wage(0.04, 0.36, 0.08)
    st = {"pc": np.tile((1.04 * cal["a_grid"] + w * np.mean(cal["s"]))[None, :], (7, 1))}

    def factory(cal):
        def solve_at(r):
            if labor:
                R = corc.labor_egm_solve(st["pc"], cal["a_grid"], cal["s"], cal["P"], r, w, 0.96,
                                         5.0, 1.0, 1.0, cal["amin"])
            else:
                R = corc.egm_solve(st["pc"], cal["a_grid"], cal["s"], cal["P"], r, w, 0.96, 5.0,
                                   cal["amin"])
            st["pc"] = R["policy_c"]; st["pk"] = R["policy_k"]
            return R["iters"]
        return solve_at

    H = _oracle_ge(cal, factory, lambda: st["pk"].T, vfi_layout=False)
    assert out["iters"] == H["iters"]
    assert out["r_history"] == H["r"]
    assert out["k_supply"] == H["ks"]


def test_ge_labor_vfi_matches_oracle(pkg, gpu):
    Na = 100
    out = pkg.ge.aiyagari_labor_vfi(Na=Na)
    cal = no.calib_aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    L = 0.01 + (1.5 - 0.01) * no.matlab_linspace01(10)
    st = {"v_old": np.zeros((7, Na)), "v_new": None, "pol": None}

    def factory(cal):
        def solve_at(r):
            w = no.wage(r, 0.36, 0.08)
            v_old = st["v_old"].copy()
            v_new = np.zeros((7, Na)) if st["v_new"] is None else st["v_new"]
            pol = st["pol"]
            for it in range(1, 1001):
                v_new, pol = corc.labor_vfi_sweep(v_old, cal["a_grid"], cal["s"], cal["P"], L, r, w,
                                                  0.96, 5.0, 1.0, 2.0, v_new=v_new, pol=pol)
                if np.nanmax(np.abs(v_new - v_old)) < 1e-5:
                    break
                v_old = v_new.copy()
            st.update(v_old=v_old, v_new=v_new, pol=pol)
            return it
        return solve_at

    H = _oracle_ge(cal, factory, lambda: st["pol"][0], vfi_layout=True)
    assert out["iters"] == H["iters"]
    assert out["r_history"] == H["r"]
    assert out["k_supply"] == H["ks"]


def test_ge_histogram_supply_runs(pkg, gpu):
    """A10 as the supply estimator: a different (deterministic) estimator of K_s, so only
    sanity is asserted: r stays in the bracket and the bisection ends near the crossing."""
    out = pkg.ge.aiyagari_vfi(supply="histogram")
    assert -0.05 < out["r"] < 1 / 0.96 - 1
    gap = abs(out["k_supply"][-1] - out["k_demand"][-1])
    assert gap < 1.0


def test_ge_overlapped_pool_reuse_other_calibration(pkg, gpu):
    """the overlapped driver's pooled workspaces cache feasible prefixes keyed
    on (r, w) and the addresses of a and s.  Two calls at the same Na with different
    calibrations (so different a and s, possibly at reused addresses, and the same bisection
    midpoints) must each equal the sequential driver."""
    kw = dict(Na=300, T=3000)
    for rho, sig in ((0.75, 0.75), (0.6, 0.2), (0.75, 0.75)):
        seq = pkg.ge.aiyagari_vfi(rho=rho, sigma_e=sig, **kw)
        ovl = pkg.ge.aiyagari_vfi_overlapped(rho=rho, sigma_e=sig, **kw)
        for key in ("r_history", "k_supply", "k_demand", "iters", "r"):
            assert ovl[key] == seq[key], (rho, sig, key)
