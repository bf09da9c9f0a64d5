"""GPU parity for A4/A5 (Aiyagari_EGM.m:71-110, Aiyagari_Endogenous_Labor_EGM.m:64-107).
Against the C restatement: bit-exact (shared portable aiy_pow for RHS^(-1/σ)).  Against the
numpy golden (numpy's own SIMD pow): the north-star tolerance 1e-10."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def test_egm_solve_vs_golden(pkg, gpu, golden):
    g = golden("a4_egm_defaults")
    R = pkg.egm_solve(g["policy_c0"], g["a_grid"], g["s"], g["P"], float(g["r"]), float(g["w"]),
                      0.96, 5.0, float(g["amin"]))
    assert R["iters"] == int(g["iters"]) == 213
    assert np.max(np.abs(R["policy_c"] - g["policy_c"])) < 1e-10
    assert np.max(np.abs(R["policy_k"] - g["policy_k"])) < 1e-10
    assert abs(R["dist"] - float(g["dist"])) < 1e-10


def test_egm_step_vs_oracle(pkg, gpu, golden):
    g = golden("a4_egm_defaults")
    c1, k1, d1 = pkg.egm_step(g["policy_c0"], g["a_grid"], g["s"], g["P"], float(g["r"]),
                              float(g["w"]), 0.96, 5.0, float(g["amin"]))
    co, ko, do = corc.egm_step(g["policy_c0"].T, g["a_grid"], g["s"], g["P"], float(g["r"]),
                               float(g["w"]), 0.96, 5.0, float(g["amin"]))
    assert np.array_equal(c1, co.T) and np.array_equal(k1, ko.T) and d1 == do


def test_labor_egm_solve_vs_golden(pkg, gpu, golden):
    g = golden("a5_labor_egm_defaults")
    R = pkg.labor_egm_solve(g["policy_c0"], g["a_grid"], g["s"], g["P"], float(g["r"]),
                            float(g["w"]), 0.96, 5.0, 1.0, 1.0, float(g["amin"]))
    assert R["iters"] == int(g["iters"]) == 227
    for k in ("policy_c", "policy_k", "policy_l"):
        assert np.max(np.abs(R[k] - g[k])) < 1e-10, k


@pytest.mark.parametrize("Na,sigma,theta", [(20000, 5.0, 1.0), (5000, 2.5, 2.0)])
def test_egm_large_and_nonint(pkg, gpu, Na, sigma, theta):
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst", sigma=sigma)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.03, 0.36, 0.08)
    pc0 = np.tile(((1.03) * a + w * np.mean(s))[:, None], (1, 7))
    R = pkg.egm_solve(pc0, a, s, P, 0.03, w, 0.96, sigma, cal["amin"], 1e-5, 40)
    Ro = corc.egm_solve(pc0.T, a, s, P, 0.03, w, 0.96, sigma, cal["amin"], 1e-5, 40)
    assert R["iters"] == Ro["iters"]
    assert np.array_equal(R["policy_c"], Ro["policy_c"].T)
    assert np.array_equal(R["policy_k"], Ro["policy_k"].T)
    L = pkg.labor_egm_solve(pc0, a, s, P, 0.03, w, 0.96, sigma, 1.0, theta, cal["amin"], 1e-5, 20)
    Lo = corc.labor_egm_solve(pc0.T, a, s, P, 0.03, w, 0.96, sigma, 1.0, theta, cal["amin"], 1e-5, 20)
    assert L["iters"] == Lo["iters"]
    for k in ("policy_c", "policy_k", "policy_l"):
        assert np.array_equal(L[k], Lo[k].T), k


def test_egm_nonmonotone_grid_is_reported(pkg, gpu):
    """interp1 needs a monotone endogenous grid; a decreasing one is an error, not garbage."""
    a = np.linspace(0, 10, 50)
    pc0 = np.tile(np.linspace(50, 0.01, 50)[:, None], (1, 2))  # steeply decreasing c → â folds
    with pytest.raises(pkg.AiyError) as e:
        pkg.egm_step(pc0, a, np.array([1.0, 1.2]), np.full((2, 2), 0.5), 0.02, 1.0, 0.96, 5.0, 0.0)
    assert e.value.status == "AIY_BAD_ARG"


@pytest.mark.parametrize("tol,max_iter", [(1e-5, 7), (1e-3, 1000), (1e-5, 1), (2e-2, 1000),
                                          (1e-5, 16), (1e-5, 17)])
def test_egm_speculative_solve_matches_oracle(pkg, gpu, tol, max_iter):
    """The host-tier solve enqueues up to 16 steps between dist reads (ring of policy_c buffers,
    the stopping step re-run for its policy_k): iteration count, dist and both policies equal
    the one-read-per-step C loop for stops inside a batch, on a batch edge and at max_iter."""
    cal = no.calib_aiyagari(Na=400, shocks="tauchen")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.04, 0.36, 0.08)
    pc0 = np.tile(((1.04) * a + w * np.mean(s))[:, None], (1, s.size))
    R = pkg.egm_solve(pc0, a, s, P, 0.04, w, 0.96, 5.0, cal["amin"], tol, max_iter)
    Ro = corc.egm_solve(pc0.T, a, s, P, 0.04, w, 0.96, 5.0, cal["amin"], tol, max_iter)
    assert R["iters"] == Ro["iters"]
    assert np.array_equal(R["policy_c"], Ro["policy_c"].T)
    assert np.array_equal(R["policy_k"], Ro["policy_k"].T)
    assert R["dist"] == Ro["dist"]
    L = pkg.labor_egm_solve(pc0, a, s, P, 0.04, w, 0.96, 5.0, 1.0, 1.0, cal["amin"], tol, max_iter)
    Lo = corc.labor_egm_solve(pc0.T, a, s, P, 0.04, w, 0.96, 5.0, 1.0, 1.0, cal["amin"], tol,
                              max_iter)
    assert L["iters"] == Lo["iters"]
    for k in ("policy_c", "policy_k", "policy_l"):
        assert np.array_equal(L[k], Lo[k].T), k


def test_egm_solve_nonmonotone_grid_is_reported(pkg, gpu):
    a = np.linspace(0, 10, 50)
    pc0 = np.tile(np.linspace(50, 0.01, 50)[:, None], (1, 2))
    with pytest.raises(pkg.AiyError) as e:
        pkg.egm_solve(pc0, a, np.array([1.0, 1.2]), np.full((2, 2), 0.5), 0.02, 1.0, 0.96, 5.0,
                      0.0, 1e-6, 50)
    assert e.value.status == "AIY_BAD_ARG"
