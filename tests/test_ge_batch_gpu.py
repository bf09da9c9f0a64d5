"""GPU: config 4's multisection GE on the HIP path (one rank): identical trace to the
sequential bisection over the same evaluator, and to the C-restatement evaluator (every
kernel is bit-exact), at the reference defaults (Na = 400, Tauchen, T = 10,000)."""
import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


def test_multisection_matches_sequential_and_oracle(pkg, gpu, golden):
    gb = pkg.ge_batch
    cb = pkg.calibration
    A = gb.aiyagari_vfi_multisection(levels=6)
    cal = cb.aiyagari(Na=400)
    w0 = cb.wage(0.04, cal["alpha"], cal["delta"])
    v0 = pkg.vfi_solve(np.zeros((7, 400)), cal["a_grid"], cal["s"], cal["P"], 0.04, w0,
                       cal["beta"], cal["sigma"])["v_old"]
    ev = gb.hip_vfi_evaluator(cal, v0)
    S = gb.bisection(ev, -0.05, 1 / cal["beta"] - 1)
    assert A.r_history == S.r_history and A.k_supply == S.k_supply and A.iters == S.iters
    assert A.rounds == 2 and A.candidates == 63 + 15
    # Aiyagari_VFI.m:142-206's own trace (golden, chained warm start): warm-starting every
    # candidate from the r0 solution moves K_s by ~1e-3 but takes every bracket decision the
    # same way, so the r sequence and the equilibrium r are identical
    g = golden("a11_ge_vfi_defaults")
    assert A.r_history == [float(x) for x in g["r_history"]]
    assert A.r == float(g["r_final"])
    assert np.max(np.abs(np.array(A.k_supply) - g["k_supply"])) < 1e-2

    def solve(v, r, w):
        return corc.vfi_solve(v, cal["a_grid"], cal["s"], cal["P"], r, w, cal["beta"], cal["sigma"])

    def simulate(pk, z1, k1, u):
        return corc.sim_capital(pk, cal["a_grid"], cal["P"], z1 - 1, k1, u)
    v0o = corc.vfi_solve(np.zeros((7, 400)), cal["a_grid"], cal["s"], cal["P"], 0.04, w0,
                         cal["beta"], cal["sigma"])["v_old"]
    assert np.array_equal(v0o, v0)
    O = gb.bisection(gb.vfi_evaluator(cal, solve, simulate, v0o), -0.05, 1 / cal["beta"] - 1)
    assert O.r_history == A.r_history and O.k_supply == A.k_supply
