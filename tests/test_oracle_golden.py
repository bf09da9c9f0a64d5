"""CPU: the C restatement (oracle/liborc.so) against the golden fixtures produced by the
independent numpy restatement (tests/golden/make_golden.py).  Parity vs MATLAB: unpinned."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no


def test_rng_matches_matlab_documentation(golden):
    g = golden("rng_mt5489")
    assert np.array_equal(no.matlab_rand_stream(10), g["first10"])
    # MATLAB doc, fresh session rand(3) (column-major), 4 decimals
    assert np.allclose(g["first10"][:9], g["matlab_doc_4dp"], atol=5e-5)


def test_vfi_sweep_bitwise(golden):
    g = golden("a1_vfi_defaults")
    v, idx, pk, pc = corc.vfi_sweep(g["v20"], g["a_grid"], g["s"], g["P"], float(g["r"]),
                                    float(g["w"]), 0.96, 5.0)
    assert np.array_equal(v, g["v21"])
    assert np.array_equal(idx, g["idx21"])
    assert np.array_equal(pk, g["policy_k21"]) and np.array_equal(pc, g["policy_c21"])


def test_vfi_solve_break_semantics(golden):
    g = golden("a1_vfi_defaults")
    R = corc.vfi_solve(np.zeros((7, 400)), g["a_grid"], g["s"], g["P"], float(g["r"]),
                       float(g["w"]), 0.96, 5.0, 1e-5, 1000)
    assert R["iters"] == int(g["solve_iters"]) == 249
    assert np.array_equal(R["v_new"], g["solve_v_new"])
    assert np.array_equal(R["v_old"], g["solve_v_old"])
    assert not np.array_equal(R["v_new"], R["v_old"])
    assert np.array_equal(R["idx"], g["solve_idx"])


def test_labor_vfi_bitwise(golden):
    g = golden("a3_labor_vfi_na100")
    R = corc.labor_vfi_solve(np.zeros((7, 100)), g["a_grid"], g["s"], g["P"], g["L"],
                             float(g["r"]), float(g["w"]), 0.96, 5.0, 1.0, 2.0)
    assert R["iters"] == int(g["iters"])
    for k in ("v_new", "v_old", "policy_k", "policy_l", "policy_c"):
        assert np.array_equal(R[k], g[k]), k
    assert np.array_equal(R["lin"], g["lin"])


def test_egm_close(golden):
    g = golden("a4_egm_defaults")
    R = corc.egm_solve(g["policy_c0"].T, g["a_grid"], g["s"], g["P"], float(g["r"]),
                       float(g["w"]), 0.96, 5.0, float(g["amin"]))
    assert R["iters"] == int(g["iters"]) == 213
    # pow(RHS, -1/sigma): numpy's SIMD pow and glibc pow differ by an ulp
    assert np.max(np.abs(R["policy_c"] - g["policy_c"].T)) < 1e-10
    assert np.max(np.abs(R["policy_k"] - g["policy_k"].T)) < 1e-10
    c1, k1, d1 = corc.egm_step(g["policy_c0"].T, g["a_grid"], g["s"], g["P"], float(g["r"]),
                               float(g["w"]), 0.96, 5.0, float(g["amin"]))
    assert np.max(np.abs(c1 - g["step1_c"].T)) < 1e-12


def test_labor_egm_close(golden):
    g = golden("a5_labor_egm_defaults")
    R = corc.labor_egm_solve(g["policy_c0"].T, g["a_grid"], g["s"], g["P"], float(g["r"]),
                             float(g["w"]), 0.96, 5.0, 1.0, 1.0, float(g["amin"]))
    assert R["iters"] == int(g["iters"]) == 227
    for k in ("policy_c", "policy_k", "policy_l"):
        assert np.max(np.abs(R[k] - g[k].T)) < 1e-10, k


def test_sim_and_ge_trace(golden):
    g = golden("a11_ge_vfi_defaults")
    a1 = golden("a1_vfi_defaults")
    R = corc.vfi_solve(np.zeros((7, 400)), a1["a_grid"], a1["s"], a1["P"], 0.04,
                       float(a1["w"]), 0.96, 5.0)
    U = no.matlab_rand_stream(2 + 9999)[2:]
    Ks, path = corc.sim_capital(R["policy_k"], a1["a_grid"], a1["P"], int(g["z1"]),
                                float(g["k1"]), U, return_path=True)
    assert Ks == float(g["Ks0"]) and np.array_equal(path, g["sim_k0"])
    # full GE trace with C solves (bisection decisions identical → same r sequence)
    cal = no.calib_aiyagari()
    H = no.ge_bisection_vfi(cal, solve=lambda *a: corc.vfi_solve(*a))
    assert np.array_equal(H["r"], g["r_history"])
    assert H["iters"] == list(g["iters"])
    assert abs(H["r_final"] - float(g["r_final"])) == 0.0
    assert np.array_equal(H["k_supply"], g["k_supply"])


def test_dist_update(golden):
    g = golden("a10_dist_defaults")
    a1 = golden("a1_vfi_defaults")
    out = corc.dist_update_ongrid(g["lam0"], g["idx"], a1["P"])
    assert np.max(np.abs(out - g["lam1"])) < 1e-15 and abs(out.sum() - 1) < 1e-12
    outL = corc.dist_update_lottery(g["lam0"], g["kp_egm"], a1["a_grid"], a1["P"])
    assert np.max(np.abs(outL - g["lam1_lottery"])) < 1e-15


def test_ks_bitwise(golden):
    g = golden("ks_defaults")
    p = corc.ks_params(beta=float(g["beta"]), alpha=float(g["alpha"]), delta=float(g["delta"]),
                       k_min=float(g["k_min"]), k_max=float(g["k_max"]), ug=float(g["ug"]),
                       ub=float(g["ub"]), l_bar=float(g["l_bar"]), mu=float(g["mu"]),
                       z_grid=(1.01, 0.99), eps_grid=(1.0, 0.0))
    ko, nf = corc.ks_policy_improve(p, g["k_grid"], g["K_grid"], g["V0"], g["B"], g["P"])
    assert np.array_equal(ko, g["k_opt"]) and np.array_equal(nf, g["nfev"])
    V2 = corc.ks_howard(p, g["k_grid"], g["K_grid"], g["V0"], ko, g["B"], g["P"], 2)
    assert np.array_equal(V2, g["V_howard2"])


def test_portable_log_close_to_libm():
    import math
    rng = np.random.default_rng(3)
    xs = np.concatenate([rng.uniform(1e-12, 1e4, 2000), 10 ** rng.uniform(-300, 300, 500)])
    for x in xs:
        y = no.fdlibm_log(float(x))
        assert abs(y - math.log(x)) <= math.ulp(math.log(x))


def _ks_cparams(g):
    return corc.ks_params(beta=float(g["beta"]), alpha=float(g["alpha"]), delta=float(g["delta"]),
                          k_min=float(g["k_min"]), k_max=float(g["k_max"]), ug=float(g["ug"]),
                          ub=float(g["ub"]), l_bar=float(g["l_bar"]), mu=float(g["mu"]),
                          z_grid=(1.01, 0.99), eps_grid=(1.0, 0.0))


def test_ks_egm_bitwise(golden):
    """A8 (Krusell_Smith_EGM.m:129-209): the C restatement equals the numpy restatement bit for
    bit after 1 and 3 Gauss-Seidel sweeps and over the whole solve (994 sweeps to 1e-6)."""
    g = golden("ks_egm_defaults")
    p = _ks_cparams(g)
    args = (p, g["k_grid"], g["K_grid"], g["B"], g["P"], g["k_opt0"])
    r1 = corc.ks_egm_solve(*args, max_iter=1)
    assert np.array_equal(r1["k_opt"], g["k_opt1"])
    r3 = corc.ks_egm_solve(*args, max_iter=3)
    assert np.array_equal(r3["k_opt"], g["k_opt3"]) and r3["diff"] == float(g["diff3"])
    rf = corc.ks_egm_solve(*args, tol=1e-6, max_iter=10000)
    assert rf["iters"] == int(g["iters"]) == 994
    assert np.array_equal(rf["k_opt"], g["k_opt_final"]) and rf["diff"] == float(g["diff_final"])
    # properties of the converged policy: inside [k_min, k_max], nondecreasing in k
    assert (rf["k_opt"] >= float(g["k_min"])).all() and (rf["k_opt"] <= float(g["k_max"])).all()
    assert (np.diff(rf["k_opt"], axis=0) >= 0).all()


def test_ks_egm_jacobi_variant_restatements_agree(golden):
    """F1 (not the reference's result): the Jacobi KS EGM sweep — every (s, K) pair reads the
    previous sweep's k_opt instead of Krusell_Smith_EGM.m:199's in-place Gauss-Seidel update —
    restated in C and numpy, bit-identical to each other; it differs from the Gauss-Seidel
    iterate after one sweep but converges to the same fixed point within tolerance."""
    from oracle import np_oracle as no
    g = golden("ks_egm_defaults")
    p = _ks_cparams(g)
    args = (p, g["k_grid"], g["K_grid"], g["B"], g["P"], g["k_opt0"])
    pn, *_ = no.ks_setup()
    for m in (1, 2):
        rc = corc.ks_egm_solve(*args, max_iter=m, jacobi=True)
        rn = no.ks_egm_solve(pn, g["k_grid"], g["K_grid"], g["B"], g["P"], g["k_opt0"],
                             max_iter=m, jacobi=True)
        assert np.array_equal(rc["k_opt"], rn["k_opt"]) and rc["diff"] == rn["diff"]
    assert not np.array_equal(corc.ks_egm_solve(*args, max_iter=1, jacobi=True)["k_opt"],
                              g["k_opt1"])
    rj = corc.ks_egm_solve(*args, tol=1e-6, max_iter=10000, jacobi=True)
    assert rj["diff"] < 1e-6
    assert np.max(np.abs(rj["k_opt"] - g["k_opt_final"])) < 1e-3
