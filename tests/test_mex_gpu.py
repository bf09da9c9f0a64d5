"""GPU: the MEX gateways end to end (stub mx API → C ABI → HIP), against the Python host
mirror and the C oracle: same numbers through the MATLAB-facing boundary."""
import numpy as np
import pytest

from tests import mexstub
from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def test_vfi_solve_gateway(pkg, gpu, golden):
    g = golden("a1_vfi_defaults")
    v_new, v_old, pk, pc, it = mexstub.call("aiy_vfi_solve_mex", 5, np.zeros((7, 400)),
                                            g["a_grid"], g["s"], g["P"], float(g["r"]),
                                            float(g["w"]), 0.96, 5.0, 1e-5, 1000.0)
    assert int(it[0, 0]) == 249
    assert np.array_equal(v_new, g["solve_v_new"]) and np.array_equal(v_old, g["solve_v_old"])
    v2, pk2, pc2, idx = mexstub.call("aiy_vfi_sweep_mex", 4, g["v20"], g["a_grid"], g["s"], g["P"],
                                     float(g["r"]), float(g["w"]), 0.96, 5.0)
    assert np.array_equal(v2, g["v21"]) and np.array_equal(idx - 1, g["idx21"])
    # the optional 6th output: the last sweep's 1-based argmax (Aiyagari_VFI.m:79-80), so the
    # host script needs no N x Na x Na min to rebuild it
    out = mexstub.call("aiy_vfi_solve_mex", 6, np.zeros((7, 400)), g["a_grid"], g["s"], g["P"],
                       float(g["r"]), float(g["w"]), 0.96, 5.0, 1e-5, 1000.0)
    R = corc.vfi_solve(np.zeros((7, 400)), g["a_grid"], g["s"], g["P"], float(g["r"]),
                       float(g["w"]), 0.96, 5.0)
    idx6 = out[5]
    assert idx6.shape == (7, 400) and np.array_equal(idx6 - 1, R["idx"])
    assert np.array_equal(out[2], g["a_grid"][idx6.astype(int) - 1])  # policy_k = a_grid(idx)
    assert np.array_equal(out[0], v_new)


def test_egm_and_sim_gateways(pkg, gpu, golden):
    g = golden("a4_egm_defaults")
    pc, pk, dist, it = mexstub.call("aiy_egm_solve_mex", 4, g["policy_c0"], g["a_grid"], g["s"],
                                    g["P"], float(g["r"]), float(g["w"]), 0.96, 5.0,
                                    float(g["amin"]), 1e-5, 1000.0)
    R = pkg.egm_solve(g["policy_c0"], g["a_grid"], g["s"], g["P"], float(g["r"]), float(g["w"]),
                      0.96, 5.0, float(g["amin"]))
    assert int(it[0, 0]) == R["iters"] and np.array_equal(pc, R["policy_c"])
    U = no.matlab_rand_stream(100)
    K, path, zs = mexstub.call("aiy_sim_capital_mex", 3, pk, g["a_grid"], g["P"], 3.0,
                               float(g["a_grid"][50]), U)
    Ko, po = corc.sim_capital(pk.T, g["a_grid"], g["P"], 2, float(g["a_grid"][50]), U,
                              return_path=True)
    assert K[0, 0] == Ko and np.array_equal(path[:, 0], po)


def test_labor_vfi_and_dist_gateways(pkg, gpu, golden):
    g = golden("a3_labor_vfi_na100")
    out = mexstub.call("aiy_labor_vfi_solve_mex", 6, np.zeros((7, 100)), g["a_grid"], g["s"],
                       g["P"], g["L"], float(g["r"]), float(g["w"]), 0.96, 5.0, 1.0, 2.0, 1e-5,
                       1000.0)
    v_new, v_old, pk, pl, pc, it = out
    assert int(it[0, 0]) == int(g["iters"])
    assert np.array_equal(v_new, g["v_new"]) and np.array_equal(pl, g["policy_l"])
    a1 = golden("a1_vfi_defaults")
    d = golden("a10_dist_defaults")
    lam, K, it2, dist = mexstub.call("aiy_dist_stationary_mex", 4, d["idx"] + 1.0, a1["a_grid"],
                                     a1["P"], d["lam0"], 0.0, 1.0, 1.0)
    assert np.array_equal(lam, corc.dist_update_ongrid(d["lam0"], d["idx"], a1["P"]))


def test_ks_gateway(pkg, gpu, golden):
    g = golden("ks_defaults")
    prm = pkg.ks_params()
    B = np.array([0.0, 1.0, 0.0, 1.0])
    V, ko, it, rel = mexstub.call("ks_vfi_solve_mex", 4, g["V0"], g["V0"] * 0 + 1, g["k_grid"],
                                  g["K_grid"], B, g["P"], prm, 5.0, 1e-6, 3.0, 1.0)
    R = pkg.ks_vfi_solve(g["V0"], g["V0"] * 0 + 1, g["k_grid"], g["K_grid"], B, g["P"], prm,
                         howard_steps=5, tol=1e-6, max_vfi=3)
    assert int(it[0, 0]) == R["iters"]
    assert np.array_equal(V.reshape(R["value"].shape, order="F"), R["value"])
    # n_devices = 8 at the reference K = 4: the (K, Z)-sliced path, depth 2 (12th argument)
    V8, ko8, it8, _ = mexstub.call("ks_vfi_solve_mex", 4, g["V0"], g["V0"] * 0 + 1, g["k_grid"],
                                   g["K_grid"], B, g["P"], prm, 5.0, 1e-6, 3.0, 8.0, 2.0)
    assert int(it8[0, 0]) == R["iters"]
    assert np.array_equal(V8.reshape(R["value"].shape, order="F"), R["value"])
    assert np.array_equal(ko8.reshape(R["k_opt"].shape, order="F"), R["k_opt"])


def test_ks_egm_gateway(pkg, gpu, golden):
    """ks_egm_solve_mex (Krusell_Smith_EGM.m:129-209) returns the golden policy after 3 sweeps."""
    g = golden("ks_egm_defaults")
    prm = pkg.ks_params()
    ko, it, diff = mexstub.call("ks_egm_solve_mex", 3, g["k_opt0"], g["k_grid"], g["K_grid"],
                                g["B"], g["P"], prm, 1e-6, 3.0)
    assert int(it[0, 0]) == 3
    assert np.array_equal(ko.reshape(g["k_opt3"].shape, order="F"), g["k_opt3"])
    assert float(diff[0, 0]) == float(g["diff3"])


def test_ks_egm_gateway_jacobi(pkg, gpu, golden):
    """ks_egm_solve_mex(..., jacobi=1): the F1 variant (flagged non-parity) through the gateway
    equals the library's Jacobi solve bit for bit."""
    g = golden("ks_egm_defaults")
    prm = pkg.ks_params()
    ko, it, diff = mexstub.call("ks_egm_solve_mex", 3, g["k_opt0"], g["k_grid"], g["K_grid"],
                                g["B"], g["P"], prm, 1e-6, 40.0, 1.0)
    R = pkg.ks_egm_solve(g["k_opt0"], g["k_grid"], g["K_grid"], g["B"], g["P"], prm, tol=1e-6,
                         max_iter=40, jacobi=True)
    assert int(it[0, 0]) == R["iters"] == 40
    assert np.array_equal(ko.reshape(R["k_opt"].shape, order="F"), R["k_opt"])
    assert float(diff[0, 0]) == R["diff"]


def test_ks_panel_gateways(pkg, gpu, golden):
    """ks_shocks_mex / ks_simulate_capital_mex (Krusell_Smith_VFI.m:57-94, :206-248) reproduce
    the committed panel fixture."""
    from oracle import np_oracle as no
    g = golden("ks_panel_small")
    T, pop = int(g["T"]), int(g["population"])
    U = no.matlab_rand_stream(no.ks_shock_draws(T, pop))
    zi, ep = mexstub.call("ks_shocks_mex", 2, float(T), float(pop), U, pkg.ks_params())
    assert np.array_equal(zi.ravel(), g["zi"]) and np.array_equal(ep, g["eps"] + 1)
    K_ts, kf = mexstub.call("ks_simulate_capital_mex", 2, g["k_opt"], g["k_grid"], g["K_grid"],
                            zi, ep, np.full(pop, g["K_grid"][0]))
    assert np.array_equal(K_ts.ravel(), g["K_ts"]) and np.array_equal(kf.ravel(), g["k_final"])


def test_clear_mex_releases_device_buffers(pkg, gpu, golden):
    """B3: `clear mex` (mexAtExit -> aiy_release_all) frees every cached device buffer of the
    host tier; the next call re-creates them and gives the same answer."""
    import ctypes as C
    lib = pkg.lib()
    lib.aiy_host_cache_bytes.restype = C.c_int64
    g = golden("a1_vfi_defaults")
    args = (np.zeros((7, 400)), g["a_grid"], g["s"], g["P"], float(g["r"]), float(g["w"]), 0.96,
            5.0, 1e-5, 1000.0)
    first = mexstub.call("aiy_vfi_solve_mex", 5, *args)
    assert lib.aiy_host_cache_bytes() > 0
    assert mexstub.lib().stub_lock_depth() == 0
    assert mexstub.lib().stub_clear_mex() >= 1
    assert lib.aiy_host_cache_bytes() == 0
    again = mexstub.call("aiy_vfi_solve_mex", 5, *args)
    for x, y in zip(first, again):
        assert np.array_equal(x, y)


def test_ge_batch_gateway(pkg, gpu):
    """Config 4 through the MATLAB-facing boundary equals the Python host mirror."""
    cal = pkg.calibration.aiyagari(Na=400)
    w0 = pkg.calibration.wage(0.04, cal["alpha"], cal["delta"])
    v0 = corc.vfi_solve(np.zeros((7, 400)), cal["a_grid"], cal["s"], cal["P"], 0.04, w0,
                        cal["beta"], cal["sigma"])["v_old"]
    r = np.array([-0.004166666666666667, -0.027083333333333334, 0.01875])
    U = no.matlab_rand_stream(2 + 3 * 9999)[2:].reshape(3, 9999).T  # one block per candidate
    ks, kd, it = mexstub.call("aiy_ge_batch_mex", 3, r, v0, cal["a_grid"], cal["s"], cal["P"],
                              cal["alpha"], cal["delta"], cal["beta"], cal["sigma"], cal["labor"],
                              1e-5, 1000.0, 6.0, float(cal["a_grid"][57]), U, 1.0)
    Ks, Kd, It = pkg.ge_batch.ge_batch_call(r, v0, cal, 6, float(cal["a_grid"][57]),
                                            [U[:, c] for c in range(3)])
    assert np.array_equal(ks[:, 0], Ks) and np.array_equal(kd[:, 0], Kd)
    assert np.array_equal(it[:, 0].astype(np.int64), It)


def test_step_gateways(pkg, gpu, golden):
    """SURVEY B2's step-level entry points through the MATLAB-facing boundary: one EGM pass
    (Aiyagari_EGM.m:77-107) iterated by the caller reproduces the solve gateway's loop; one
    labour EGM pass and one labour VFI sweep (…Labor_VFI.m:69-112) equal the C oracle's."""
    g = golden("a4_egm_defaults")
    args = (g["a_grid"], g["s"], g["P"], float(g["r"]), float(g["w"]), 0.96, 5.0)
    c = g["policy_c0"]
    it, dist = 0, 1.0
    while dist > 1e-5 and it < 1000:  # the script's own loop (:74) around the step gateway
        c_next, k, d = mexstub.call("aiy_egm_step_mex", 3, c, *args, float(g["amin"]))
        dist = float(d[0, 0])
        c = c_next
        it += 1
    pc, pk, dist2, it2 = mexstub.call("aiy_egm_solve_mex", 4, g["policy_c0"], *args,
                                      float(g["amin"]), 1e-5, 1000.0)
    assert it == int(it2[0, 0]) and dist == float(dist2[0, 0])
    assert np.array_equal(c, pc) and np.array_equal(k, pk)
    cl, kl, ll, dl = mexstub.call("aiy_labor_egm_step_mex", 4, g["policy_c0"], *args, 1.0, 1.0,
                                  float(g["amin"]))
    co, ko, lo, do = corc.labor_egm_step(g["policy_c0"].T, g["a_grid"], g["s"], g["P"],
                                         float(g["r"]), float(g["w"]), 0.96, 5.0, 1.0, 1.0,
                                         float(g["amin"]))
    assert np.array_equal(cl, co.T) and np.array_equal(kl, ko.T) and np.array_equal(ll, lo.T)
    assert float(dl[0, 0]) == do
    h = golden("a3_labor_vfi_na100")
    V = h["v_new"] + 0.25
    v1, k1, l1, c1, lin = mexstub.call("aiy_labor_vfi_sweep_mex", 5, V, h["a_grid"], h["s"],
                                       h["P"], h["L"], float(h["r"]), float(h["w"]), 0.96, 5.0,
                                       1.0, 2.0)
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(V, h["a_grid"], h["s"], h["P"], h["L"],
                                                     float(h["r"]), float(h["w"]), 0.96, 5.0,
                                                     1.0, 2.0)
    assert np.array_equal(v1, vo) and np.array_equal(lin - 1, lino)
    assert np.array_equal(k1, pko) and np.array_equal(l1, plo) and np.array_equal(c1, pco)


def test_ks_step_gateways(pkg, gpu, golden):
    """ks_policy_improve_mex (Krusell_Smith_VFI.m:148-168) and ks_howard_mex (:172-192) return
    the golden policy, fminbnd evaluation counts and two-sweep Howard values."""
    g = golden("ks_defaults")
    prm = np.array([g["beta"], g["alpha"], g["delta"], g["k_min"], g["k_max"], g["ug"], g["ub"],
                    g["l_bar"], g["mu"], 1.01, 0.99, 1.0, 0.0])
    shape = g["V0"].shape
    ko, nf = mexstub.call("ks_policy_improve_mex", 2, g["V0"], g["k_grid"], g["K_grid"], g["B"],
                          g["P"], prm)
    ko = ko.reshape(shape, order="F")
    assert np.array_equal(ko, g["k_opt"])
    assert np.array_equal(nf.reshape(shape, order="F"), g["nfev"])
    (V2,) = mexstub.call("ks_howard_mex", 1, g["V0"], ko, g["k_grid"], g["K_grid"], g["B"], g["P"],
                         prm, 2.0)
    assert np.array_equal(V2.reshape(shape, order="F"), g["V_howard2"])
