"""GPU parity for F3/F2 (Krusell_Smith_VFI.m:57-94 shock panel, :206-248 panel simulation):
HIP kernels through the C ABI vs the numpy restatement — bit-exact (integer shocks, and the
interpolation/mean use only IEEE basic operations in the same order)."""
import numpy as np
import pytest

from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def _prm(pkg):
    return pkg.ks_params()


def test_shocks_fixture(pkg, gpu, golden):
    g = golden("ks_panel_small")
    T, pop = int(g["T"]), int(g["population"])
    U = no.matlab_rand_stream(no.ks_shock_draws(T, pop))
    zi, eps = pkg.ks_panel.ks_shocks(T, pop, U, _prm(pkg))
    assert np.array_equal(zi, g["zi"])
    assert np.array_equal(eps, g["eps"] + 1)


def test_simulate_fixture(pkg, gpu, golden):
    g = golden("ks_panel_small")
    T, pop = int(g["T"]), int(g["population"])
    K_ts, kf = pkg.ks_panel.ks_simulate_capital(g["k_opt"], g["k_grid"], g["K_grid"], g["zi"],
                                                g["eps"] + 1, np.full(pop, g["K_grid"][0]))
    assert np.array_equal(K_ts, g["K_ts"]) and np.array_equal(kf, g["k_final"])


@pytest.mark.parametrize("T,pop", [(1100, 10000), (2, 1), (7, 255), (9, 257), (33, 300001),
                                   (3, 5 * 262144 + 7)])
def test_reference_size_and_ragged(pkg, gpu, golden, T, pop):
    """The script's panel (T = 1100, 10,000 agents) and ragged/edge populations (one agent,
    one block short/over, > 1024 blocks so lanes hold several agents)."""
    import torch
    g = golden("ks_panel_small")
    p, kg, Kg, *_ = no.ks_setup()
    U = no.matlab_rand_stream(no.ks_shock_draws(T, pop))
    zi_o, e_o = no.ks_shocks(p, T, pop, U)
    rng = np.random.default_rng(pop)
    k0 = rng.uniform(0.0, 200.0, pop)
    K_o, kf_o = no.ks_panel_simulate(kg, Kg, g["k_opt"], zi_o, e_o, k0)
    dev = torch.device("cuda", 0)
    Ut = torch.as_tensor(U, device=dev)
    zi, eps = pkg.ks_panel.ks_shocks_dev(Ut, _prm(pkg), T, pop)
    torch.cuda.synchronize()
    assert np.array_equal(zi.cpu().numpy(), zi_o) and np.array_equal(eps.cpu().numpy(), e_o)
    ko = torch.as_tensor(np.ascontiguousarray(g["k_opt"].transpose(2, 1, 0)), device=dev)
    sim = pkg.ks_panel.PanelSim(torch.as_tensor(kg, device=dev), torch.as_tensor(Kg, device=dev),
                                zi, eps, torch.as_tensor(k0, device=dev))
    K_ts = sim(ko)
    torch.cuda.synchronize()
    assert np.array_equal(K_ts.cpu().numpy(), K_o)
    assert np.array_equal(sim.k_pop.cpu().numpy(), kf_o)


def test_host_tier_validation(pkg, gpu):
    g_k = np.linspace(0, 1, 5)
    with pytest.raises(pkg.AiyError):
        pkg.ks_panel.ks_simulate_capital(np.zeros((5, 2, 4)), g_k, np.array([30.0, 50.0]),
                                         np.array([0.0, 2.0]), np.ones((2, 3)), np.ones(3))
    with pytest.raises(pkg.AiyError):
        pkg.ks_panel.ks_simulate_capital(np.zeros((5, 2, 4)), g_k, np.array([30.0, 50.0]),
                                         np.array([0.0, 1.0]), np.full((2, 3), 3.0), np.ones(3))


def test_alm_driver_one_iteration(pkg, gpu):
    """Krusell_Smith_VFI.m:138-296, one ALM iteration at the reference size: VFI (A6/A7), panel
    simulation (F2) and regression composed; the simulated K path equals the oracle
    simulation driven by the same GPU policy."""
    R = pkg.ks_panel.krusell_smith_vfi(max_iter_B=1, max_vfi=60)
    p, kg, Kg, *_ = no.ks_setup()
    U = no.matlab_rand_stream(no.ks_shock_draws(1100, 10000))
    zi, e = no.ks_shocks(p, 1100, 10000, U)
    K_o, _ = no.ks_panel_simulate(kg, Kg, R["k_opt"], zi, e, np.full(10000, Kg[0]))
    assert np.array_equal(R["K_ts"], K_o)
    B, r2g, r2b = no.ks_alm_regress(K_o, zi)
    assert np.allclose(R["B_history"][0], B, rtol=0, atol=1e-10)
