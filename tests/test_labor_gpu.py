"""GPU parity for A3 (Aiyagari_Endogenous_Labor_VFI.m:64-122): joint (l, a') max in
column-major order, bit-exact against the golden fixture (numpy restatement) and the C oracle."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def test_labor_solve_matches_golden_bitwise(pkg, gpu, golden):
    g = golden("a3_labor_vfi_na100")
    R = pkg.labor_vfi_solve(np.zeros((7, 100)), g["a_grid"], g["s"], g["P"], g["L"],
                            float(g["r"]), float(g["w"]), 0.96, 5.0, 1.0, 2.0)
    assert R["iters"] == int(g["iters"])
    for k in ("v_new", "v_old", "policy_k", "policy_l", "policy_c"):
        assert np.array_equal(R[k], g[k]), k
    assert np.array_equal(R["lin"] - 1, g["lin"])


@pytest.mark.parametrize("Na", [400, 1333])
def test_labor_sweep_vs_oracle(pkg, gpu, Na):
    cal = no.calib_aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    L = 0.01 + (1.5 - 0.01) * no.matlab_linspace01(10)
    w = no.wage(0.04, 0.36, 0.08)
    V = corc.labor_vfi_solve(np.zeros((7, Na)), a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0,
                             1e-5, 12)["v_new"]
    v, pk, pl, pc, lin = pkg.labor_vfi_sweep(V, a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0)
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(V, a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0)
    assert np.array_equal(v, vo)
    assert np.array_equal(lin - 1, lino)
    assert np.array_equal(pk, pko) and np.array_equal(pl, plo) and np.array_equal(pc, pco)


def test_labor_nonuniform_levels_and_sigma(pkg, gpu):
    """Unsorted labour grid, odd Nl (ragged last block), σ = 3 and non-integer η."""
    cal = no.calib_aiyagari(Na=257, rho=0.6, sigma_e=0.2, sigma=3.0)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    L = np.array([0.7, 0.05, 1.2, 0.3, 1.0, 0.5, 0.9])
    w = no.wage(0.03, 0.36, 0.08)
    V = corc.labor_vfi_solve(np.zeros((7, 257)), a, s, P, L, 0.03, w, 0.96, 3.0, 1.0, 1.5,
                             1e-5, 8)["v_new"]
    v, pk, pl, pc, lin = pkg.labor_vfi_sweep(V, a, s, P, L, 0.03, w, 0.96, 3.0, 1.0, 1.5)
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(V, a, s, P, L, 0.03, w, 0.96, 3.0, 1.0, 1.5)
    # eta = 1.5 → L^(2.5) through the shared aiy_pow: bit-exact
    assert np.array_equal(v, vo) and np.array_equal(lin - 1, lino)
    assert np.array_equal(pk, pko) and np.array_equal(pl, plo) and np.array_equal(pc, pco)


def test_labor_infeasible_state_keeps_incoming(pkg, gpu):
    """A state whose cash on hand is below a_grid(1) for every labour level keeps v_new and the
    policies it came in with (:85)."""
    a = np.array([5.0, 6.0, 7.0])
    s = np.array([0.1])
    L = np.array([0.5, 1.0])
    v_in = np.full((1, 3), 42.0)
    pol = (np.full((1, 3), 1.5), np.full((1, 3), 2.5), np.full((1, 3), 3.5), np.full((1, 3), 7, np.int32))
    v, pk, pl, pc, lin = pkg.labor_vfi_sweep(np.zeros((1, 3)), a, s, np.ones((1, 1)), L, -0.5,
                                             1.0, 0.9, 5.0, 1.0, 2.0, v_new=v_in, policies=pol)
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(np.zeros((1, 3)), a, s, np.ones((1, 1)), L,
                                                    -0.5, 1.0, 0.9, 5.0, 1.0, 2.0,
                                                    v_new=v_in, pol=(pol[0], pol[1], pol[2], pol[3] - 1))
    assert np.array_equal(v, vo)
    assert np.array_equal(pk, pko) and np.array_equal(pl, plo) and np.array_equal(pc, pco)
    assert np.array_equal(lin - 1, lino)


@pytest.mark.parametrize("scale", [1e-9, 1e-2])
def test_labor_screen_stress_noisy_value(pkg, gpu, scale):
    """Noisy v_old (many near-ties across (l, a')) through the fp32/fp64 screen: bit-exact."""
    rng = np.random.default_rng(11)
    Na = 611
    cal = no.calib_aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    L = 0.01 + (1.5 - 0.01) * no.matlab_linspace01(10)
    w = no.wage(0.04, 0.36, 0.08)
    V = corc.labor_vfi_solve(np.zeros((7, Na)), a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0,
                             1e-5, 15)["v_new"]
    V = V + scale * rng.standard_normal(V.shape)
    v, pk, pl, pc, lin = pkg.labor_vfi_sweep(V, a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0)
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(V, a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0)
    assert np.array_equal(v, vo) and np.array_equal(lin - 1, lino)
    assert np.array_equal(pk, pko) and np.array_equal(pl, plo) and np.array_equal(pc, pco)


@pytest.mark.parametrize("max_iter", [40, 5])
def test_labor_solve_infeasible_states_keep_incoming(pkg, gpu, max_iter):
    """the host-tier labour solve runs speculative batches of sweeps on
    ring buffers; states with no feasible choice (Labor_VFI.m:85) must still end with the
    incoming v_new and policies, exactly as the literal loop (sweep, stop test, v_old = v_new)
    over the C oracle's sweep — for a stop inside a batch and for max_iter exhaustion."""
    a = np.array([0.5, 1.0, 2.0, 3.0, 4.5, 6.0, 8.0])
    s = np.array([0.2, 0.6])
    P = np.array([[0.7, 0.3], [0.4, 0.6]])
    L = np.array([0.4, 1.0])
    r, w, tol = -0.5, 1.0, 1e-6
    v0 = np.zeros((2, 7))
    v_in = np.full((2, 7), 42.0)
    pol = (np.full((2, 7), 1.5), np.full((2, 7), 2.5), np.full((2, 7), 3.5),
           np.full((2, 7), 3, np.int32))
    R = pkg.labor_vfi_solve(v0, a, s, P, L, r, w, 0.9, 5.0, 1.0, 2.0, tol, max_iter,
                            v_new=v_in, policies=pol)
    # the literal loop on the C oracle's sweep (lin 0-based there)
    v_old, v_new = v0.copy(), v_in.copy()
    p = (pol[0], pol[1], pol[2], pol[3] - 1)
    it = 0
    for it in range(1, max_iter + 1):
        v_new, p = corc.labor_vfi_sweep(v_old, a, s, P, L, r, w, 0.9, 5.0, 1.0, 2.0,
                                        v_new=v_new, pol=p)
        if np.nanmax(np.abs(v_new - v_old)) < tol:
            break
        v_old = v_new.copy()
    feasible = (1 + r) * a[None, :] + w * s[:, None] * L.max() > a[0]
    assert (~feasible).any() and feasible.any()
    assert R["iters"] == it
    assert np.array_equal(R["v_new"], v_new)
    assert np.array_equal(R["policy_k"], p[0]) and np.array_equal(R["policy_l"], p[1])
    assert np.array_equal(R["policy_c"], p[2]) and np.array_equal(R["lin"] - 1, p[3])
    assert np.all(R["v_new"][~feasible] == 42.0) and np.all(R["lin"][~feasible] == 3)


# 4096 (bit 12): the first superblock's passing 8-blocks split round-robin over the waves
@pytest.mark.parametrize("Na,variant", [(400, 16), (400, 2), (400, 4), (400, 6), (1100, 4),
                                        (2000, 18), (2000, 6), (400, 1024), (1100, 1024),
                                        (400, 4098), (400, 4100), (400, 4102), (1100, 4100),
                                        (2000, 4102), (100, 4100), (1100, 2064), (2000, 80),
                                        (5000, 2064), (5000, 80), (5000, 16 | 1 << 21),
                                        (1100, 4100 | 1 << 21), (5000, 16 | 1 << 21 | 1 << 23)])
def test_labor_cooperating_waves_vs_oracle(pkg, gpu, Na, variant):
    """Labour tree kernel with 1, 2, 4 and 8 cooperating waves per tile (variant bits 1-2; the
    Na <= 4096 default is 2 waves), and the exhaustive scan (bit 10): device-tier sweeps with the hint chain of a solve, then one
    sweep compared with the C oracle bit for bit (values, linear index, all three policies)."""
    import torch
    cal = no.calib_aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    L = 0.01 + (1.5 - 0.01) * no.matlab_linspace01(10)
    r = 0.04
    w = no.wage(r, 0.36, 0.08)
    dev = torch.device("cuda", 0)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t, L_t = t(a), t(s), t(P), t(L)
    ws = pkg.Workspace(7, Na, 10)
    ws.set_variant(variant)
    v = [torch.zeros((7, Na), dtype=torch.float64, device=dev) for _ in range(2)]
    lin = torch.zeros((7, Na), dtype=torch.int32, device=dev)
    pk, pl, pc = (torch.zeros((7, Na), dtype=torch.float64, device=dev) for _ in range(3))
    cur = 0
    for q in range(7):
        if q == 6:
            V = v[cur].cpu().numpy()
        ws.labor_vfi_sweep(v[cur], a_t, s_t, P_t, L_t, r, w, 0.96, 5.0, 1.0, 2.0, v[1 - cur], lin,
                           pk, pl, pc, hint=None if q == 0 else lin)
        cur = 1 - cur
    torch.cuda.synchronize()
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(V, a, s, P, L, r, w, 0.96, 5.0, 1.0, 2.0)
    assert np.array_equal(v[cur].cpu().numpy(), vo)
    assert np.array_equal(lin.cpu().numpy(), lino)
    assert np.array_equal(pk.cpu().numpy(), pko) and np.array_equal(pl.cpu().numpy(), plo)
    assert np.array_equal(pc.cpu().numpy(), pco)
