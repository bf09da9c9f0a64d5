"""Parity pinned in the configurations the benchmarks run, and the size gaps of round 1.

* The headline path exactly as bench.py drives it (BASELINE configs[1]: Aiyagari_VFI.m:70-83 at
  Na = 20,000, Nz = 7 Rouwenhorst, device tier, default geometry, `hint` aliased to the output
  index buffer, a solve from v = 0): after 24 sweeps, sweep 25 — one of the timed sweeps — is
  compared bit for bit with the C oracle's exhaustive sweep of the same input.
* The 249-sweep solve to tol at that size (bench.py's solve_to_tol leg, A2 :65-90): its v_new
  must be the oracle sweep of its v_old, bit for bit, with the break semantics of :85-88.
* The labour VFI (A3, Aiyagari_Endogenous_Labor_VFI.m:69-112) for one sweep at Na = 20,000.
* The histogram stationary distribution (A10) at Na = 20,000 against the C restatement.
* F4 (Aiyagari_VFI.m:314-410) on HIP-produced outputs: Gini / quintiles of the A9 Monte-Carlo
  path and of the A10 histogram, against the same statistics of the oracle-composed pipeline.
"""
import os

import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu

NA = 20000


@pytest.fixture(scope="module")
def cal20k():
    return no.calib_aiyagari(Na=NA, shocks="rouwenhorst")


def _bench_tensors(pkg, cal, torch):
    dev = torch.device("cuda:0")
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    return t(cal["a_grid"]), t(cal["s"]), t(cal["P"])


def test_bench_device_path_sweep25_bitwise(pkg, gpu, cal20k):
    """bench.py's step(): ws.vfi_sweep(v[cur], ..., v[1-cur], idx, pk, pc, hint=idx)."""
    import torch
    cal = cal20k
    N = cal["N"]
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    a_t, s_t, P_t = _bench_tensors(pkg, cal, torch)
    dev = a_t.device
    v = [torch.zeros((N, NA), dtype=torch.float64, device=dev) for _ in range(2)]
    idx = torch.zeros((N, NA), dtype=torch.int32, device=dev)
    pk = torch.empty((N, NA), dtype=torch.float64, device=dev)
    pc = torch.empty_like(pk)
    ws = pkg.Workspace(N, NA)
    ws.set_search(0, 1024)   # bench.py's setting; the geometry stays the default (variant -1)
    cur = 0
    for q in range(25):
        if q == 24:
            torch.cuda.synchronize()
            v_in = v[cur].cpu().numpy()
        ws.vfi_sweep(v[cur], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], v[1 - cur], idx, pk,
                     pc, hint=None if q == 0 else idx, mode=1)
        cur = 1 - cur
    torch.cuda.synchronize()
    vo, io, pko, pco = corc.vfi_sweep(v_in, cal["a_grid"], cal["s"], cal["P"], r, w, cal["beta"],
                                      cal["sigma"])
    assert np.array_equal(v[cur].cpu().numpy(), vo)
    assert np.array_equal(idx.cpu().numpy(), io)
    assert np.array_equal(pk.cpu().numpy(), pko) and np.array_equal(pc.cpu().numpy(), pco)


def test_batch_config4_share_sweep25_bitwise(pkg, gpu, cal20k):
    """bench_legs.batch_leg's exact path (BASELINE configs[3] per-GPU share, Aiyagari_VFI.m:
    142-171): 8 rates linspace(-0.03, 0.035) solved as ONE batched solve at Na = 20,000
    Rouwenhorst from v = 0 with tol = 0 (no early stop).  The batch is run for 24 sweeps, each
    candidate's V copied back, then re-run from v = 0 for 25: every candidate's sweep 25
    (v_new, argmax, policy_k, policy_c) must equal the C oracle's exhaustive sweep of its own
    sweep-24 value bit for bit."""
    import torch
    cal = cal20k
    N = cal["N"]
    C = 8
    a_t, s_t, P_t = _bench_tensors(pkg, cal, torch)
    dev = a_t.device
    rs = list(np.linspace(-0.03, 0.035, C))
    w = [pkg.calibration.wage(r, cal["alpha"], cal["delta"]) for r in rs]
    ws = pkg.Workspace(N, NA)

    def run(sweeps):
        va = torch.zeros((C, N, NA), dtype=torch.float64, device=dev)
        vb = torch.zeros_like(va)
        idx = torch.zeros((C, N, NA), dtype=torch.int32, device=dev)
        pk, pc = torch.zeros_like(va), torch.zeros_like(va)
        it, which = pkg.vfi.solve_batch_dev(ws, rs, w, va, vb, a_t, s_t, P_t, cal["beta"],
                                            cal["sigma"], 0.0, sweeps, idx, pk, pc)
        torch.cuda.synchronize()
        assert it == [sweeps] * C
        vn = [(vb if which[c] else va)[c].cpu().numpy() for c in range(C)]
        return vn, idx.cpu().numpy(), pk.cpu().numpy(), pc.cpu().numpy()

    v24, _, _, _ = run(24)
    v25, idx, pk, pc = run(25)
    corc.num_threads(min(16, os.cpu_count() or 1))  # 8 exhaustive sweeps of 2.8e9 candidates
    for c in range(C):
        vo, io, pko, pco = corc.vfi_sweep(v24[c], cal["a_grid"], cal["s"], cal["P"], rs[c], w[c],
                                          cal["beta"], cal["sigma"])
        assert np.array_equal(v25[c], vo), c
        assert np.array_equal(idx[c], io), c
        assert np.array_equal(pk[c], pko) and np.array_equal(pc[c], pco), c


def test_solve_to_tol_full_size_fixed_point(pkg, gpu, cal20k):
    """bench.py's solve_to_tol leg: 249 sweeps (speculative batches), then v_new == T(v_old)."""
    import torch
    cal = cal20k
    N = cal["N"]
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    a_t, s_t, P_t = _bench_tensors(pkg, cal, torch)
    dev = a_t.device
    va = torch.zeros((N, NA), dtype=torch.float64, device=dev)
    vb = torch.zeros_like(va)
    idx = torch.zeros((N, NA), dtype=torch.int32, device=dev)
    pk, pc = torch.empty_like(va), torch.empty_like(va)
    ws = pkg.Workspace(N, NA)
    iters, which = ws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5,
                                1000, idx, pk, pc, mode=1)
    torch.cuda.synchronize()
    v_new = (vb if which else va).cpu().numpy()
    v_old = (va if which else vb).cpu().numpy()
    assert iters == 249
    vo, io, pko, pco = corc.vfi_sweep(v_old, cal["a_grid"], cal["s"], cal["P"], r, w,
                                      cal["beta"], cal["sigma"])
    assert np.array_equal(v_new, vo)
    assert np.array_equal(idx.cpu().numpy(), io)
    assert np.array_equal(pk.cpu().numpy(), pko) and np.array_equal(pc.cpu().numpy(), pco)
    assert np.max(np.abs(v_new - v_old)) < 1e-5  # :85 (v_old kept the previous iterate)
    assert (pc.cpu().numpy() > 0).all()


def test_labor_sweep_full_size(pkg, gpu):
    """A3 at Na = 20,000 (D4 size): one sweep bit-exact vs the C oracle, V interpolated from the
    Na = 400 labour solution (smooth, non-trivial)."""
    cal = no.calib_aiyagari(Na=NA, rho=0.6, sigma_e=0.2)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    L = 0.01 + (1.5 - 0.01) * no.matlab_linspace01(10)
    w = no.wage(0.04, 0.36, 0.08)
    c4 = no.calib_aiyagari(Na=400, rho=0.6, sigma_e=0.2)
    V4 = corc.labor_vfi_solve(np.zeros((7, 400)), c4["a_grid"], c4["s"], c4["P"], L, 0.04, w,
                              0.96, 5.0, 1.0, 2.0)["v_new"]
    V = np.stack([np.interp(a, c4["a_grid"], V4[i]) for i in range(7)])
    v, pk, pl, pc, lin = pkg.labor_vfi_sweep(V, a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0)
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(V, a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0)
    assert np.array_equal(v, vo) and np.array_equal(lin - 1, lino)
    assert np.array_equal(pk, pko) and np.array_equal(pl, plo) and np.array_equal(pc, pco)


def test_dist_stationary_full_size(pkg, gpu, cal20k):
    """A10 at Na = 20,000: the on-grid histogram fixed point of a config-2 policy, bit-exact vs
    the C restatement (the same additions in the same order)."""
    cal = cal20k
    w = no.wage(0.04, 0.36, 0.08)
    c4 = no.calib_aiyagari(Na=400, shocks="rouwenhorst")
    V4 = corc.vfi_solve(np.zeros((7, 400)), c4["a_grid"], c4["s"], c4["P"], 0.04, w, 0.96,
                        5.0)["v_new"]
    V = np.stack([np.interp(cal["a_grid"], c4["a_grid"], V4[i]) for i in range(7)])
    _, idx, _, _ = corc.vfi_sweep(V, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    lam0 = np.full((7, NA), 1.0 / (7 * NA))
    lam, K, it, dist = pkg.dist_stationary(cal["a_grid"], cal["P"], policy_idx=idx + 1,
                                           lam0=lam0, tol=1e-13, max_iter=3000)
    lo, Ko, ito, disto = corc.dist_stationary(lam0, cal["a_grid"], cal["P"], idx=idx, tol=1e-13,
                                              max_iter=3000)
    assert it == ito and np.array_equal(lam, lo)
    assert abs(K - Ko) <= 1e-12 * abs(Ko)
    assert abs(lam.sum() - 1.0) < 1e-9 and (lam >= 0).all()


def test_f4_statistics_on_hip_outputs(pkg, gpu, golden):
    """Aiyagari_VFI.m:314-410 evaluated on what the HIP pipeline produced — the MC capital path
    (A9, MATLAB's rand stream) and the histogram λ (A10) — equal the statistics of the
    oracle-composed pipeline (C restatement for every stage) exactly."""
    g = golden("a11_ge_vfi_defaults")
    cal = no.calib_aiyagari()
    w = no.wage(0.04, 0.36, 0.08)
    R = pkg.vfi_solve(np.zeros((7, 400)), cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    Ro = corc.vfi_solve(np.zeros((7, 400)), cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    U = no.matlab_rand_stream(2 + 9999)       # randi(N), randi(Na), then :106's draws
    z1, k1 = int(g["z1"]) + 1, float(g["k1"])  # the fixture stores z1 0-based
    Ks, path, _ = pkg.sim_capital(R["policy_k"], cal["a_grid"], cal["P"], z1, k1, U[2:],
                                  return_path=True)
    Kso, patho = corc.sim_capital(Ro["policy_k"], cal["a_grid"], cal["P"], z1 - 1, k1, U[2:],
                                  return_path=True)
    assert Ks == float(g["Ks0"])
    assert np.array_equal(path, patho) and np.array_equal(path, g["sim_k0"])
    st, sto = pkg.stats.inequality_report(path), pkg.stats.inequality_report(patho)
    assert st == sto
    assert 0 < st["gini_wealth"] < 1 and abs(sum(st["wealth_quintile_shares"]) - 100) < 1e-9
    lam0 = np.full((7, 400), 1.0 / 2800)
    lam, _, _, _ = pkg.dist_stationary(cal["a_grid"], cal["P"], policy_idx=R["idx"], lam0=lam0,
                                       tol=1e-13, max_iter=5000)
    lo, _, _, _ = corc.dist_stationary(lam0, cal["a_grid"], cal["P"], idx=Ro["idx"], tol=1e-13,
                                       max_iter=5000)
    h, ho = (pkg.stats.histogram_wealth_stats(x, cal["a_grid"]) for x in (lam, lo))
    assert h == ho and 0 < h["gini_wealth"] < 1
