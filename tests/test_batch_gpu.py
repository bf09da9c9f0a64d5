"""Config 4 (BASELINE configs[3]): C candidate rates in one batched solve.

aiy_vfi_solve_batch_dev must give, for every candidate, exactly what a separate A2 solve
(Aiyagari_VFI.m:147-171 from the same v_old) gives: iteration count, v_new, v_old (break
semantics of :85-88, or v_old = v_new when max_iter is exhausted), argmax and policies.
aiy_ge_batch adds the Monte-Carlo supply (:174-193, MATLAB's rand stream, each candidate its own
block) and K_d (:195); its results equal the sequential evaluator's, and the multisection
trace driven by it equals the reference loop's golden trace."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def _batch_vs_single(pkg, torch, cal, rs, v0, max_iter=1000, sigma=5.0, hint=None):
    dev = torch.device("cuda:0")
    N, Na = cal["N"], cal["Na"]
    C = len(rs)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a, s, P = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    ws = [pkg.Workspace(N, Na), pkg.Workspace(N, Na)]
    w = np.array([pkg.calibration.wage(r, cal["alpha"], cal["delta"]) for r in rs])
    va = t(np.broadcast_to(v0, (C, N, Na)).copy())
    vb = torch.zeros_like(va)
    idx = t(np.broadcast_to(hint, (C, N, Na)).copy()) if hint is not None else \
        torch.zeros((C, N, Na), dtype=torch.int32, device=dev)
    pk, pc = torch.zeros_like(va), torch.zeros_like(va)
    it, which = pkg.vfi.solve_batch_dev(ws[0], rs, w, va, vb, a, s, P, cal["beta"], sigma, 1e-5,
                                        max_iter, idx, pk, pc, use_hint=hint is not None)
    torch.cuda.synchronize()
    for c in range(C):
        sa, sb = t(v0.copy()), torch.zeros((N, Na), dtype=torch.float64, device=dev)
        sidx = t(hint.copy()) if hint is not None else torch.zeros((N, Na), dtype=torch.int32, device=dev)
        spk, spc = torch.zeros_like(sa), torch.zeros_like(sa)
        # the single-rate solve with the same first hint (it uses idx as the hint from sweep 2)
        i1, w1 = ws[1].vfi_solve(sa, sb, a, s, P, rs[c], w[c], cal["beta"], sigma, 1e-5,
                                 max_iter, sidx, spk, spc, mode=0)
        torch.cuda.synchronize()
        assert it[c] == i1 and which[c] == w1, (c, it[c], i1)
        vn_b = (vb if which[c] else va)[c].cpu().numpy()
        vo_b = (va if which[c] else vb)[c].cpu().numpy()
        vn_s = (sb if w1 else sa).cpu().numpy()
        vo_s = (sa if w1 else sb).cpu().numpy()
        assert np.array_equal(vn_b, vn_s) and np.array_equal(vo_b, vo_s), c
        assert np.array_equal(idx[c].cpu().numpy(), sidx.cpu().numpy()), c
        assert np.array_equal(pk[c].cpu().numpy(), spk.cpu().numpy()), c
        assert np.array_equal(pc[c].cpu().numpy(), spc.cpu().numpy()), c
    return it


@pytest.mark.parametrize("Na", [400, 1500, 5000])
def test_batch_equals_separate_solves(pkg, gpu, Na):
    import torch
    cal = pkg.calibration.aiyagari(Na=Na)
    rng = np.random.default_rng(Na)
    rs = list(rng.uniform(-0.05, 1 / cal["beta"] - 1, 6)) + [0.04]
    it = _batch_vs_single(pkg, torch, cal, rs, np.zeros((7, Na)))
    assert len(set(it)) > 1  # candidates stop at different sweeps


def test_batch_warm_start_exhaustion_and_hint(pkg, gpu):
    """Warm start from a converged V (a candidate at its own r stops at sweep 1), max_iter
    exhausted for the others (v_old = v_new), and a starting hint."""
    import torch
    cal = pkg.calibration.aiyagari(Na=400)
    w0 = pkg.calibration.wage(0.04, cal["alpha"], cal["delta"])
    R0 = corc.vfi_solve(np.zeros((7, 400)), cal["a_grid"], cal["s"], cal["P"], 0.04, w0,
                        cal["beta"], cal["sigma"])
    v0 = R0["v_new"]
    rs = [0.04, 0.0, 0.02, -0.03]
    it = _batch_vs_single(pkg, torch, cal, rs, v0, max_iter=9)
    assert it[0] == 1 and max(it) == 9
    _batch_vs_single(pkg, torch, cal, rs, R0["v_old"], hint=R0["idx"].astype(np.int32))


def test_batch_generic_sigma_falls_back_exactly(pkg, gpu):
    import torch
    cal = pkg.calibration.aiyagari(Na=300, sigma=2.5)
    _batch_vs_single(pkg, torch, cal, [0.01, 0.03], np.zeros((7, 300)), max_iter=12, sigma=2.5)


def test_ge_batch_host_tier_matches_sequential_evaluator(pkg, gpu):
    gb = pkg.ge_batch
    cal = pkg.calibration.aiyagari(Na=400)
    w0 = pkg.calibration.wage(0.04, cal["alpha"], cal["delta"])
    v0 = corc.vfi_solve(np.zeros((7, 400)), cal["a_grid"], cal["s"], cal["P"], 0.04, w0,
                        cal["beta"], cal["sigma"])["v_old"]
    nodes = gb.subtree(-0.05, 1 / cal["beta"] - 1, 1, 3)  # 7 candidates, depths 1..3

    def solve(v, r, w):
        return corc.vfi_solve(v, cal["a_grid"], cal["s"], cal["P"], r, w, cal["beta"], cal["sigma"])

    def simulate(pk, z1, k1, u):
        return corc.sim_capital(pk, cal["a_grid"], cal["P"], z1 - 1, k1, u)
    seq = gb.vfi_evaluator(cal, solve, simulate, v0)
    bat = gb.hip_batch_evaluator(cal, v0)
    out = bat.many(nodes)
    for n, o in zip(nodes, out):
        assert o == seq(n), n


def test_multisection_batched_matches_golden(pkg, gpu, golden):
    gb = pkg.ge_batch
    A = gb.aiyagari_vfi_multisection(levels=6, batched=True)
    B = gb.aiyagari_vfi_multisection(levels=6, batched=False)
    assert A.r_history == B.r_history and A.k_supply == B.k_supply and A.iters == B.iters
    g = golden("a11_ge_vfi_defaults")
    assert A.r_history == [float(x) for x in g["r_history"]] and A.r == float(g["r_final"])


def test_ge_batch_rejects_bad_input(pkg, gpu):
    gb = pkg.ge_batch
    cal = pkg.calibration.aiyagari(Na=50)
    v = np.zeros((7, 50))
    with pytest.raises(pkg.AiyError):
        gb.ge_batch_call([0.02], v, cal, 9, cal["a_grid"][0], [np.full(99, 0.5)])  # z1 > N
    bad = dict(cal)
    bad["a_grid"] = cal["a_grid"].copy()
    bad["a_grid"][5] = bad["a_grid"][4]  # repeated grid point (interp1 would error)
    with pytest.raises(pkg.AiyError):
        gb.ge_batch_call([0.02], v, bad, 1, bad["a_grid"][0], [np.full(99, 0.5)])
