"""GPU parity for the small-grid one-launch sweep (csrc/bellman_wide_kernels.hip): A1
(Aiyagari_VFI.m:70-83) and A3 (Aiyagari_Endogenous_Labor_VFI.m:69-112) bit-exact against the
C oracle for every geometry (splits of the candidate range over workgroups, waves per
workgroup), cold and hinted, ragged tiles, near-tie value functions, the keep-incoming rule,
and solves through the speculative loop equal to the tree path's solves."""
import numpy as np
import pytest
import torch

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu

# (splits S, waves NW, states per wave SB)
GEOS = [(1, 16, 64), (1, 4, 64), (2, 8, 64), (3, 16, 64), (4, 4, 64), (8, 8, 64), (16, 16, 64),
        (1, 8, 32), (1, 8, 16), (1, 4, 8), (2, 8, 8), (3, 4, 16), (1, 16, 8)]


def _t(x, dev, dt=torch.float64):
    return torch.as_tensor(np.ascontiguousarray(x), device=dev, dtype=dt)


def _a1_state(Na, sweeps=6, sigma=5.0, noise=0.0, seed=3):
    cal = no.calib_aiyagari(Na=Na, sigma=sigma)
    w = no.wage(0.04, 0.36, 0.08)
    V = corc.vfi_solve(np.zeros((7, Na)), cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, sigma,
                       0.0, sweeps)["v_new"]
    if noise:
        V = V + noise * np.random.default_rng(seed).standard_normal(V.shape)
    return cal, w, V


def _a1_sweep(pkg, dev, cal, w, V, sigma, S, NW, SB=64, hint=None, wide=True):
    N, Na = V.shape
    ws = pkg.Workspace(N, Na)
    ws.set_wide(Na if wide else 0, S, NW, SB)
    vo, vn = _t(V, dev), torch.zeros((N, Na), dtype=torch.float64, device=dev)
    idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    pk, pc = torch.zeros_like(vn), torch.zeros_like(vn)
    diff = torch.zeros(2, dtype=torch.float64, device=dev)
    h = None if hint is None else _t(hint, dev, torch.int32)
    ws.vfi_sweep(vo, _t(cal["a_grid"], dev), _t(cal["s"], dev), _t(cal["P"], dev), 0.04, w, 0.96,
                 sigma, vn, idx, pk, pc, hint=h, mode=1, diff=diff)
    torch.cuda.synchronize()
    out = tuple(x.cpu().numpy() for x in (vn, idx, pk, pc, diff))
    ws.close()
    return out


@pytest.mark.parametrize("Na", [2, 37, 64, 65, 400, 1000, 2048])
@pytest.mark.parametrize("S,NW,SB", GEOS)
def test_a1_wide_sweep_vs_oracle(pkg, gpu, Na, S, NW, SB):
    cal, w, V = _a1_state(Na)
    vo, io, pko, pco = corc.vfi_sweep(V, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    for hint in (None, io, np.full_like(io, Na - 1), (io * 7919) % Na):  # cold / exact / far / junk
        v, idx, pk, pc, diff = _a1_sweep(pkg, gpu, cal, w, V, 5.0, S, NW, SB, hint=hint)
        assert np.array_equal(v, vo), (Na, S, NW, SB)
        assert np.array_equal(idx, io)
        assert np.array_equal(pk, pko) and np.array_equal(pc, pco)
        assert diff.view(np.uint64)[1] == 1 and diff[0] == np.max(np.abs(vo - V))


@pytest.mark.parametrize("sigma", [2.0, 3.0, 5.0, 9.0])
def test_a1_wide_other_sigmas(pkg, gpu, sigma):
    cal, w, V = _a1_state(333, sigma=sigma)
    vo, io, pko, pco = corc.vfi_sweep(V, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, sigma)
    for S, NW, SB in ((1, 16, 64), (4, 8, 64), (1, 8, 16), (2, 4, 8)):
        v, idx, pk, pc, _ = _a1_sweep(pkg, gpu, cal, w, V, sigma, S, NW, SB, hint=io)
        assert np.array_equal(v, vo) and np.array_equal(idx, io)
        assert np.array_equal(pk, pko) and np.array_equal(pc, pco)


@pytest.mark.parametrize("scale", [1e-12, 1e-9, 1e-3])
def test_a1_wide_near_ties(pkg, gpu, scale):
    """Noisy v_old: many near-ties in the screen and the merge (first index wins)."""
    cal, w, V = _a1_state(611, sweeps=20, noise=scale)
    vo, io, _, _ = corc.vfi_sweep(V, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    for S, NW, SB in GEOS:
        v, idx, _, _, _ = _a1_sweep(pkg, gpu, cal, w, V, 5.0, S, NW, SB, hint=io)
        assert np.array_equal(v, vo) and np.array_equal(idx, io), (S, NW, SB)
    # exact ties: a flat value function (every candidate value equal where feasible)
    Vf = np.zeros_like(V)
    vo, io, _, _ = corc.vfi_sweep(Vf, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    for S, NW, SB in ((2, 8, 64), (1, 8, 8)):
        v, idx, _, _, _ = _a1_sweep(pkg, gpu, cal, w, Vf, 5.0, S, NW, SB)
        assert np.array_equal(v, vo) and np.array_equal(idx, io)
    assert np.array_equal(v, vo) and np.array_equal(idx, io)


def _labor_sweep(pkg, dev, a, s, P, L, r, w, V, S, NW, SB=64, hint=None, v_in=None, pol=None,
                 sigma=5.0, eta=2.0, wide=True):
    N, Na = V.shape
    ws = pkg.Workspace(N, Na, len(L))
    ws.set_wide(Na if wide else 0, S, NW, SB)
    vn = _t(np.zeros((N, Na)) if v_in is None else v_in, dev)
    pol = pol or (np.zeros((N, Na)),) * 3 + (np.zeros((N, Na), np.int32),)
    pk, pl, pc = (_t(p, dev) for p in pol[:3])
    lin = _t(pol[3], dev, torch.int32)
    h = None if hint is None else _t(hint, dev, torch.int32)
    ws.labor_vfi_sweep(_t(V, dev), _t(a, dev), _t(s, dev), _t(P, dev), _t(L, dev), r, w, 0.96,
                       sigma, 1.0, eta, vn, lin, pk, pl, pc, hint=h)
    torch.cuda.synchronize()
    out = tuple(x.cpu().numpy() for x in (vn, lin, pk, pl, pc))
    ws.close()
    return out


@pytest.mark.parametrize("Na", [100, 400, 611])
@pytest.mark.parametrize("S,NW,SB", GEOS)
def test_labor_wide_sweep_vs_oracle(pkg, gpu, Na, S, NW, SB):
    cal = no.calib_aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    L = 0.01 + (1.5 - 0.01) * no.matlab_linspace01(10)
    w = no.wage(0.04, 0.36, 0.08)
    V = corc.labor_vfi_solve(np.zeros((7, Na)), a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0,
                             0.0, 9)["v_new"]
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(V, a, s, P, L, 0.04, w, 0.96, 5.0, 1.0, 2.0)
    for hint in (None, lino, (lino * 31) % (10 * Na)):
        v, lin, pk, pl, pc = _labor_sweep(pkg, gpu, a, s, P, L, 0.04, w, V, S, NW, SB, hint=hint)
        assert np.array_equal(v, vo) and np.array_equal(lin, lino), (Na, S, NW, SB)
        assert np.array_equal(pk, pko) and np.array_equal(pl, plo) and np.array_equal(pc, pco)


def test_labor_wide_unsorted_levels_sigma3(pkg, gpu):
    cal = no.calib_aiyagari(Na=257, rho=0.6, sigma_e=0.2, sigma=3.0)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    L = np.array([0.7, 0.05, 1.2, 0.3, 1.0, 0.5, 0.9])
    w = no.wage(0.03, 0.36, 0.08)
    V = corc.labor_vfi_solve(np.zeros((7, 257)), a, s, P, L, 0.03, w, 0.96, 3.0, 1.0, 1.5,
                             1e-5, 8)["v_new"]
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(V, a, s, P, L, 0.03, w, 0.96, 3.0, 1.0, 1.5)
    for S, NW, SB in ((1, 16, 64), (5, 4, 64), (1, 8, 8), (2, 4, 16)):
        v, lin, pk, pl, pc = _labor_sweep(pkg, gpu, a, s, P, L, 0.03, w, V, S, NW, SB, hint=lino,
                                          sigma=3.0, eta=1.5)
        assert np.array_equal(v, vo) and np.array_equal(lin, lino)
        assert np.array_equal(pk, pko) and np.array_equal(pl, plo) and np.array_equal(pc, pco)


def test_labor_wide_infeasible_keeps_incoming(pkg, gpu):
    a = np.array([5.0, 6.0, 7.0])
    s = np.array([0.1])
    L = np.array([0.5, 1.0])
    v_in = np.full((1, 3), 42.0)
    pol = (np.full((1, 3), 1.5), np.full((1, 3), 2.5), np.full((1, 3), 3.5), np.full((1, 3), 5, np.int32))
    vo, (pko, plo, pco, lino) = corc.labor_vfi_sweep(np.zeros((1, 3)), a, s, np.ones((1, 1)), L,
                                                    -0.5, 1.0, 0.9, 5.0, 1.0, 2.0, v_new=v_in,
                                                    pol=pol)
    for S, NW, SB in ((1, 16, 64), (2, 4, 64), (1, 4, 8)):
        v, lin, pk, pl, pc = _labor_sweep(pkg, gpu, a, s, np.ones((1, 1)), L, -0.5, 1.0,
                                          np.zeros((1, 3)), S, NW, SB, v_in=v_in, pol=pol)
        assert np.array_equal(v, vo) and np.array_equal(lin, lino)
        assert np.array_equal(pk, pko) and np.array_equal(pl, plo) and np.array_equal(pc, pco)


@pytest.mark.parametrize("Na", [400, 1500])
def test_wide_solve_equals_tree_solve(pkg, gpu, Na):
    """The A2 loop (speculative batches: diff slots folded by the next sweep's launch) on the
    wide path and on the tree path: same iteration count, v_new, v_old and policies."""
    cal = no.calib_aiyagari(Na=Na)
    w = no.wage(0.04, 0.36, 0.08)
    a_t, s_t, P_t = _t(cal["a_grid"], gpu), _t(cal["s"], gpu), _t(cal["P"], gpu)
    res = []
    for wide in (True, False):
        ws = pkg.Workspace(7, Na)
        ws.set_wide(Na if wide else 0)
        va = torch.zeros((7, Na), dtype=torch.float64, device=gpu)
        vb = torch.zeros_like(va)
        idx = torch.zeros((7, Na), dtype=torch.int32, device=gpu)
        pk, pc = torch.zeros_like(va), torch.zeros_like(va)
        it, which = ws.vfi_solve(va, vb, a_t, s_t, P_t, 0.04, w, 0.96, 5.0, 1e-5, 1000, idx, pk, pc,
                                 mode=1)
        torch.cuda.synchronize()
        res.append((it, which) + tuple(x.cpu().numpy() for x in (va, vb, idx, pk, pc)))
        ws.close()
    assert res[0][:2] == res[1][:2]
    for x, y in zip(res[0][2:], res[1][2:]):
        assert np.array_equal(x, y)
    if Na == 400:  # and the C oracle's loop
        R = corc.vfi_solve(np.zeros((7, Na)), cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
        assert res[0][0] == R["iters"]
        vnew = res[0][3] if res[0][1] else res[0][2]
        assert np.array_equal(vnew, R["v_new"])


def test_wide_and_tree_sweeps_alternate_on_one_workspace(pkg, gpu):
    """The diff slots of the two paths (a rotating pair for the wide launch, the table kernel's
    set for the tree) stay consistent when one workspace switches between them."""
    Na = 300
    cal, w, V = _a1_state(Na, sweeps=3)
    ws = pkg.Workspace(7, Na)
    a_t, s_t, P_t = _t(cal["a_grid"], gpu), _t(cal["s"], gpu), _t(cal["P"], gpu)
    v = [_t(V, gpu), torch.zeros((7, Na), dtype=torch.float64, device=gpu)]
    idx = torch.zeros((7, Na), dtype=torch.int32, device=gpu)
    diff = torch.zeros(2, dtype=torch.float64, device=gpu)
    Vc = V.copy()
    for g, wide in enumerate([True, True, False, True, False, False, True, True]):
        ws.set_wide(Na if wide else 0)
        ws.vfi_sweep(v[g & 1], a_t, s_t, P_t, 0.04, w, 0.96, 5.0, v[1 - (g & 1)], idx, mode=1,
                     hint=idx if g else None, diff=diff)
        torch.cuda.synchronize()
        vo, io, _, _ = corc.vfi_sweep(Vc, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
        got = v[1 - (g & 1)].cpu().numpy()
        assert np.array_equal(got, vo) and np.array_equal(idx.cpu().numpy(), io), g
        assert diff.cpu().numpy()[0] == np.max(np.abs(vo - Vc)), g
        Vc = vo
    ws.close()


def test_wide_counters(pkg, gpu):
    """The instrumented pass counts the wide launch's exact evaluations and candidate tests."""
    Na = 400
    cal, w, V = _a1_state(Na)
    ws = pkg.Workspace(7, Na)
    vo, io, _, _ = corc.vfi_sweep(V, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    ws.set_timing(False, count=True)
    vn = torch.zeros((7, Na), dtype=torch.float64, device=gpu)
    idx = torch.zeros((7, Na), dtype=torch.int32, device=gpu)
    ws.vfi_sweep(_t(V, gpu), _t(cal["a_grid"], gpu), _t(cal["s"], gpu), _t(cal["P"], gpu), 0.04, w,
                 0.96, 5.0, vn, idx, hint=_t(io, gpu, torch.int32), mode=1)
    torch.cuda.synchronize()
    ex, sup, blk, cand = ws.counters()
    ws.close()
    feas = sum(int(np.searchsorted(cal["a_grid"], (1.04) * cal["a_grid"] + w * si).sum())
               for si in cal["s"])
    assert ex >= 7 * Na             # at least the bar of every state
    # every feasible candidate is covered by a block bound (one per 8) or screened itself
    assert feas // 8 <= cand <= 2 * feas
    assert np.array_equal(vn.cpu().numpy(), vo)
