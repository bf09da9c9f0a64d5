"""Chained sweeps: the tree kernel of sweep g builds sweep g+1's table from the v_new it writes
(BellArgs::nEV, `chain_table_tile`), so a chain of A1 sweeps (Aiyagari_VFI.m:70-83 repeated, the
A2 loop :65-90 without its stop test) is one launch per sweep after the first.

Chaining is opt-in (ws.set_chain(True); measured slower than a table launch per sweep at
Na = 20,000).  Bit for bit against one table launch per sweep (the default) and against the C oracle's
exhaustive sweep of the device's own v_old: the table the last arriver of each 64-candidate tile
builds (EV in m order, D, the 8- and 64-block maxima) must equal bell_table_kernel's, and the
level-0 bounds taken from the 64-block maxima may change which blocks are screened, never the
result.  Sizes: the benched Na = 20,000 (partial last tile: 20,000 = 312·64 + 32), Na just above
the 4,096 default switch, small grids with the one-wave geometry forced (variant 0), N from 2 to
kChainMaxN = 16, sigma 2 / 3 / 5 (NP = 1, 2, 4 instantiations), cold starts and hinted starts.
"""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def _setup(pkg, torch, cal, r):
    dev = torch.device("cuda:0")
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    return t(cal["a_grid"]), t(cal["s"]), t(cal["P"]), w


def _run(pkg, torch, cal, nsweeps, chain, sigma=None, variant=-1, per_call=False, r=0.04,
         ws=None, repeat=1):
    """nsweeps sweeps from v = 0 (sweep 1 cold, later sweeps hinted by idx); returns the final
    (v_new, v_old, idx, pk, pc, diff) of the last of `repeat` identical runs on one workspace."""
    a, s, P, w = _setup(pkg, torch, cal, r)
    N, Na = cal["N"], cal["Na"]
    sig = cal["sigma"] if sigma is None else sigma
    if ws is None:
        ws = pkg.Workspace(N, Na)
        ws.set_chain(chain)
        if variant >= 0:
            ws.set_variant(variant)
    dev = a.device
    for _ in range(repeat):
        v = [torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(2)]
        idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
        pk = torch.empty((N, Na), dtype=torch.float64, device=dev)
        pc = torch.empty_like(pk)
        diff = torch.zeros(2, dtype=torch.float64, device=dev)
        if per_call:
            cur = 0
            for g in range(nsweeps):
                ws.vfi_sweep(v[cur], a, s, P, r, w, cal["beta"], sig, v[1 - cur], idx, pk, pc,
                             hint=None if g == 0 else idx, mode=1,
                             diff=diff if g == nsweeps - 1 else None)
                cur = 1 - cur
        else:
            ws.vfi_sweeps(v[0], v[1], a, s, P, r, w, cal["beta"], sig, nsweeps, idx, pk, pc,
                          hint=None, mode=1, diff=diff)
        torch.cuda.synchronize()
    new = nsweeps & 1
    return dict(v_new=v[new].cpu().numpy(), v_old=v[1 - new].cpu().numpy(),
                idx=idx.cpu().numpy(), pk=pk.cpu().numpy(), pc=pc.cpu().numpy(),
                diff=diff.cpu().numpy().view(np.uint64).copy()), ws


def _same(x, y):
    for k in ("v_new", "v_old", "idx", "pk", "pc", "diff"):
        a, b = x[k], y[k]
        if a.dtype.kind == "f":
            assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), k
        else:
            assert np.array_equal(a, b), k


def _oracle_last_sweep(cal, out, sigma=None, r=0.04):
    w = no.wage(r, cal["alpha"], cal["delta"])
    sig = cal["sigma"] if sigma is None else sigma
    v, idx, pk, pc = corc.vfi_sweep(out["v_old"], cal["a_grid"], cal["s"], cal["P"], r, w,
                                    cal["beta"], sig)
    assert np.array_equal(out["v_new"].view(np.uint64), v.view(np.uint64))
    assert np.array_equal(out["idx"], idx)
    assert np.array_equal(out["pk"].view(np.uint64), pk.view(np.uint64))
    assert np.array_equal(out["pc"].view(np.uint64), pc.view(np.uint64))


def test_chain_bench_config_bitwise(pkg, gpu):
    """bench.py's timed path: 25 chained sweeps at Na = 20,000 == 25 separate sweeps, and the
    25th equals the oracle sweep of its v_old."""
    import torch
    cal = no.calib_aiyagari(Na=20000, shocks="rouwenhorst")
    ch, _ = _run(pkg, torch, cal, 25, True)
    sep, _ = _run(pkg, torch, cal, 25, False, per_call=True)
    _same(ch, sep)
    _oracle_last_sweep(cal, ch)


@pytest.mark.parametrize("Na,variant,shocks,N", [
    (4160, -1, "rouwenhorst", 7),   # whole tiles, one wave per tile by default (Na > 4096)
    (4097, -1, "tauchen", 7),       # one state in the last tile
    (6000, -1, "tauchen", 7),
    (300, 0, "rouwenhorst", 7),     # small grid, one-wave geometry forced
    (1000, 16, "rouwenhorst", 3),
    (700, 0, "rouwenhorst", 2),
    (513, 0, "rouwenhorst", 16),    # kChainMaxN rows per tile
])
def test_chain_equals_table_per_sweep(pkg, gpu, Na, variant, shocks, N):
    import torch
    cal = no.calib_aiyagari(Na=Na, shocks=shocks, N=N)
    ch, _ = _run(pkg, torch, cal, 12, True, variant=variant)
    sep, _ = _run(pkg, torch, cal, 12, False, variant=variant)
    _same(ch, sep)
    _oracle_last_sweep(cal, ch)


@pytest.mark.parametrize("sigma", [2.0, 3.0])
def test_chain_other_sigma(pkg, gpu, sigma):
    """NP = 1 and 2 (the tree kernel's one-wave instantiations outside the tuned NP = 4)."""
    import torch
    cal = no.calib_aiyagari(Na=5000, shocks="rouwenhorst")
    ch, _ = _run(pkg, torch, cal, 9, True, sigma=sigma)
    sep, _ = _run(pkg, torch, cal, 9, False, sigma=sigma)
    _same(ch, sep)
    _oracle_last_sweep(cal, ch, sigma=sigma)


def test_chain_counters_rearm(pkg, gpu):
    """Three chains on one workspace (the per-tile arrival counters are re-armed by the last
    arriver and the slot ring is cleared ahead): every run equals a fresh unchained run."""
    import torch
    cal = no.calib_aiyagari(Na=8192, shocks="rouwenhorst")
    ref, _ = _run(pkg, torch, cal, 7, False)
    out, ws = _run(pkg, torch, cal, 7, True, repeat=3)
    _same(out, ref)
    out2, _ = _run(pkg, torch, cal, 7, True, ws=ws)
    _same(out2, ref)


def test_chain_single_sweep_and_fallbacks(pkg, gpu):
    """nsweeps = 1 (table launch + one tree launch) and geometries that cannot chain (W = 2,
    N > 16) take the table-per-sweep path with the same results."""
    import torch
    cal = no.calib_aiyagari(Na=5000, shocks="tauchen")
    one, _ = _run(pkg, torch, cal, 1, True)
    ref, _ = _run(pkg, torch, cal, 1, False, per_call=True)
    _same(one, ref)
    w2, _ = _run(pkg, torch, cal, 6, True, variant=2 | 16)
    ref2, _ = _run(pkg, torch, cal, 6, False, per_call=True)
    _same(w2, ref2)
    cal17 = no.calib_aiyagari(Na=600, shocks="rouwenhorst", N=17)
    a17, _ = _run(pkg, torch, cal17, 5, True, variant=0)
    b17, _ = _run(pkg, torch, cal17, 5, False, variant=0, per_call=True)
    _same(a17, b17)


def test_chain_solve_equals_unchained(pkg, gpu):
    """The speculative solve runs one chain per solve: iterations, v_new / v_old and policies
    equal the table-per-sweep solve at the benched size."""
    import torch
    cal = no.calib_aiyagari(Na=20000, shocks="rouwenhorst")
    a, s, P, w = _setup(pkg, torch, cal, 0.04)
    N, Na = cal["N"], cal["Na"]
    res = []
    for chain in (True, False):
        ws = pkg.Workspace(N, Na)
        ws.set_chain(chain)
        va = torch.zeros((N, Na), dtype=torch.float64, device=a.device)
        vb = torch.zeros_like(va)
        idx = torch.zeros((N, Na), dtype=torch.int32, device=a.device)
        pk, pc = torch.empty_like(va), torch.empty_like(va)
        it, which = ws.vfi_solve(va, vb, a, s, P, 0.04, w, cal["beta"], cal["sigma"], 1e-5, 1000,
                                 idx, pk, pc, mode=1)
        torch.cuda.synchronize()
        res.append((it, which, va.cpu().numpy(), vb.cpu().numpy(), idx.cpu().numpy(),
                    pk.cpu().numpy(), pc.cpu().numpy()))
    assert res[0][:2] == res[1][:2]
    for x, y in zip(res[0][2:], res[1][2:]):
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8))


@pytest.mark.parametrize("Na", [5000, 20000])
def test_reversed_xcd_order_bitwise(pkg, gpu, Na):
    """Variant bit 17 (each XCD's tile range dealt in reverse) changes the work order only: the
    sweeps equal the default order bit for bit, unchained and chained."""
    import torch
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst")
    ref, _ = _run(pkg, torch, cal, 10, False, variant=16)
    rev, _ = _run(pkg, torch, cal, 10, False, variant=16 | 131072)
    _same(rev, ref)
    revc, _ = _run(pkg, torch, cal, 10, True, variant=16 | 131072)
    _same(revc, ref)
    _oracle_last_sweep(cal, rev)
