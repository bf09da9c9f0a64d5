"""A2 (Aiyagari_VFI.m:65-90) speculative solve: sweeps enqueued in batches between reads of
max|Δv| (aiy_ws_set_speculation) must give exactly the one-sync-per-sweep loop's results —
iteration count, which buffer holds v_new, v_new, v_old (break before `v_old = v_new`, or
`v_old = v_new` after max_iter), the argmax and both policies — for every batch cap, including
ring wrap-around (cap < sweeps), exhaustion inside a batch, a stop on the first sweep, and the
plain (non-screened) sweep.  The host tier runs the default cap and is pinned to the golden
fixtures by test_vfi_gpu.py / test_labor_gpu.py."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def _solve(pkg, torch, spec, v0, cal, r, sigma, tol, max_iter, mode=0, v_b=None):
    dev = torch.device("cuda:0")
    N, Na = v0.shape
    ws = pkg.Workspace(N, Na)
    ws.set_speculation(spec)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    va, at, st, Pt = t(v0), t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    vb = torch.zeros_like(va) if v_b is None else t(v_b)
    pk = torch.empty_like(va); pc = torch.empty_like(va)
    idx = torch.empty((N, Na), dtype=torch.int32, device=dev)
    w = no.wage(r, 0.36, 0.08)
    it, which = ws.vfi_solve(va, vb, at, st, Pt, r, w, 0.96, sigma, tol, max_iter, idx, pk, pc,
                             mode=mode)
    torch.cuda.synchronize()
    bufs = (va.cpu().numpy(), vb.cpu().numpy())
    out = dict(iters=it, which=which, v_new=bufs[which], v_old=bufs[1 - which],
               idx=idx.cpu().numpy(), pk=pk.cpu().numpy(), pc=pc.cpu().numpy())
    ws.close()
    return out


def _same(A, B):
    assert A["iters"] == B["iters"] and A["which"] == B["which"]
    for k in ("v_new", "v_old", "idx", "pk", "pc"):
        assert np.array_equal(A[k], B[k], equal_nan=True), k


@pytest.mark.parametrize("max_iter", [1000, 7, 1])
def test_speculative_equals_synchronous(pkg, gpu, max_iter):
    import torch
    cal = no.calib_aiyagari(Na=400)
    v0 = np.zeros((7, 400))
    ref = _solve(pkg, torch, 0, v0, cal, 0.04, 5.0, 1e-5, max_iter)
    for spec in (2, 3, 16, 64):  # the speculative host loop (default)
        _same(_solve(pkg, torch, spec, v0, cal, 0.04, 5.0, 1e-5, max_iter), ref)
    if max_iter == 1000:  # and both equal the C oracle's solve
        R = corc.vfi_solve(v0, cal["a_grid"], cal["s"], cal["P"], 0.04, no.wage(0.04, 0.36, 0.08),
                           0.96, 5.0, 1e-5, 1000)
        assert R["iters"] == ref["iters"]
        assert np.array_equal(R["v_new"], ref["v_new"]) and np.array_equal(R["v_old"], ref["v_old"])
        assert np.array_equal(R["idx"], ref["idx"])


def test_speculative_warm_start_and_first_sweep_stop(pkg, gpu):
    import torch
    cal = no.calib_aiyagari(Na=777, shocks="rouwenhorst")
    w = no.wage(0.03, 0.36, 0.08)
    V = corc.vfi_solve(np.zeros((7, 777)), cal["a_grid"], cal["s"], cal["P"], 0.03, w, 0.96, 5.0,
                       1e-9, 1000)["v_new"]
    # warm start near the fixed point: stop on sweep 1 or 2
    for tol in (1e-5, 1e-12):
        ref = _solve(pkg, torch, 0, V, cal, 0.03, 5.0, tol, 1000, v_b=V + 1.0)
        for spec in (2, 16):
            _same(_solve(pkg, torch, spec, V, cal, 0.03, 5.0, tol, 1000, v_b=V + 1.0), ref)


@pytest.mark.parametrize("sigma,mode", [(2.5, 0), (5.0, 2)])
def test_speculative_plain_sweep(pkg, gpu, sigma, mode):
    import torch
    cal = no.calib_aiyagari(Na=300, sigma=sigma)
    v0 = np.zeros((7, 300))
    ref = _solve(pkg, torch, 0, v0, cal, 0.03, sigma, 1e-5, 1000, mode=mode)
    _same(_solve(pkg, torch, 5, v0, cal, 0.03, sigma, 1e-5, 1000, mode=mode), ref)


def test_set_speculation_validates(pkg, gpu):
    ws = pkg.Workspace(7, 100)
    with pytest.raises(Exception):
        ws.set_speculation(-1)
    with pytest.raises(Exception):
        ws.set_speculation(1000)
    ws.set_speculation(0)
    ws.set_speculation(1)
    ws.close()


@pytest.mark.parametrize("Na,sigma,max_iter", [(4096, 5.0, 60), (1000, 3.0, 400), (64, 2.0, 1000),
                                               (2500, 9.0, 37)])
def test_speculative_solve_sizes(pkg, gpu, Na, sigma, max_iter):
    """The speculative solve across grid sizes (one to 448 tree items, one to eight
    512-candidate table chunks per row) and CRRA powers: equal to the synchronous loop, and —
    run to tol — to the C oracle's solve."""
    import torch
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst", sigma=sigma)
    v0 = np.zeros((7, Na))
    ref = _solve(pkg, torch, 0, v0, cal, 0.03, sigma, 1e-5, max_iter)
    got = _solve(pkg, torch, 16, v0, cal, 0.03, sigma, 1e-5, max_iter)
    _same(got, ref)
    R = corc.vfi_solve(v0, cal["a_grid"], cal["s"], cal["P"], 0.03, no.wage(0.03, 0.36, 0.08),
                       0.96, sigma, 1e-5, max_iter)
    assert R["iters"] == got["iters"]
    assert np.array_equal(R["v_new"], got["v_new"]) and np.array_equal(R["v_old"], got["v_old"])
