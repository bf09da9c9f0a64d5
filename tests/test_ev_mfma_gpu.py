"""The expectation EV = (βP)·V on the fp64 matrix cores (north star: "fp64 MFMA only when Nz is
large enough to be a real contraction"; Aiyagari_VFI.m:79 `beta * P(i,:) * v_old`,
Aiyagari_Endogenous_Labor_VFI.m:69 `EV = beta * P * v_old`).

From Nz = 32 (bellman.hpp kEvMfmaMinN) the table kernel takes EV from bell_ev_mfma_kernel
(v_mfma_f64_16x16x4_f64); variant bit 15 forces it at any Nz, bit 14 forces the sequential VALU
sum the C oracle restates.  The MFMA sums in the hardware's order, so:
  * with data on which every product and partial sum is exact (β = 1/2, P in multiples of 1/8,
    V small integers) the whole sweep equals the C oracle bit for bit at Nz = 7, 9 and 37 —
    the lane maps, the k-steps, padding rows/columns and the tree downstream are all pinned;
  * on real calibrations (Rouwenhorst Nz = 32, 48) the value agrees with the oracle to 1e-10
    and the policy indices are identical (the north-star tolerance; MATLAB's BLAS order for the
    same product is unpinned too);
  * the batched config-4 solve takes the same EV path, so batched == separate stays bit-exact."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def _exact_problem(N, Na, rng):
    P = rng.integers(0, 9, (N, N)).astype(np.float64)
    P[:, 0] += 1.0
    P = P / 8.0  # multiples of 1/8 (rows need not sum to one for the arithmetic)
    V = rng.integers(-40, 40, (N, Na)).astype(np.float64)
    a = np.linspace(0.0, 30.0, Na) ** 1.0
    s = np.linspace(0.5, 2.0, N)
    return P, V, a, s


def _sweep(pkg, torch, P, V, a, s, r, w, beta, sigma, variant, mode=1):
    dev = torch.device("cuda", 0)
    N, Na = V.shape
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    ws = pkg.Workspace(N, Na)
    ws.set_variant(variant)
    vn = torch.empty((N, Na), dtype=torch.float64, device=dev)
    idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    pk, pc = torch.empty_like(vn), torch.empty_like(vn)
    ws.vfi_sweep(t(V), t(a), t(s), t(P), r, w, beta, sigma, vn, idx, pk, pc, mode=mode)
    torch.cuda.synchronize()
    return vn.cpu().numpy(), idx.cpu().numpy(), pk.cpu().numpy(), pc.cpu().numpy()


@pytest.mark.parametrize("N,Na", [(7, 400), (9, 1000), (37, 700)])
def test_mfma_ev_exact_data_bitwise(pkg, gpu, N, Na):
    import torch
    rng = np.random.default_rng(N)
    P, V, a, s = _exact_problem(N, Na, rng)
    for var in (2 | 32768, 16 | 32768, 2 | 16384):  # MFMA (two geometries), VALU
        out = _sweep(pkg, torch, P, V, a, s, 0.02, 1.0, 0.5, 5.0, var)
        ref = corc.vfi_sweep(V, a, s, P, 0.02, 1.0, 0.5, 5.0)
        for x, y in zip(out, ref):
            assert np.array_equal(x, y), var
        ex = _sweep(pkg, torch, P, V, a, s, 0.02, 1.0, 0.5, 5.0, var, mode=2)  # plain scan
        for x, y in zip(ex, ref):
            assert np.array_equal(x, y), var


@pytest.mark.parametrize("N", [32, 48])
def test_mfma_ev_real_calibration_tolerance(pkg, gpu, N):
    """Nz >= 32 takes MFMA by default: value within 1e-10 of the C oracle relative to
    max(1, |v|), identical argmax.  The north star's 1e-10 sup-norm is read relative: at low
    assets this calibration's v reaches -2e6, where one fp64 ulp is 4.7e-10, so no reordered
    sum (MFMA here, BLAS in MATLAB) can meet an absolute 1e-10 there."""
    import torch
    cal = no.calib_aiyagari(Na=2000, shocks="rouwenhorst", N=N)
    w = no.wage(0.03, 0.36, 0.08)
    Vs = corc.vfi_solve(np.zeros((N, 2000)), cal["a_grid"], cal["s"], cal["P"], 0.03, w, 0.96,
                        5.0, 1e-5, 40)["v_new"]
    vn, idx, pk, pc = _sweep(pkg, torch, cal["P"], Vs, cal["a_grid"], cal["s"], 0.03, w, 0.96,
                             5.0, -1)
    vo, io, pko, pco = corc.vfi_sweep(Vs, cal["a_grid"], cal["s"], cal["P"], 0.03, w, 0.96, 5.0)
    assert np.max(np.abs(vn - vo) / np.maximum(1.0, np.abs(vo))) <= 1e-10
    assert np.array_equal(idx, io) and np.array_equal(pk, pko)
    vv, iv, _, _ = _sweep(pkg, torch, cal["P"], Vs, cal["a_grid"], cal["s"], 0.03, w, 0.96, 5.0,
                          16 | 16384)  # forced VALU EV: the oracle's bits
    assert np.array_equal(vv, vo) and np.array_equal(iv, io)


def test_mfma_ev_batch_equals_separate(pkg, gpu):
    from tests.test_batch_gpu import _batch_vs_single
    import torch
    cal = pkg.calibration.aiyagari(Na=600, shocks="rouwenhorst", N=32)
    _batch_vs_single(pkg, torch, cal, [0.01, 0.03, -0.02], np.zeros((32, 600)), max_iter=15)
