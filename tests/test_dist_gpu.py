"""GPU parity for A10 (new component, no reference code; oracle = the C restatement of its
definition, sequential scatter): the monotone-run gather reproduces the scatter bit for bit;
non-monotone policies take the exact ordered-scan fallback."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def _vfi_policy(Na, shocks="tauchen"):
    cal = no.calib_aiyagari(Na=Na, shocks=shocks)
    w = no.wage(0.04, 0.36, 0.08)
    R = corc.vfi_solve(np.zeros((7, Na)), cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    return cal, R


def test_one_push_matches_golden(pkg, gpu, golden):
    g = golden("a10_dist_defaults")
    a1 = golden("a1_vfi_defaults")
    lam, K, it, dist = pkg.dist_stationary(a1["a_grid"], a1["P"], policy_idx=g["idx"] + 1,
                                           lam0=g["lam0"], tol=0.0, max_iter=1)
    # the numpy golden projects with BLAS (P.T @ mass: another summation order) → rounding;
    # the C restatement (sequential, same order as the kernels) must match bit for bit
    assert it == 1 and np.max(np.abs(lam - g["lam1"])) < 1e-15
    assert np.array_equal(lam, corc.dist_update_ongrid(g["lam0"], g["idx"], a1["P"]))
    lamL, _, _, _ = pkg.dist_stationary(a1["a_grid"], a1["P"], policy_k=g["kp_egm"],
                                        lam0=g["lam0"], tol=0.0, max_iter=1)
    assert np.max(np.abs(lamL - g["lam1_lottery"])) < 1e-15
    assert np.array_equal(lamL, corc.dist_update_lottery(g["lam0"], g["kp_egm"], a1["a_grid"],
                                                         a1["P"]))


@pytest.mark.parametrize("Na", [400, 4000])
def test_stationary_ongrid_bitwise(pkg, gpu, Na):
    cal, R = _vfi_policy(Na)
    lam0 = np.full((7, Na), 1.0 / (7 * Na))
    lam, K, it, dist = pkg.dist_stationary(cal["a_grid"], cal["P"], policy_idx=R["idx"] + 1,
                                           lam0=lam0, tol=1e-13, max_iter=5000)
    lo, Ko, ito, disto = corc.dist_stationary(lam0, cal["a_grid"], cal["P"], idx=R["idx"],
                                              tol=1e-13, max_iter=5000)
    assert it == ito
    assert np.array_equal(lam, lo)
    assert abs(K - Ko) <= 1e-12 * abs(Ko)       # K: fixed-order tree sum vs sequential sum
    assert abs(lam.sum() - 1.0) < 1e-10


def test_stationary_lottery_bitwise(pkg, gpu, golden):
    g = golden("a4_egm_defaults")
    kp = g["policy_k"].T  # [N][Na]
    lam0 = np.full((7, 400), 1.0 / 2800)
    lam, K, it, dist = pkg.dist_stationary(g["a_grid"], g["P"], policy_k=kp, lam0=lam0,
                                           tol=1e-13, max_iter=5000)
    lo, Ko, ito, _ = corc.dist_stationary(lam0, g["a_grid"], g["P"], kp=kp, tol=1e-13,
                                          max_iter=5000)
    assert it == ito and np.array_equal(lam, lo)
    assert abs(K - Ko) <= 1e-12 * abs(Ko)


def test_non_monotone_policy_fallback(pkg, gpu):
    rng = np.random.default_rng(0)
    Na = 300
    cal = no.calib_aiyagari(Na=Na)
    idx = rng.integers(0, Na, (7, Na)).astype(np.int32)  # arbitrary, non-monotone
    lam0 = rng.random((7, Na)); lam0 /= lam0.sum()
    lam, K, it, _ = pkg.dist_stationary(cal["a_grid"], cal["P"], policy_idx=idx + 1, lam0=lam0,
                                        tol=0.0, max_iter=3)
    lo, _, _, _ = corc.dist_stationary(lam0, cal["a_grid"], cal["P"], idx=idx, tol=0.0,
                                       max_iter=3)
    assert np.array_equal(lam, lo)
    kp = rng.uniform(-1, cal["a_grid"][-1] + 1, (7, Na))
    lam, _, _, _ = pkg.dist_stationary(cal["a_grid"], cal["P"], policy_k=kp, lam0=lam0, tol=0.0,
                                       max_iter=2)
    lo, _, _, _ = corc.dist_stationary(lam0, cal["a_grid"], cal["P"], kp=kp, tol=0.0, max_iter=2)
    assert np.array_equal(lam, lo)


def test_bad_index_rejected(pkg, gpu):
    cal = no.calib_aiyagari(Na=50)
    idx = np.ones((7, 50), np.int32); idx[2, 7] = 51
    with pytest.raises(pkg.AiyError):
        pkg.dist_stationary(cal["a_grid"], cal["P"], policy_idx=idx, tol=0.0, max_iter=1)


def _long_run_policy(Na, rng):
    """Monotone on-grid policy with runs far longer than one chunk (32) and than one wave's
    64 chunks (2,048): a borrowing-constraint run of 4,500 sources, a top-of-grid run of 2,600,
    short runs and gaps in between."""
    idx = np.empty((3, Na), np.int32)
    for i in range(3):
        body = np.sort(rng.integers(1, Na - 1, Na - 4500 - 2600 * (i > 0)))
        parts = [np.zeros(4500, np.int64), body]
        if i > 0:
            parts.append(np.full(2600, Na - 1))
        idx[i] = np.concatenate(parts)[:Na]
    return idx


def test_long_runs_chunked_order_bitwise(pkg, gpu):
    """Runs of 33 … 4,500 terms take the wave-cooperative chunk path (dist.hpp kDistChunk);
    the C restatement sums the same chunks in the same order."""
    rng = np.random.default_rng(7)
    Na = 9000
    a = np.linspace(0.0, 50.0, Na) ** 1.5
    P = rng.random((3, 3)); P /= P.sum(1, keepdims=True)
    idx = _long_run_policy(Na, rng)
    lam0 = rng.random((3, Na)); lam0 /= lam0.sum()
    lam, _, it, _ = pkg.dist_stationary(a, P, policy_idx=idx + 1, lam0=lam0, tol=0.0, max_iter=3)
    lo, _, ito, _ = corc.dist_stationary(lam0, a, P, idx=idx, tol=0.0, max_iter=3)
    assert it == ito == 3 and np.array_equal(lam, lo)
    # lottery: a long run below the grid (key 0, weight 0) and one at its top (weight 1)
    kp = np.concatenate([np.full((3, 3000), -1.0), np.sort(rng.uniform(0, a[-1], (3, Na - 5000)), 1),
                         np.full((3, 2000), a[-1] + 1.0)], 1)
    lam, _, _, _ = pkg.dist_stationary(a, P, policy_k=kp, lam0=lam0, tol=0.0, max_iter=2)
    lo, _, _, _ = corc.dist_stationary(lam0, a, P, kp=kp, tol=0.0, max_iter=2)
    assert np.array_equal(lam, lo)


@pytest.mark.parametrize("tol,max_iter", [(1e-13, 5000), (1e-9, 5000), (0.0, 45), (1e-13, 70)])
def test_stationary_dev_speculative_batches(pkg, gpu, tol, max_iter):
    """aiy_dist_stationary_dev (plan once, up to 32 pushes per read) stops at the push the
    one-read-per-push loop stops at — in the middle of a batch, at max_iter, on push counts that
    are not multiples of the batch — with the same λ, dist and K."""
    import torch
    cal, R = _vfi_policy(1000)
    dev = torch.device("cuda:0")
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    lam0 = np.full((7, 1000), 1.0 / 7000)
    ws = pkg.Workspace(7, 1000)
    out = torch.empty((7, 1000), dtype=torch.float64, device=dev)
    K = torch.zeros(1, dtype=torch.float64, device=dev)
    it, dist = pkg.dist_stationary_dev(ws, t(lam0), t(cal["a_grid"]), t(cal["P"]), out,
                                       policy_idx=t(R["idx"].astype(np.int32)), tol=tol,
                                       max_iter=max_iter, k_supply=K)
    lo, Ko, ito, disto = corc.dist_stationary(lam0, cal["a_grid"], cal["P"], idx=R["idx"],
                                              tol=tol, max_iter=max_iter)
    assert it == ito and dist == disto
    assert np.array_equal(out.cpu().numpy(), lo)
    assert abs(float(K[0]) - Ko) <= 1e-12 * abs(Ko)


@pytest.mark.parametrize("N,Na", [(16, 3000), (1, 70), (5, 1025)])
def test_staged_push_shapes_bitwise(pkg, gpu, N, Na):
    """The push stages each wave's source range in LDS (kDistStage within a 64 KB budget: 512
    sources per wave on the on-grid path at N = 16, 256 with lottery weights); random monotone
    policies with runs from 0 to a few hundred sources, N = 1 … 16, ragged last tiles — on-grid
    and lottery pushes bit-exact against the C restatement."""
    rng = np.random.default_rng(N * 1000 + Na)
    a = np.linspace(0.0, 30.0, Na) ** 2 / 30.0
    P = rng.random((N, N)); P /= P.sum(1, keepdims=True)
    steps = rng.choice([0, 1, 1, 1, 2, 0, 0], size=(N, Na))
    idx = np.minimum(np.cumsum(steps, 1), Na - 1).astype(np.int64)
    lam0 = rng.random((N, Na)); lam0 /= lam0.sum()
    lam, _, _, _ = pkg.dist_stationary(a, P, policy_idx=idx + 1, lam0=lam0, tol=0.0, max_iter=3)
    lo, _, _, _ = corc.dist_stationary(lam0, a, P, idx=idx, tol=0.0, max_iter=3)
    assert np.array_equal(lam, lo)
    kp = np.sort(rng.uniform(-1.0, a[-1] * 0.8, (N, Na)), 1)
    lam, _, _, _ = pkg.dist_stationary(a, P, policy_k=kp, lam0=lam0, tol=0.0, max_iter=2)
    lo, _, _, _ = corc.dist_stationary(lam0, a, P, kp=kp, tol=0.0, max_iter=2)
    assert np.array_equal(lam, lo)


@pytest.mark.parametrize("N,Na", [(17, 900), (32, 2000), (48, 401)])
def test_push_more_than_16_states_bitwise(pkg, gpu, N, Na):
    """N > 16 (Rouwenhorst Nz = 32/48, the MFMA EV calibrations): the run gather + projection
    path, on-grid and lottery, against the C restatement — and through the host tier's
    speculative fixed-point loop (diff slots cleared per push on this path)."""
    rng = np.random.default_rng(N * 7 + Na)
    a = np.linspace(0.0, 30.0, Na) ** 2 / 30.0
    P = rng.random((N, N)); P /= P.sum(1, keepdims=True)
    steps = rng.choice([0, 1, 1, 1, 2, 0, 0, 40], size=(N, Na))  # incl. runs > one chunk
    idx = np.minimum(np.cumsum(steps, 1) // 3, Na - 1).astype(np.int64)
    lam0 = rng.random((N, Na)); lam0 /= lam0.sum()
    lam, _, it, _ = pkg.dist_stationary(a, P, policy_idx=idx + 1, lam0=lam0, tol=0.0, max_iter=3)
    lo, _, _, _ = corc.dist_stationary(lam0, a, P, idx=idx, tol=0.0, max_iter=3)
    assert it == 3 and np.array_equal(lam, lo)
    kp = np.sort(rng.uniform(-1.0, a[-1] * 0.8, (N, Na)), 1)
    lam, _, _, _ = pkg.dist_stationary(a, P, policy_k=kp, lam0=lam0, tol=0.0, max_iter=2)
    lo, _, _, _ = corc.dist_stationary(lam0, a, P, kp=kp, tol=0.0, max_iter=2)
    assert np.array_equal(lam, lo)
    lam, K, it, d = pkg.dist_stationary(a, P, policy_idx=idx + 1, lam0=lam0, tol=1e-12,
                                        max_iter=400)
    lo, Ko, ito, do = corc.dist_stationary(lam0, a, P, idx=idx, tol=1e-12, max_iter=400)
    assert it == ito and d == do and np.array_equal(lam, lo)


def test_ge_pipeline_rouwenhorst_32(pkg, gpu):
    """VFI at Nz = 32 (MFMA EV) followed by dist_stationary on its policy — the
    combination ge() runs — succeeds and matches the C restatement's histogram on that policy."""
    from oracle import np_oracle as no2
    cal = no2.calib_aiyagari(Na=300, shocks="rouwenhorst", N=32)
    w = no2.wage(0.04, 0.36, 0.08)
    R = pkg.vfi_solve(np.zeros((32, 300)), cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0,
                      1e-5, 400)
    lam0 = np.full((32, 300), 1.0 / (32 * 300))
    lam, K, it, _ = pkg.dist_stationary(cal["a_grid"], cal["P"], policy_idx=R["idx"], lam0=lam0,
                                        tol=1e-12, max_iter=3000)
    lo, Ko, ito, _ = corc.dist_stationary(lam0, cal["a_grid"], cal["P"], idx=R["idx"] - 1,
                                          tol=1e-12, max_iter=3000)
    assert it == ito and np.array_equal(lam, lo)
    assert abs(K - Ko) <= 1e-12 * abs(Ko)
