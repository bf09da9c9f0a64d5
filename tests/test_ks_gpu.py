"""GPU parity for A6/A7 (Krusell_Smith_VFI.m:143-204): MATLAB-fminbnd policy improvement and
Jacobi Howard sweeps with pchip refresh.  log is the shared fdlibm aiy_log, so fminbnd's
value-dependent branches match the C oracle and results are bit-exact."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def _setup(golden):
    g = golden("ks_defaults")
    prm = np.array([g["beta"], g["alpha"], g["delta"], g["k_min"], g["k_max"], g["ug"], g["ub"],
                    g["l_bar"], g["mu"], 1.01, 0.99, 1.0, 0.0])
    return g, prm


def test_improve_and_howard_match_golden(pkg, gpu, golden):
    g, prm = _setup(golden)
    ko, nf = pkg.ks_policy_improve(g["V0"], g["k_grid"], g["K_grid"], g["B"], g["P"], prm)
    assert np.array_equal(ko, g["k_opt"]) and np.array_equal(nf, g["nfev"])
    V2 = pkg.ks_howard(g["V0"], ko, g["k_grid"], g["K_grid"], g["B"], g["P"], prm, steps=2)
    assert np.array_equal(V2, g["V_howard2"])


def _ks_oracle_params(prm):
    return corc.ks_params(beta=prm[0], alpha=prm[1], delta=prm[2], k_min=prm[3], k_max=prm[4],
                          ug=prm[5], ub=prm[6], l_bar=prm[7], mu=prm[8], z_grid=(prm[9], prm[10]),
                          eps_grid=(prm[11], prm[12]))


def test_fused_vfi_matches_oracle(pkg, gpu, golden):
    """The single-workgroup LDS-resident loop (whole VFI in one launch) vs the C pieces, with
    a non-identity ALM so K'_idx differs from K."""
    g, prm = _setup(golden)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    R = pkg.ks_vfi_solve(g["V0"], g["V0"] * 0 + 1.0, g["k_grid"], g["K_grid"], B, g["P"], prm,
                         howard_steps=10, tol=1e-6, max_vfi=12)
    Ro = corc.ks_vfi_solve(_ks_oracle_params(prm), g["k_grid"], g["K_grid"], g["V0"],
                           g["V0"] * 0 + 1.0, B, g["P"], howard=10, tol=1e-6, max_vfi=12)
    assert R["iters"] == Ro["iters"]
    assert np.array_equal(R["value"], Ro["value"])
    assert np.array_equal(R["k_opt"], Ro["k_opt"])
    assert R["rel_diff"] == Ro["rel_diff"]


@pytest.mark.parametrize("shards", [1, 3, 4])
def test_tiled_and_sharded_match_fused(pkg, gpu, shards):
    """A grid too large for one workgroup (tiled kernels) and the same problem sharded over
    K-ranges (peer/local copies of the needed columns): identical results."""
    p, kg, Kg, P, _, _ = no.ks_setup(k_size=300, K_size=12)
    prm = pkg.ks_params()
    V0 = np.log(0.1 / 0.9 * 0.9 * np.repeat(np.repeat(kg[:, None, None], 12, 1), 4, 2)) / (1 - 0.99)
    B = np.array([0.05, 0.985, 0.04, 0.99])
    k0 = 0.9 * np.repeat(np.repeat(kg[:, None, None], 12, 1), 4, 2)
    R = pkg.ks_vfi_solve(V0, k0, kg, Kg, B, P, prm, howard_steps=6, tol=1e-8, max_vfi=11,
                         n_devices=shards)
    Ro = corc.ks_vfi_solve(_ks_oracle_params(prm), kg, Kg, V0, k0, B, P, howard=6, tol=1e-8,
                           max_vfi=11)
    assert R["iters"] == Ro["iters"]
    assert np.array_equal(R["value"], Ro["value"])
    assert np.array_equal(R["k_opt"], Ro["k_opt"])


def test_scaling_size_sharded_equals_unsharded(pkg, gpu):
    """BASELINE configs[4]'s scaling grid (k = 32,768, K = 64 on [30, 50], 8.4 M nodes): one
    VFI iteration (policy improvement + 3 Jacobi Howard sweeps, Krusell_Smith_VFI.m:148-192)
    sharded over 4 in-process shards (targeted peer/local copies of the forecast columns)
    equals the unsharded solve bit for bit."""
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=32768, K_size=64)
    prm = pkg.ks_params()
    B = np.array([0.1, 0.97, 0.08, 0.975])
    k0 = np.ones_like(V0)
    R1 = pkg.ks_vfi_solve(V0, k0, kg, Kg, B, P, prm, howard_steps=3, tol=0.0, max_vfi=1)
    R4 = pkg.ks_vfi_solve(V0, k0, kg, Kg, B, P, prm, howard_steps=3, tol=0.0, max_vfi=1,
                          n_devices=4)
    assert R1["iters"] == R4["iters"] == 1
    assert np.array_equal(R1["value"], R4["value"])
    assert np.array_equal(R1["k_opt"], R4["k_opt"])
    assert R1["rel_diff"] == R4["rel_diff"]
    assert np.isfinite(R1["value"]).all()


@pytest.mark.parametrize("shards,depth", [(8, 1), (8, 2), (8, 4), (5, 3), (2, 7), (6, 4)])
def test_kz_sliced_ghost_blocks_reference_size(pkg, gpu, golden, shards, depth):
    """The MATLAB-facing multi-device path (ks_vfi_solve_sharded) at the
    reference grid (k = 100, K = 4, Krusell_Smith_VFI.m:8): up to 8 (K, Z) slices on this card,
    ghost-rectangle blocks of `depth` Howard sweeps (10 sweeps: blocks that do not divide it),
    improvement every 5th iteration — bit for bit the single-device solve and the C oracle."""
    g, prm = _setup(golden)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    args = (g["V0"], g["V0"] * 0 + 1.0, g["k_grid"], g["K_grid"], B, g["P"], prm)
    R1 = pkg.ks_vfi_solve(*args, howard_steps=10, tol=1e-6, max_vfi=12)
    Rs = pkg.ks_vfi_solve(*args, howard_steps=10, tol=1e-6, max_vfi=12, n_devices=shards,
                          depth=depth)
    assert Rs["iters"] == R1["iters"] and Rs["rel_diff"] == R1["rel_diff"]
    assert np.array_equal(Rs["value"], R1["value"])
    assert np.array_equal(Rs["k_opt"], R1["k_opt"])


def test_kz_sliced_ghost_blocks_k4096(pkg, gpu):
    """ks_vfi_solve(n_devices = 8) (depth 4) at k = 4,096, K = 16 (the fused Howard+slopes
    kernel with multi-block columns: 4 halo nodes per 256), 2 policy improvements and 7
    Howard sweeps per iteration, vs the single-device tiled solve."""
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=4096, K_size=16)
    prm = pkg.ks_params()
    B = np.array([0.1, 0.97, 0.08, 0.975])
    k0 = np.ones_like(V0)
    R1 = pkg.ks_vfi_solve(V0, k0, kg, Kg, B, P, prm, howard_steps=7, tol=0.0, max_vfi=6)
    R8 = pkg.ks_vfi_solve(V0, k0, kg, Kg, B, P, prm, howard_steps=7, tol=0.0, max_vfi=6,
                          n_devices=8)
    assert R1["iters"] == R8["iters"] == 6 and R1["rel_diff"] == R8["rel_diff"]
    assert np.array_equal(R1["value"], R8["value"])
    assert np.array_equal(R1["k_opt"], R8["k_opt"])
    assert np.isfinite(R1["value"]).all()


def test_fused_howard_equals_two_launch_sweep(pkg, gpu):
    """ks_dev_howard_fused (value + the next sweep's slopes in one launch) vs ks_dev_howard
    (slopes launch + sweep) over a sharded rectangle, nk = 300 (two blocks per column, halo
    nodes evaluated twice) and nk = 4,099 (a short last block)."""
    import torch
    for nk, nK in ((300, 6), (4099, 5)):
        kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
        B = np.array([0.1, 0.97, 0.08, 0.975])
        kd = pkg.ks_dist
        dev = torch.device("cuda:0")
        V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
        ko = torch.ones_like(V)
        sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), 1, nK - 1, 0, 4)
        sh.improve(V, ko)
        A = V.clone()
        for _ in range(3):  # two-launch sweeps
            An = A.clone()
            sh.howard(A, ko, An)
            A = An
        dV, dV2 = torch.zeros_like(V), torch.zeros_like(V)
        Bv, B2 = V.clone(), V.clone()
        sh.slopes(Bv, dV)
        for _ in range(3):
            sh.howard_fused(Bv, dV, ko, B2, dV2)
            Bv, B2 = B2, Bv
            dV, dV2 = dV2, dV
        torch.cuda.synchronize()
        own = slice(1, nK - 1)
        assert torch.equal(A[:, own], Bv[:, own]), nk
        ref = torch.zeros_like(V)
        sh.slopes(Bv, ref)  # slopes of the final values, by the separate kernel
        torch.cuda.synchronize()
        x, y = ref[:, own], dV[:, own]  # (NaN slopes at a degenerate first node: same places)
        assert torch.equal(torch.isnan(x), torch.isnan(y)), nk
        assert torch.equal(torch.nan_to_num(x, nan=0.0), torch.nan_to_num(y, nan=0.0)), nk
        sh.close()


@pytest.mark.parametrize("shards", [8, 6, 5, 3, 2, 1])
def test_direct_peer_reads_reference_size(pkg, gpu, golden, shards):
    """The direct schedule (ks_vfi_solve_sharded depth = 0): no column copies, no ghost sweeps —
    every Howard sweep and improvement reads each forecast column (Krusell_Smith_VFI.m:343-349)
    where its owning shard keeps it (pointer tables into the owners' double buffers) after
    stream-event waits on the neighbours' previous sweep.  Up to 8 (K, Z) slices on this card
    at the reference grid: bit for bit the single-device solve."""
    g, prm = _setup(golden)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    args = (g["V0"], g["V0"] * 0 + 1.0, g["k_grid"], g["K_grid"], B, g["P"], prm)
    R1 = pkg.ks_vfi_solve(*args, howard_steps=10, tol=1e-6, max_vfi=12)
    Rs = pkg.ks_vfi_solve(*args, howard_steps=10, tol=1e-6, max_vfi=12, n_devices=shards,
                          depth=0)
    assert Rs["iters"] == R1["iters"] and Rs["rel_diff"] == R1["rel_diff"]
    assert np.array_equal(Rs["value"], R1["value"])
    assert np.array_equal(Rs["k_opt"], R1["k_opt"])


@pytest.mark.parametrize("nk,nK,howard,vfi", [(4096, 16, 7, 6), (32768, 64, 3, 1)])
def test_direct_peer_reads_large(pkg, gpu, nk, nK, howard, vfi):
    """The direct schedule on 8 shards at k = 4,096, K = 16 (multi-block columns, 2 policy
    improvements) and at the scaling size k = 32,768, K = 64 (8.4 M nodes, one VFI iteration):
    bit for bit the single-device solve."""
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
    prm = pkg.ks_params()
    B = np.array([0.1, 0.97, 0.08, 0.975])
    k0 = np.ones_like(V0)
    R1 = pkg.ks_vfi_solve(V0, k0, kg, Kg, B, P, prm, howard_steps=howard, tol=0.0, max_vfi=vfi)
    R8 = pkg.ks_vfi_solve(V0, k0, kg, Kg, B, P, prm, howard_steps=howard, tol=0.0, max_vfi=vfi,
                          n_devices=8, depth=0)
    assert R1["iters"] == R8["iters"] == vfi and R1["rel_diff"] == R8["rel_diff"]
    assert np.array_equal(R1["value"], R8["value"])
    assert np.array_equal(R1["k_opt"], R8["k_opt"])
    assert np.isfinite(R1["value"]).all()
