"""GPU parity for A1/A2 (Aiyagari_VFI.m:65-90): the HIP sweep against the golden fixtures
and the C oracle.  Results are bit-exact for every σ: same operation sequence, -ffp-contract=off
on both sides, and the shared portable aiy_pow/aiy_log for non-integer powers."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def test_sweep_matches_golden_bitwise(pkg, gpu, golden):
    g = golden("a1_vfi_defaults")
    v, pk, pc, idx = pkg.vfi_sweep(g["v20"], g["a_grid"], g["s"], g["P"], float(g["r"]),
                                   float(g["w"]), 0.96, 5.0)
    assert np.array_equal(v, g["v21"])
    assert np.array_equal(idx - 1, g["idx21"])
    assert np.array_equal(pk, g["policy_k21"])
    assert np.array_equal(pc, g["policy_c21"])


def test_solve_matches_golden_bitwise(pkg, gpu, golden):
    g = golden("a1_vfi_defaults")
    R = pkg.vfi_solve(np.zeros((7, 400)), g["a_grid"], g["s"], g["P"], float(g["r"]),
                      float(g["w"]), 0.96, 5.0, 1e-5, 1000)
    assert R["iters"] == 249
    assert np.array_equal(R["v_new"], g["solve_v_new"])
    assert np.array_equal(R["v_old"], g["solve_v_old"])  # break before v_old = v_new
    assert np.array_equal(R["idx"] - 1, g["solve_idx"])


def test_solve_max_iter_exhausted(pkg, gpu, golden):
    g = golden("a1_vfi_defaults")
    R = pkg.vfi_solve(np.zeros((7, 400)), g["a_grid"], g["s"], g["P"], float(g["r"]),
                      float(g["w"]), 0.96, 5.0, 1e-5, 20)
    assert R["iters"] == 20
    assert np.array_equal(R["v_new"], g["v20"])
    assert np.array_equal(R["v_old"], R["v_new"])  # :88 ran after the last sweep


def _device_sweep(pkg, torch, V, a, s, P, r, w, beta, sigma, mode, hint=None, ws=None,
                  variant=0, k_chunk=1024):
    dev = torch.device("cuda:0")
    N, Na = V.shape
    ws = ws or pkg.Workspace(N, Na)
    ws.set_variant(variant)
    ws.set_search(0, k_chunk)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    vo, at, st, Pt = t(V), t(a), t(s), t(P)
    vn = torch.empty_like(vo); pk = torch.empty_like(vo); pc = torch.empty_like(vo)
    idx = torch.empty((N, Na), dtype=torch.int32, device=dev)
    ht = None if hint is None else t(hint.astype(np.int32))
    ws.vfi_sweep(vo, at, st, Pt, r, w, beta, sigma, vn, idx, pk, pc, hint=ht, mode=mode)
    torch.cuda.synchronize()
    return vn.cpu().numpy(), idx.cpu().numpy(), pk.cpu().numpy(), pc.cpu().numpy()


@pytest.mark.parametrize("variant,k_chunk", [(0, 1024), (1, 1024), (2, 1024), (6, 1024), (16, 1024),
                                             (8, 1024), (9, 512), (11, 256), (12, 1024), (13, 256),
                                             (32, 1024), (64, 1024), (80, 1024), (96, 1024)])
@pytest.mark.parametrize("Na,shocks", [(1500, "rouwenhorst"), (777, "tauchen")])
def test_screened_equals_plain_and_oracle(pkg, gpu, Na, shocks, variant, k_chunk):
    import torch
    cal = no.calib_aiyagari(Na=Na, shocks=shocks)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    r = 0.02
    w = no.wage(r, 0.36, 0.08)
    V = corc.vfi_solve(np.zeros((7, Na)), a, s, P, r, w, 0.96, 5.0, 1e-5, 15)["v_new"]
    vs, is_, pks, pcs = _device_sweep(pkg, torch, V, a, s, P, r, w, 0.96, 5.0, mode=1,
                                      variant=variant, k_chunk=k_chunk)
    vp, ip_, _, _ = _device_sweep(pkg, torch, V, a, s, P, r, w, 0.96, 5.0, mode=2)
    vo, io, pko, pco = corc.vfi_sweep(V, a, s, P, r, w, 0.96, 5.0)
    assert np.array_equal(vs, vo) and np.array_equal(is_, io)
    assert np.array_equal(vp, vo) and np.array_equal(ip_, io)
    assert np.array_equal(pks, pko) and np.array_equal(pcs, pco)


@pytest.mark.parametrize("variant", [0, 16, 4098, 4100, 1 << 21, 2064 | 1 << 16 | 1 << 21,
                                     2064 | 1 << 16 | 1 << 21 | 1 << 23,
                                     2064 | 1 << 16 | 1 << 21 | 3 << 23])
def test_hint_does_not_change_result(pkg, gpu, variant):
    import torch
    cal = no.calib_aiyagari(Na=900)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.04, 0.36, 0.08)
    V = corc.vfi_solve(np.zeros((7, 900)), a, s, P, 0.04, w, 0.96, 5.0, 1e-5, 40)["v_new"]
    ref = _device_sweep(pkg, torch, V, a, s, P, 0.04, w, 0.96, 5.0, mode=1, variant=variant)
    rng = np.random.default_rng(0)
    for hint in (np.zeros((7, 900)), rng.integers(0, 900, (7, 900)), np.full((7, 900), 10**6),
                 np.full((7, 900), -1)):
        out = _device_sweep(pkg, torch, V, a, s, P, 0.04, w, 0.96, 5.0, mode=1, hint=hint,
                            variant=variant)
        for x, y in zip(out, ref):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("sigma", [2.0, 3.0, 1.0, 2.5])
def test_other_sigmas(pkg, gpu, sigma):
    cal = no.calib_aiyagari(Na=300, sigma=sigma)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.03, 0.36, 0.08)
    V = corc.vfi_solve(np.zeros((7, 300)), a, s, P, 0.03, w, 0.96, sigma, 1e-5, 10)["v_new"]
    v, pk, pc, idx = pkg.vfi_sweep(V, a, s, P, 0.03, w, 0.96, sigma)
    vo, io, pko, pco = corc.vfi_sweep(V, a, s, P, 0.03, w, 0.96, sigma)
    # powers/logs are the shared portable aiy_pow/aiy_log: bit-exact for every sigma
    assert np.array_equal(v, vo) and np.array_equal(idx - 1, io)
    assert np.array_equal(pk, pko) and np.array_equal(pc, pco)


def test_edge_cases(pkg, gpu):
    # N = 1, Na = 2; a state with no feasible a' (a_grid above cash on hand) -> NaN, idx 1
    a = np.array([5.0, 6.0])
    v, pk, pc, idx = pkg.vfi_sweep(np.zeros((1, 2)), a, np.array([0.1]), np.ones((1, 1)),
                                   0.0, 1.0, 0.9, 5.0)
    vo, io, pko, pco = corc.vfi_sweep(np.zeros((1, 2)), a, np.array([0.1]), np.ones((1, 1)),
                                      0.0, 1.0, 0.9, 5.0)
    assert np.array_equal(np.isnan(v), np.isnan(vo))
    assert np.array_equal(idx - 1, io)
    assert np.allclose(pk, pko) and np.allclose(pc, pco, equal_nan=True)
    # NaN entries in v_old propagate as in MATLAB (ignored by max where possible)
    cal = no.calib_aiyagari(Na=50)
    V = np.zeros((7, 50)); V[3, 10] = np.nan
    w = no.wage(0.04, 0.36, 0.08)
    v, pk, pc, idx = pkg.vfi_sweep(V, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    vo, io, pko, pco = corc.vfi_sweep(V, cal["a_grid"], cal["s"], cal["P"], 0.04, w, 0.96, 5.0)
    assert np.array_equal(v, vo, equal_nan=True) and np.array_equal(idx - 1, io)


def test_full_size_bitwise_vs_oracle(pkg, gpu):
    """BASELINE config 2 size (Na = 20,000, Nz = 7 Rouwenhorst): one warm sweep, bit-exact
    against the C oracle (≈3e9 candidates on the host; a few seconds with OpenMP)."""
    import torch
    cal = no.calib_aiyagari(Na=20000, shocks="rouwenhorst")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.04, 0.36, 0.08)
    # a smooth non-trivial V: the Na=400 converged solution interpolated up
    c4 = no.calib_aiyagari(Na=400, shocks="rouwenhorst")
    V4 = corc.vfi_solve(np.zeros((7, 400)), c4["a_grid"], c4["s"], c4["P"], 0.04, w, 0.96,
                        5.0)["v_new"]
    V = np.stack([np.interp(a, c4["a_grid"], V4[i]) for i in range(7)])
    vs, is_, pks, pcs = _device_sweep(pkg, torch, V, a, s, P, 0.04, w, 0.96, 5.0, mode=1)
    vo, io, pko, pco = corc.vfi_sweep(V, a, s, P, 0.04, w, 0.96, 5.0)
    assert np.array_equal(vs, vo)
    assert np.array_equal(is_, io)
    # size-independent properties: policy monotone in a (Topkis), policy_c > 0
    assert (np.diff(is_, axis=1) >= 0).all()
    assert (pcs > 0).all()


@pytest.mark.parametrize("variant", [0, 1, 2, 6, 8, 12, 16, 32, 96, 512, 4098, 4100, 4102, 80, 2064,
                                     8192, 8208, 8272, 10256, 2064 | 2 << 16,
                                     10240 | 1 << 16, 64 | 3 << 16, 1 << 21, 4100 | 1 << 21,
                                     1 << 21 | 1 << 23, 16 | 1 << 23, 1 << 21 | 3 << 23])
def test_screen_stress_noisy_value(pkg, gpu, variant):
    """Rough value functions put many candidates within rounding distance of the running best
    (near-ties everywhere, multi-modal objectives): the fp32 pre-screen, the fp64 screen and
    the exact merge must still reproduce the plain exhaustive scan bit for bit — with and
    without hints, including odd chunk/region boundaries (Na odd, small k_chunk)."""
    import torch
    rng = np.random.default_rng(7 + variant)
    for Na, scale in ((2001, 1e-9), (1537, 1e-3), (999, 1.0)):
        cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst")
        a, s, P = cal["a_grid"], cal["s"], cal["P"]
        w = no.wage(0.03, 0.36, 0.08)
        V = corc.vfi_solve(np.zeros((7, Na)), a, s, P, 0.03, w, 0.96, 5.0, 1e-5, 25)["v_new"]
        V = V + scale * rng.standard_normal(V.shape)
        vo, io, pko, pco = corc.vfi_sweep(V, a, s, P, 0.03, w, 0.96, 5.0)
        for hint in (None, rng.integers(0, Na, (7, Na))):
            vs, is_, pks, pcs = _device_sweep(pkg, torch, V, a, s, P, 0.03, w, 0.96, 5.0,
                                              mode=1, hint=hint, variant=variant, k_chunk=320)
            assert np.array_equal(vs, vo) and np.array_equal(is_, io), (Na, scale)
            assert np.array_equal(pks, pko) and np.array_equal(pcs, pco)


_HY = 16 | 2048 | 1 << 16 | 1 << 21 | 1 << 23 | 1 << 24 | 1 << 26  # the hybrid tree launch


@pytest.mark.parametrize("variant", [16, 80, 2064, 8208, 8272, 10256, 2064 | 1 << 16,
                                     2064 | 2 << 16, 2064 | 3 << 16, 80 | 2 << 16,
                                     10256 | 2 << 16, 16 | 2048 | 1 << 16 | 1 << 21,
                                     16 | 2048 | 1 << 16 | 1 << 21 | 1 << 23,
                                     16 | 2048 | 1 << 16 | 1 << 21 | 3 << 23,
                                     _HY, _HY | 2 << 27, _HY | 5 << 27])
def test_full_size_dispatch_orders_and_tile_widths(pkg, gpu, variant):
    """Na = 20,000 (configs[1]): the tree's dispatch orders (bit 6: each XCD's range heaviest
    first; bit 11: its cheapest tiles last), the narrow one-wave tiles (bit 13: 46 states per
    tile, three tiles per SIMD) and packed workgroups (bits 16-17: 2, 4 or 8 one-wave tiles per
    workgroup), and the hybrid launch (bit 26: the 8, 32 or 256 heaviest tiles of each XCD range
    on two cooperating waves, the rest packed two per workgroup) change only the work split — a
    hinted warm sweep is bit-exact against the C oracle for each."""
    import torch
    cal = no.calib_aiyagari(Na=20000, shocks="rouwenhorst")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.04, 0.36, 0.08)
    c4 = no.calib_aiyagari(Na=400, shocks="rouwenhorst")
    V4 = corc.vfi_solve(np.zeros((7, 400)), c4["a_grid"], c4["s"], c4["P"], 0.04, w, 0.96,
                        5.0)["v_new"]
    V = np.stack([np.interp(a, c4["a_grid"], V4[i]) for i in range(7)])
    vo, io, pko, pco = corc.vfi_sweep(V, a, s, P, 0.04, w, 0.96, 5.0)
    hint = np.clip(io + 3, 0, 19999)
    vs, is_, pks, pcs = _device_sweep(pkg, torch, V, a, s, P, 0.04, w, 0.96, 5.0, mode=1,
                                      hint=hint, variant=variant)
    assert np.array_equal(vs, vo) and np.array_equal(is_, io)
    assert np.array_equal(pks, pko) and np.array_equal(pcs, pco)


@pytest.mark.parametrize("Na,variant", [(1100, 2048 | 2 << 16), (1100, 64 | 3 << 16),
                                        (333, 2048 | 1 << 16), (4100, 8192 | 2048 | 2 << 16),
                                        (333, 2048 | 1 << 26 | 1 << 27), (1100, 2048 | 1 << 26),
                                        (4100, 8192 | 2048 | 1 << 26 | 2 << 27)])
def test_packed_workgroups_ragged(pkg, gpu, Na, variant):
    """Packed workgroups whose last one is partly empty (7 rows x 18 tiles = 126 one-wave
    items in 4-wave workgroups: 2 unused slots; 7 x 6 = 42 in 2-wave ones at Na = 333; the
    narrow-tile count at Na = 4,100): the unused slots exit, every state is written once —
    a cold sweep and a hinted one, bit-exact against the C oracle."""
    import torch
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.04, 0.36, 0.08)
    V = corc.vfi_solve(np.zeros((7, Na)), a, s, P, 0.04, w, 0.96, 5.0, 1e-3, 1000)["v_new"]
    vo, io, pko, pco = corc.vfi_sweep(V, a, s, P, 0.04, w, 0.96, 5.0)
    for hint in (None, np.clip(io - 2, 0, Na - 1)):
        vs, is_, pks, pcs = _device_sweep(pkg, torch, V, a, s, P, 0.04, w, 0.96, 5.0, mode=1,
                                          hint=hint, variant=variant)
        assert np.array_equal(vs, vo) and np.array_equal(is_, io)
        assert np.array_equal(pks, pko) and np.array_equal(pcs, pco)
