"""GPU parity for A4/A5 (Aiyagari_EGM.m:71-110, Aiyagari_Endogenous_Labor_EGM.m:64-107).
Against the C restatement: bit-exact (shared portable aiy_pow for RHS^(-1/σ)).  Against the
numpy golden (numpy's own SIMD pow): the north-star tolerance 1e-10."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def test_egm_solve_vs_golden(pkg, gpu, golden):
    g = golden("a4_egm_defaults")
    R = pkg.egm_solve(g["policy_c0"], g["a_grid"], g["s"], g["P"], float(g["r"]), float(g["w"]),
                      0.96, 5.0, float(g["amin"]))
    assert R["iters"] == int(g["iters"]) == 213
    assert np.max(np.abs(R["policy_c"] - g["policy_c"])) < 1e-10
    assert np.max(np.abs(R["policy_k"] - g["policy_k"])) < 1e-10
    assert abs(R["dist"] - float(g["dist"])) < 1e-10


def test_egm_step_vs_oracle(pkg, gpu, golden):
    g = golden("a4_egm_defaults")
    c1, k1, d1 = pkg.egm_step(g["policy_c0"], g["a_grid"], g["s"], g["P"], float(g["r"]),
                              float(g["w"]), 0.96, 5.0, float(g["amin"]))
    co, ko, do = corc.egm_step(g["policy_c0"].T, g["a_grid"], g["s"], g["P"], float(g["r"]),
                               float(g["w"]), 0.96, 5.0, float(g["amin"]))
    assert np.array_equal(c1, co.T) and np.array_equal(k1, ko.T) and d1 == do


def test_labor_egm_solve_vs_golden(pkg, gpu, golden):
    g = golden("a5_labor_egm_defaults")
    R = pkg.labor_egm_solve(g["policy_c0"], g["a_grid"], g["s"], g["P"], float(g["r"]),
                            float(g["w"]), 0.96, 5.0, 1.0, 1.0, float(g["amin"]))
    assert R["iters"] == int(g["iters"]) == 227
    for k in ("policy_c", "policy_k", "policy_l"):
        assert np.max(np.abs(R[k] - g[k])) < 1e-10, k


@pytest.mark.parametrize("Na,sigma,theta", [(20000, 5.0, 1.0), (5000, 2.5, 2.0)])
def test_egm_large_and_nonint(pkg, gpu, Na, sigma, theta):
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst", sigma=sigma)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.03, 0.36, 0.08)
    pc0 = np.tile(((1.03) * a + w * np.mean(s))[:, None], (1, 7))
    R = pkg.egm_solve(pc0, a, s, P, 0.03, w, 0.96, sigma, cal["amin"], 1e-5, 40)
    Ro = corc.egm_solve(pc0.T, a, s, P, 0.03, w, 0.96, sigma, cal["amin"], 1e-5, 40)
    assert R["iters"] == Ro["iters"]
    assert np.array_equal(R["policy_c"], Ro["policy_c"].T)
    assert np.array_equal(R["policy_k"], Ro["policy_k"].T)
    L = pkg.labor_egm_solve(pc0, a, s, P, 0.03, w, 0.96, sigma, 1.0, theta, cal["amin"], 1e-5, 20)
    Lo = corc.labor_egm_solve(pc0.T, a, s, P, 0.03, w, 0.96, sigma, 1.0, theta, cal["amin"], 1e-5, 20)
    assert L["iters"] == Lo["iters"]
    for k in ("policy_c", "policy_k", "policy_l"):
        assert np.array_equal(L[k], Lo[k].T), k


def test_egm_nonmonotone_grid_is_reported(pkg, gpu):
    """interp1 needs a monotone endogenous grid; a decreasing one is an error, not garbage."""
    a = np.linspace(0, 10, 50)
    pc0 = np.tile(np.linspace(50, 0.01, 50)[:, None], (1, 2))  # steeply decreasing c → â folds
    with pytest.raises(pkg.AiyError) as e:
        pkg.egm_step(pc0, a, np.array([1.0, 1.2]), np.full((2, 2), 0.5), 0.02, 1.0, 0.96, 5.0, 0.0)
    assert e.value.status == "AIY_BAD_ARG"


@pytest.mark.parametrize("tol,max_iter", [(1e-5, 7), (1e-3, 1000), (1e-5, 1), (2e-2, 1000),
                                          (1e-5, 16), (1e-5, 17)])
def test_egm_speculative_solve_matches_oracle(pkg, gpu, tol, max_iter):
    """The host-tier solve enqueues up to 16 steps between dist reads (ring of policy_c buffers,
    the stopping step re-run for its policy_k): iteration count, dist and both policies equal
    the one-read-per-step C loop for stops inside a batch, on a batch edge and at max_iter."""
    cal = no.calib_aiyagari(Na=400, shocks="tauchen")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    w = no.wage(0.04, 0.36, 0.08)
    pc0 = np.tile(((1.04) * a + w * np.mean(s))[:, None], (1, s.size))
    R = pkg.egm_solve(pc0, a, s, P, 0.04, w, 0.96, 5.0, cal["amin"], tol, max_iter)
    Ro = corc.egm_solve(pc0.T, a, s, P, 0.04, w, 0.96, 5.0, cal["amin"], tol, max_iter)
    assert R["iters"] == Ro["iters"]
    assert np.array_equal(R["policy_c"], Ro["policy_c"].T)
    assert np.array_equal(R["policy_k"], Ro["policy_k"].T)
    assert R["dist"] == Ro["dist"]
    L = pkg.labor_egm_solve(pc0, a, s, P, 0.04, w, 0.96, 5.0, 1.0, 1.0, cal["amin"], tol, max_iter)
    Lo = corc.labor_egm_solve(pc0.T, a, s, P, 0.04, w, 0.96, 5.0, 1.0, 1.0, cal["amin"], tol,
                              max_iter)
    assert L["iters"] == Lo["iters"]
    for k in ("policy_c", "policy_k", "policy_l"):
        assert np.array_equal(L[k], Lo[k].T), k


def test_egm_solve_nonmonotone_grid_is_reported(pkg, gpu):
    a = np.linspace(0, 10, 50)
    pc0 = np.tile(np.linspace(50, 0.01, 50)[:, None], (1, 2))
    with pytest.raises(pkg.AiyError) as e:
        pkg.egm_solve(pc0, a, np.array([1.0, 1.2]), np.full((2, 2), 0.5), 0.02, 1.0, 0.96, 5.0,
                      0.0, 1e-6, 50)
    assert e.value.status == "AIY_BAD_ARG"


@pytest.mark.parametrize("Na,N", [(2, 7), (3, 7), (65, 7), (400, 7), (1024, 7), (1025, 7),
                                  (1090, 7), (4099, 7), (20000, 7), (3000, 2),
                                  (2000, 16)])
@pytest.mark.parametrize("labor", [False, True])
def test_egm_fused_small_grid_equals_two_launches(pkg, gpu, Na, N, labor):
    """The default step — egm_fused_kernel (one launch, a workgroup per productivity state) for
    Na <= 1024, the two-launch step above — against the EGM knobs 18 | 20 (the two-launch step
    on small grids, interp1 without segment windows).  Both, and the C restatement, agree bit
    for bit over several steps (policy_c, policy_k, policy_l and the step's dist), N = 1 … 16."""
    import torch
    dev = torch.device("cuda", 0)
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst", N=N) if N != 7 else \
        no.calib_aiyagari(Na=Na, shocks="rouwenhorst")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    N = P.shape[0]
    r = 0.03
    w = no.wage(r, 0.36, 0.08)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t = t(a), t(s), t(P)
    pc = np.tile(((1 + r) * a + w * np.mean(s))[None, :], (N, 1))
    runs = []
    for var in (-1, (1 << 18) | (1 << 20)):
        ws = pkg.Workspace(N, Na)
        if var >= 0:
            ws.set_variant(var)
        c = t(pc)
        outs = []
        for _ in range(6):
            o, k = torch.empty_like(c), torch.empty_like(c)
            l = torch.empty_like(c) if labor else None
            dd = torch.zeros(2, dtype=torch.int64, device=dev)
            pkg.egm_step_dev(ws, c, a_t, s_t, P_t, r, w, 0.96, 5.0, cal["amin"], o, k,
                             labor=labor, phi=1.0, theta=1.0, policy_l=l, diff=dd)
            outs.append([x.cpu().numpy() for x in (c, o, k) + ((l,) if labor else ())] +
                        [dd.cpu().numpy()])
            c = o
        runs.append(outs)
    for step_f, step_t in zip(*runs):
        for x, y in zip(step_f, step_t):
            assert np.array_equal(x, y)
    for cin, o, k, *rest in runs[0][:2]:
        if labor:
            co, ko, lo, _ = corc.labor_egm_step(cin, a, s, P, r, w, 0.96, 5.0, 1.0, 1.0, cal["amin"])
            assert np.array_equal(rest[0], lo)
        else:  # (corc works on [N][Na], the device layout)
            co, ko, _ = corc.egm_step(cin, a, s, P, r, w, 0.96, 5.0, cal["amin"])
        assert np.array_equal(o, co) and np.array_equal(k, ko)


def test_egm_nonmonotone_grid_is_reported_large_grid(pkg, gpu):
    """Na > 1024: the two-launch step (flag word) reports a folding â like the small-grid
    step, with and without the segment windows (EGM knob bit 20)."""
    import torch
    a = np.linspace(0, 10, 5000)
    pc0 = np.tile(np.linspace(50, 0.01, 5000)[:, None], (1, 2))
    with pytest.raises(pkg.AiyError) as e:
        pkg.egm_step(pc0, a, np.array([1.0, 1.2]), np.full((2, 2), 0.5), 0.02, 1.0, 0.96, 5.0, 0.0)
    assert e.value.status == "AIY_BAD_ARG"
    with pytest.raises(pkg.AiyError):
        pkg.egm_solve(pc0, a, np.array([1.0, 1.2]), np.full((2, 2), 0.5), 0.02, 1.0, 0.96, 5.0,
                      0.0, 1e-6, 50)
    dev = torch.device("cuda", 0)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    for var in (-1, 1 << 20):
        ws = pkg.Workspace(2, 5000)
        ws.set_variant(var)
        c = t(pc0.T)
        o, k = torch.empty_like(c), torch.empty_like(c)
        dd = torch.zeros(2, dtype=torch.int64, device=dev)
        pkg.egm_step_dev(ws, c, t(a), t(np.array([1.0, 1.2])), t(np.full((2, 2), 0.5)), 0.02, 1.0,
                         0.96, 5.0, 0.0, o, k, diff=dd)
        torch.cuda.synchronize()  # device tier: no error return, the step still completes


@pytest.mark.parametrize("Na", [10000, 1500])
def test_egm_n1_large_grid_solve(pkg, gpu, Na):
    """N = 1 with more than 64 tiles (the slot clearing of the two-launch step) —
    the speculative solve on both large-grid paths equals the C loop."""
    a = no.calib_aiyagari(Na=Na)["a_grid"]
    s, P = np.array([1.0]), np.array([[1.0]])
    w = no.wage(0.03, 0.36, 0.08)
    pc0 = ((1.03) * a + w)[:, None]
    Ro = corc.egm_solve(pc0.T, a, s, P, 0.03, w, 0.96, 5.0, 0.0, 1e-6, 300)
    R = pkg.egm_solve(pc0, a, s, P, 0.03, w, 0.96, 5.0, 0.0, 1e-6, 300)
    assert R["iters"] == Ro["iters"] and R["dist"] == Ro["dist"]
    assert np.array_equal(R["policy_c"], Ro["policy_c"].T)
    assert np.array_equal(R["policy_k"], Ro["policy_k"].T)


@pytest.mark.parametrize("Na,N,labor", [(1025, 7, False), (4099, 7, True), (20000, 7, False),
                                        (20000, 7, True), (3000, 1, False), (2000, 16, True)])
def test_egm_chained_solve_dev(pkg, gpu, Na, N, labor):
    """aiy_egm_solve_dev: for Na > 1,024 each step of the speculative solve is ONE launch
    (egm_chain_kernel: interp1 of step t + the Euler RHS of step t+1 on the same tiles) — equal
    bit for bit to the two-launch steps (EGM knob bit 19) and to the C loop: iteration count,
    dist, policy_c, policy_k (and policy_l).  A VFI geometry variant on the same workspace
    (bits 12 | 13 | 14, formerly shared with EGM knobs) leaves the EGM path unchanged."""
    import torch
    dev = torch.device("cuda", 0)
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst", N=N) if N not in (7, 1) else \
        no.calib_aiyagari(Na=Na, shocks="rouwenhorst")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    if N == 1:
        s, P = np.array([1.0]), np.array([[1.0]])
    N = P.shape[0]
    r = 0.03
    w = no.wage(r, 0.36, 0.08)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    pc0 = np.tile(((1 + r) * a + w * np.mean(s))[None, :], (N, 1))
    outs = []
    for var in (-1, 1 << 19, 4096 | 8192 | 16384):
        ws = pkg.Workspace(N, Na)
        if var >= 0:
            ws.set_variant(var)
        c = t(pc0)
        pk = torch.zeros_like(c)
        pl = torch.zeros_like(c) if labor else None
        it, dist = pkg.egm_solve_dev(ws, c, t(a), t(s), t(P), r, w, 0.96, 5.0, cal["amin"], 1e-6,
                                     400, pk, labor=labor, phi=1.0, theta=1.0, policy_l=pl)
        outs.append((it, dist, c.cpu().numpy(), pk.cpu().numpy(),
                     pl.cpu().numpy() if labor else None))
    (i0, d0, c0_, k0, l0) = outs[0]
    for (i1, d1, c1, k1, l1) in outs[1:]:
        assert i0 == i1 and d0 == d1
        assert np.array_equal(c0_, c1) and np.array_equal(k0, k1)
        if labor:
            assert np.array_equal(l0, l1)
    if labor:
        Ro = corc.labor_egm_solve(pc0, a, s, P, r, w, 0.96, 5.0, 1.0, 1.0, cal["amin"], 1e-6, 400)
    else:
        Ro = corc.egm_solve(pc0, a, s, P, r, w, 0.96, 5.0, cal["amin"], 1e-6, 400)
    assert i0 == Ro["iters"] and d0 == Ro["dist"]
    assert np.array_equal(c0_, Ro["policy_c"]) and np.array_equal(k0, Ro["policy_k"])


@pytest.mark.parametrize("Na,N,labor,sigma,theta", [
    (2, 7, False, 5.0, 1.0), (3, 7, True, 5.0, 1.0), (65, 7, False, 5.0, 1.0),
    (400, 7, False, 5.0, 1.0), (400, 7, True, 5.0, 1.0), (400, 7, True, 2.5, 2.0),
    (1024, 7, False, 5.0, 1.0), (700, 7, True, 5.0, 1.0), (300, 16, False, 3.0, 1.0),
    (1000, 1, False, 5.0, 1.0)])
def test_egm_small_grid_solve_dev(pkg, gpu, Na, N, labor, sigma, theta):
    """Small grids (the fused one-launch step inside the speculative device-tier solve): the
    iteration count, policy_c and policy_k equal the C loop bit for bit, for N = 1 … 16, integer
    and non-integer sigma, theta != 1, stops on tol and at max_iter."""
    import torch
    dev = torch.device("cuda", 0)
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst", N=N) if N not in (7, 1) else \
        no.calib_aiyagari(Na=Na, shocks="rouwenhorst")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    if N == 1:
        s, P = np.array([1.0]), np.array([[1.0]])
    N = P.shape[0]
    r = 0.03
    w = no.wage(r, 0.36, 0.08)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    pc0 = np.tile(((1 + r) * a + w * np.mean(s))[None, :], (N, 1))
    for tol, max_iter in ((1e-6, 400), (1e-3, 400), (1e-6, 9)):
        ws = pkg.Workspace(N, Na)
        c = t(pc0)
        pk = torch.zeros_like(c)
        pl = torch.zeros_like(c) if labor else None
        it, dist = pkg.egm_solve_dev(ws, c, t(a), t(s), t(P), r, w, 0.96, sigma, cal["amin"],
                                     tol, max_iter, pk, labor=labor, phi=1.0, theta=theta,
                                     policy_l=pl)
        ws.close()
        if labor:
            Ro = corc.labor_egm_solve(pc0, a, s, P, r, w, 0.96, sigma, 1.0, theta, cal["amin"],
                                      tol, max_iter)
            assert np.array_equal(pl.cpu().numpy(), Ro["policy_l"])
        else:
            Ro = corc.egm_solve(pc0, a, s, P, r, w, 0.96, sigma, cal["amin"], tol, max_iter)
        assert it == Ro["iters"]
        assert np.array_equal(c.cpu().numpy(), Ro["policy_c"])
        assert np.array_equal(pk.cpu().numpy(), Ro["policy_k"])
