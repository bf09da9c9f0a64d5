"""GPU: the speculative-segment A9 chain (sim_chain_par_kernel) against the
serial chain kernels and the C restatement, bit for bit (Aiyagari_VFI.m:104-129).  Device tier,
the mode forced per workspace (aiy_ws_set_sim: 1 speculative in one workgroup, 2 the spread
four-launch variant, 0 serial), so the short chains the size rule would send to the serial
kernels run through the segments too.
The adversarial case is a policy whose paths never coalesce (k' = k + 0.5 everywhere, linear
extrapolation): every speculative start is wrong, each repair pass makes exactly one more
segment true, and the chain needs all 15 passes with every segment overwritten whole."""
import numpy as np
import pytest

from oracle import corc

pytestmark = pytest.mark.gpu


def _grid(rng, Na):
    a = np.sort(rng.uniform(0, 50, Na))
    a[0] = 0.0
    return a


def _P(rng, N):
    P = rng.random((N, N)) + 0.05
    P /= P.sum(axis=1, keepdims=True)
    P[:, -1] += 1e-9  # rows sum above 1: find() never empty
    return P


def _run(pkg, ws, mode, pol, a, P, z1, k1, U, path=True):
    import torch
    dev = "cuda:0"
    tt = lambda x: torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=dev)
    T = U.size + 1
    ks = torch.full((1,), np.nan, dtype=torch.float64, device=dev)
    st = torch.full((1,), -1, dtype=torch.int32, device=dev)
    sk = torch.full((T,), np.nan, dtype=torch.float64, device=dev) if path else None
    sz = torch.full((T,), -1, dtype=torch.int32, device=dev) if path else None
    ws.set_sim(mode)
    pkg.sim_capital_dev(ws, tt(pol), tt(a), tt(P), z1, k1, tt(U), ks, st, sim_k=sk, sim_z=sz)
    torch.cuda.synchronize()
    return (float(ks[0]), int(st[0]), sk.cpu().numpy() if path else None,
            sz.cpu().numpy() if path else None)


@pytest.mark.parametrize("N,Na,T", [(7, 400, 2), (7, 400, 3), (7, 400, 17), (7, 400, 18),
                                    (7, 400, 100), (7, 64, 2049), (1, 200, 500), (7, 960, 4200),
                                    (3, 500, 10000), (7, 400, 16384)])
@pytest.mark.parametrize("kind", ["smooth", "jumpy", "drift"])
@pytest.mark.parametrize("mode", [1, 2])
def test_par_chain_equals_serial_and_oracle(pkg, gpu, N, Na, T, kind, mode):
    """Every segment count edge (T - 1 below, at and above 16 steps; empty segments), the
    smallest grid (Na = 64) and the largest LDS table (Na = 960), N = 1, T at the LDS bound."""
    rng = np.random.default_rng(N * 100003 + Na * 7 + T)
    a = _grid(rng, Na)
    P = _P(rng, N)
    if kind == "smooth":
        pol = np.sort(rng.uniform(0, a[-1], (N, Na)), axis=1)
    elif kind == "jumpy":
        pol = rng.uniform(-5, 60, (N, Na))
    else:
        pol = np.tile(a + 0.5, (N, 1))
    U = rng.random(T - 1)
    z1, k1 = N - 1, float(a[Na // 2])
    ws = pkg.Workspace(N, Na)
    try:
        Kp, sp, kp, zp = _run(pkg, ws, mode, pol, a, P, z1, k1, U)
        Ks, ss, ksr, zs = _run(pkg, ws, 0, pol, a, P, z1, k1, U)
        Km, sm, _, _ = _run(pkg, ws, mode, pol, a, P, z1, k1, U, path=False)
    finally:
        ws.close()
    Ko, po = corc.sim_capital(pol, a, P, z1, k1, U, return_path=True)
    assert sp == ss == sm == 0
    assert np.array_equal(kp, ksr, equal_nan=True) and np.array_equal(kp, po, equal_nan=True)
    assert np.array_equal(zp, zs)
    # jumpy policies extrapolate to +-inf on long chains: the means are then NaN alike
    same = lambda x, y: x == y or (np.isnan(x) and np.isnan(y))
    assert same(Kp, Ks) and same(Kp, Km) and same(Kp, Ko)
    if kind == "drift":  # the never-coalescing case really is one: k_t = k_1 + t / 2
        assert kp[-1] == pytest.approx(k1 + 0.5 * (T - 1), rel=1e-9)


@pytest.mark.parametrize("T,t_bad", [(10000, 2), (10000, 626), (10000, 9999), (300, 40),
                                     (20, 19)])
@pytest.mark.parametrize("mode", [1, 2])
def test_par_chain_find_empty(pkg, gpu, T, t_bad, mode):
    """find() empty at step t_bad (first step, a segment boundary, the last step, short
    chains): the speculative chain stops there as the serial one does — status 1, and the path
    before t_bad and the z path agree."""
    N, Na = 7, 400
    rng = np.random.default_rng(T + t_bad)
    a = _grid(rng, Na)
    P = rng.random((N, N)) + 0.05
    P /= P.sum(axis=1, keepdims=True) * (1 + 1e-6)  # rows sum below 1
    U = rng.random(T - 1) * 0.99
    U[t_bad - 1] = 0.9999999
    pol = np.sort(rng.uniform(0, a[-1], (N, Na)), axis=1)
    ws = pkg.Workspace(N, Na)
    try:
        Kp, sp, kp, zp = _run(pkg, ws, mode, pol, a, P, 2, float(a[Na // 2]), U)
        Ks, ss, ksr, zs = _run(pkg, ws, 0, pol, a, P, 2, float(a[Na // 2]), U)
    finally:
        ws.close()
    assert sp == ss == 1
    assert np.array_equal(kp[:t_bad], ksr[:t_bad])
    assert np.array_equal(zp[:t_bad], zs[:t_bad])
    assert Kp == Ks or (np.isnan(Kp) and np.isnan(Ks))


def test_par_chain_shape_rule_falls_back(pkg, gpu):
    """Shapes the speculative chain does not take (N = 8, Na past the LDS table, T past the z
    buffer) run the serial kernels under mode 1: the same results as mode 0."""
    rng = np.random.default_rng(5)
    for N, Na, T in [(8, 300, 3000), (7, 1000, 3000), (7, 300, 16385)]:
        a = _grid(rng, Na)
        P = _P(rng, N)
        pol = np.sort(rng.uniform(0, a[-1], (N, Na)), axis=1)
        U = rng.random(T - 1)
        ws = pkg.Workspace(N, Na)
        try:
            r1 = _run(pkg, ws, 1, pol, a, P, 0, float(a[3]), U)
            r2 = _run(pkg, ws, 2, pol, a, P, 0, float(a[3]), U)
            r0 = _run(pkg, ws, 0, pol, a, P, 0, float(a[3]), U)
        finally:
            ws.close()
        assert r1[0] == r2[0] == r0[0] and r1[1] == r2[1] == r0[1] == 0
        assert np.array_equal(r1[2], r0[2]) and np.array_equal(r2[2], r0[2])
