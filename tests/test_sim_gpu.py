"""GPU parity for A9 (Aiyagari_VFI.m:104-129): the Monte-Carlo capital-supply chain with
MATLAB's fresh-session MT19937 stream, bit-exact against the golden path (numpy restatement)."""
import numpy as np
import pytest

from oracle import corc
from oracle import np_oracle as no

pytestmark = pytest.mark.gpu


def test_sim_matches_golden_path(pkg, gpu, golden):
    g = golden("a11_ge_vfi_defaults")
    a1 = golden("a1_vfi_defaults")
    R = corc.vfi_solve(np.zeros((7, 400)), a1["a_grid"], a1["s"], a1["P"], 0.04,
                       float(a1["w"]), 0.96, 5.0)
    U = no.matlab_rand_stream(2 + 9999)[2:]
    Ks, path, zp = pkg.sim_capital(R["policy_k"], a1["a_grid"], a1["P"], int(g["z1"]) + 1,
                                   float(g["k1"]), U, return_path=True)
    assert Ks == float(g["Ks0"])
    assert np.array_equal(path, g["sim_k0"])
    assert np.array_equal(zp - 1, g["sim_z0"])


@pytest.mark.parametrize("Na", [400, 3000, 20000])
def test_sim_offgrid_egm_layout(pkg, gpu, Na):
    """Off-grid (EGM) policies in the Na x N layout, LDS and L2 paths, extrapolation at both
    ends: bit-exact vs the C restatement."""
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst")
    a, P = cal["a_grid"], cal["P"]
    rng = np.random.default_rng(Na)
    pol = np.sort(rng.uniform(-1, a[-1] * 1.05, (Na, 7)), axis=0)  # off-grid, beyond the ends
    U = rng.random(9999)
    Ks, path, zp = pkg.sim_capital(pol, a, P, 3, a[Na // 2] + 0.123, U, vfi_layout=False,
                                   return_path=True)
    Ko, po = corc.sim_capital(pol.T, a, P, 2, a[Na // 2] + 0.123, U, return_path=True)
    assert np.array_equal(path, po)
    assert Ks == Ko


@pytest.mark.parametrize("Na,t_bad", [(400, 5), (400, 2100), (400, 6000), (1500, 2100)])
def test_sim_find_empty_late_in_the_chain(pkg, gpu, Na, t_bad):
    """find() empty at a step in a later chunk (the two-wave kernel's state walker runs one
    chunk ahead of the capital recurrence): the same error, and the C restatement agrees."""
    rng = np.random.default_rng(Na + t_bad)
    a = np.sort(rng.uniform(0, 50, Na))
    a[0] = 0.0
    N = 7
    P = rng.random((N, N)) + 0.05
    P /= P.sum(axis=1, keepdims=True) * (1 + 1e-6)  # rows sum below 1
    U = rng.random(9999) * 0.99
    U[t_bad - 1] = 0.9999999  # above every row sum: step t_bad finds nothing
    pol = np.sort(rng.uniform(0, a[-1], (N, Na)), axis=1)
    with pytest.raises(pkg.AiyError) as e:
        pkg.sim_capital(pol, a, P, 3, float(a[Na // 2]), U)
    assert e.value.status == "AIY_FIND_EMPTY"


def test_sim_find_empty_is_an_error(pkg, gpu):
    P = np.array([[0.5, 0.4999], [0.5, 0.5]])  # row 1 sums below 1
    with pytest.raises(pkg.AiyError) as e:
        pkg.sim_capital(np.zeros((2, 3)), np.array([0.0, 1.0, 2.0]), P, 1, 0.0,
                        np.array([0.99995]))
    assert e.value.status == "AIY_FIND_EMPTY"


@pytest.mark.parametrize("N,Na,T", [(7, 400, 1), (7, 400, 2), (7, 400, 65), (7, 400, 4097),
                                    (1, 50, 300), (3, 2, 300), (5, 37, 1000), (16, 300, 3000),
                                    (15, 1100, 3000), (7, 3000, 2049), (7, 400, 10000),
                                    (7, 448, 2200), (7, 449, 2200), (7, 960, 4200),
                                    (8, 448, 700), (8, 449, 700), (7, 64, 300), (7, 63, 300),
                                    (7, 1500, 3000), (15, 480, 700)])
def test_sim_chain_shapes_and_jumps(pkg, gpu, N, Na, T):
    """Chain kernel edge cases vs the C restatement: T = 1, block/chunk boundaries (64, 2048,
    the GE's T = 10,000 with a 15-step tail), tiny grids (Na < 64 window), N = 1 and the N = 16
    wide-state path, the two-wave kernel at both table strides and their edges (Na = 64,
    448 / 449, 960 at N = 7; N = 8 at 448 and past it), the window kernel beyond (Na = 63,
    N = 15, Na = 1,100 / 1,500) and the global-memory path, and policies that jump across the
    grid every step (the 64-point window misses, the full search runs)."""
    rng = np.random.default_rng(N * 1000 + Na)
    a = np.sort(rng.uniform(0, 50, Na))
    a[0] = 0.0
    P = rng.random((N, N)) + 0.05
    P /= P.sum(axis=1, keepdims=True)
    P[:, -1] += 1e-9  # rows sum above 1: find() never empty
    for jumpy in (False, True):
        if jumpy:
            pol = rng.uniform(-5, 60, (N, Na))
        else:
            pol = np.sort(rng.uniform(0, a[-1], (N, Na)), axis=1)
        U = rng.random(T - 1)
        k1 = float(a[Na // 2])
        Ks, path, zp = pkg.sim_capital(pol, a, P, N, k1, U, return_path=True)
        Ko, po = corc.sim_capital(pol, a, P, N - 1, k1, U, return_path=True)
        assert np.array_equal(path, po, equal_nan=True)
        assert Ks == Ko or (np.isnan(Ks) and np.isnan(Ko))
        assert zp.shape == (T,) and zp[0] == N and zp.min() >= 1 and zp.max() <= N


@pytest.mark.parametrize("Na", [60, 400, 2100, 20000])
def test_sim_mean_only(pkg, gpu, Na):
    """K_s without the path (the GE drivers' call: no sim_k/sim_z stores), LDS-padded and L2
    variants, vs the C restatement."""
    cal = no.calib_aiyagari(Na=Na, shocks="rouwenhorst")
    a, P = cal["a_grid"], cal["P"]
    rng = np.random.default_rng(Na + 1)
    pol = np.sort(rng.uniform(0, a[-1], (7, Na)), axis=1)
    U = rng.random(9999)
    Ks = pkg.sim_capital(pol, a, P, 4, float(a[Na // 3]), U)
    Ko = corc.sim_capital(pol, a, P, 3, float(a[Na // 3]), U)
    assert Ks == Ko
