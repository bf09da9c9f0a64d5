"""F4 (Aiyagari_VFI.m:314-410): Gini / Lorenz / quintile shares of the host mirror against a
literal element-by-element transcription of the script's lines, and the weighted (histogram)
version against the sample version on an equal-weight sample."""
import math

import numpy as np
import pytest


def _literal_gini(x):
    xs = sorted(float(v) for v in x)
    n = len(xs)
    tot = 0.0
    for v in xs:
        tot += v
    cum, acc = [], 0.0
    for v in xs:
        acc += v
        cum.append(acc / tot)
    pop = [(i + 1) / n for i in range(n)]
    area = 0.0
    for i in range(n - 1):
        area += (pop[i + 1] - pop[i]) * (cum[i] + cum[i + 1]) / 2
    return 1 - 2 * area


def test_gini_matches_literal(pkg):
    x = np.random.default_rng(0).lognormal(0, 1, 999)
    assert pkg.stats.gini(x) == pytest.approx(_literal_gini(x), abs=1e-13)


def test_quintiles_round_half_away(pkg):
    assert pkg.stats.matlab_round(2.5) == 3 and pkg.stats.matlab_round(-2.5) == -3
    x = np.arange(1, 13, dtype=float)          # n = 12: round(2.4)=2, round(4.8)=5, 7.2->7, 9.6->10
    sh = pkg.stats.quintile_shares(x)
    tot = x.sum()
    exp = [x[:2].sum(), x[2:5].sum(), x[5:7].sum(), x[7:10].sum(), x[10:].sum()]
    assert sh == pytest.approx([e / tot * 100 for e in exp], abs=1e-12)
    assert sum(sh) == pytest.approx(100.0, abs=1e-12)


def test_weighted_agrees_with_sample(pkg):
    """Equal weights: the weighted curve adds the (0,0)-(1/n, c1) trapezoid the scripts' formula
    omits, so weighted Gini = sample Gini - c1/n with c1 = min(x)/sum(x)."""
    x = np.random.default_rng(1).gamma(2.0, 1.0, 4000)
    g_s = pkg.stats.gini(x)
    g_w = pkg.stats.gini_weighted(x, np.ones_like(x))
    assert g_w == pytest.approx(g_s - (x.min() / x.sum()) / x.size, abs=1e-12)
    # a degenerate distribution has zero inequality
    assert pkg.stats.gini_weighted(np.full(10, 3.0), np.ones(10)) == pytest.approx(0.0, abs=1e-15)


def test_histogram_stats(pkg, golden):
    """On the committed A10 stationary histogram: shares sum to 100, Gini in (0, 1), and the
    bottom quintile holds the least wealth."""
    from oracle import np_oracle as no
    g = golden("a10_dist_defaults")
    lam = g["lam1"]
    a = no.calib_aiyagari()["a_grid"]          # the fixture's grid (Na = 400 defaults)
    assert lam.shape == (7, a.size)
    st = pkg.stats.histogram_wealth_stats(lam, a)
    assert 0 < st["gini_wealth"] < 1
    sh = st["wealth_quintile_shares"]
    assert sum(sh) == pytest.approx(100.0, abs=1e-9) and sh[0] == min(sh) and sh[4] == max(sh)
    assert not math.isnan(st["gini_wealth"])
