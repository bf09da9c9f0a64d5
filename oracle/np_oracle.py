"""numpy restatement of the reference's hot-path loops, in the MATLAB evaluation order.

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (``aiyagari-replication_amd/``)
imports this module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may use it, and only as the checker.

Parity status: **unpinned against MATLAB**.  The reference (kostastril/Aiyagari-Replication)
is six MATLAB scripts with no tests and no fixtures, and neither MATLAB nor Octave exists in
this image, so no reference output could be produced here.  This restatement is pinned
instead by (i) agreement with the independent C restatement in ``oracle/aiy_oracle.c``
(``tests/test_oracle_golden.py``), and (ii) MATLAB's documented fresh-session ``rand``
values (0.8147, 0.9058, 0.1270 ... = MT19937 seed 5489), which numpy's ``RandomState(5489)``
reproduces.

Every function cites the reference lines it restates.  Conventions:
  * arrays indexed as MATLAB does, 0-based here: ``v[i, j]`` is ``v_old(i+1, j+1)``;
  * ``max`` ignores NaN and returns the FIRST maximiser;
  * ``(beta*P(i,:))*v_old`` is evaluated as a sequential sum over m = 1..N;
  * integer CRRA powers use ``ipow`` (left-to-right binary powering), non-integer ones ``pow``.
"""
from __future__ import annotations

import math
import numpy as np

# ----------------------------------------------------------------------------------------
# scalar helpers shared by every restatement
# ----------------------------------------------------------------------------------------


def ipow(c, n: int):
    """c**n for integer n >= 1 by MSB-first binary powering (the product kernels use the
    same sequence, so integer-power results are reproducible bit for bit)."""
    assert n >= 1
    r = c
    for bit in bin(n)[3:]:
        r = r * r
        if bit == "1":
            r = r * c
    return r


def crra_pow(c, sigma: float):
    """c.^(1-sigma) as used by Aiyagari_VFI.m:77; integer sigma >= 2 → 1/c^(sigma-1)."""
    if float(sigma).is_integer() and sigma >= 2:
        return 1.0 / ipow(c, int(sigma) - 1)
    return np.power(c, 1.0 - sigma)


def uprime_pow(c, sigma: float):
    """c.^(-sigma) (Aiyagari_EGM.m:68); integer sigma >= 1 → 1/c^sigma."""
    if float(sigma).is_integer() and sigma >= 1:
        return 1.0 / ipow(c, int(sigma))
    return np.power(c, -sigma)


def matlab_linspace01(n: int):
    """linspace(0,1,n) with the endpoints pinned and interior points i/(n-1)."""
    if n == 1:
        return np.array([1.0])
    y = np.arange(n, dtype=np.float64) / float(n - 1)
    y[0] = 0.0
    y[-1] = 1.0
    return y


def nan_first_argmax(vals):
    """MATLAB [m, idx] = max(vals): NaN ignored, first index; all-NaN → (NaN, 0)."""
    vals = np.asarray(vals)
    ok = ~np.isnan(vals)
    if not ok.any():
        return math.nan, 0
    k = int(np.nanargmax(vals))  # numpy returns the first occurrence
    return float(vals[k]), k


def nanmax_all(x):
    """max(x, [], 'all') ignoring NaN (NaN only if all entries are NaN)."""
    x = np.asarray(x)
    if np.all(np.isnan(x)):
        return math.nan
    return float(np.nanmax(x))


# ----------------------------------------------------------------------------------------
# calibration (host-side L1).  P is an INPUT to every kernel.
# ----------------------------------------------------------------------------------------


def _norm_cdf(x):
    return 0.5 * math.erfc(-x / math.sqrt(2.0))


def tauchen_reference(rho: float, sigma_e: float, N: int = 7):
    """Aiyagari_VFI.m:18-35.  l_grid=(i-4)σe; P(i,j)=∫ normpdf(x, ρ l_i, σe√(1-ρ²)) over the
    hard-coded 7-interval edges (:23).  The integral is evaluated in closed form by normcdf
    differences (MATLAB's integral(AbsTol 1e-10) is not reproducible bit for bit)."""
    assert N == 7, "the reference's interval table (Aiyagari_VFI.m:23) only exists for N=7"
    l_grid = np.array([(i - 3) * sigma_e for i in range(N)])
    edges = [-math.inf, -2.5 * sigma_e, -1.5 * sigma_e, -0.5 * sigma_e, 0.5 * sigma_e,
             1.5 * sigma_e, 2.5 * sigma_e, math.inf]
    sd = sigma_e * math.sqrt(1.0 - rho ** 2)
    P = np.zeros((N, N))
    for i in range(N):
        mu = rho * l_grid[i]
        for j in range(N):
            lo, hi = edges[j], edges[j + 1]
            zl = -math.inf if lo == -math.inf else (lo - mu) / sd
            zh = math.inf if hi == math.inf else (hi - mu) / sd
            if zl > 0:  # upper tail: difference of survival functions (no cancellation)
                P[i, j] = 0.5 * math.erfc(zl / math.sqrt(2.0)) - (
                    0.0 if zh == math.inf else 0.5 * math.erfc(zh / math.sqrt(2.0)))
            else:
                P[i, j] = (1.0 if zh == math.inf else _norm_cdf(zh)) - (
                    0.0 if zl == -math.inf else _norm_cdf(zl))
    return l_grid, P


def rouwenhorst(rho: float, sigma_y: float, N: int):
    """Rouwenhorst discretisation (BASELINE config 2: Nz=7, ρ=.75, unconditional σ=.75)."""
    p = (1.0 + rho) / 2.0
    Pm = np.array([[p, 1 - p], [1 - p, p]])
    for n in range(3, N + 1):
        Z = np.zeros((n, n))
        Z[:-1, :-1] += p * Pm
        Z[:-1, 1:] += (1 - p) * Pm
        Z[1:, :-1] += (1 - p) * Pm
        Z[1:, 1:] += p * Pm
        Z[1:-1, :] /= 2.0
        Pm = Z
    psi = math.sqrt(N - 1) * sigma_y
    grid = np.linspace(-psi, psi, N)
    return grid, Pm


def stationary_dist(P):
    """Aiyagari_VFI.m:39-42: [P'-I; 1'] \\ [0; 1] (least squares)."""
    N = P.shape[0]
    A = np.vstack([P.T - np.eye(N), np.ones((1, N))])
    b = np.zeros(N + 1)
    b[-1] = 1.0
    return np.linalg.lstsq(A, b, rcond=None)[0]


def wage(r, alpha, delta):
    """Aiyagari_VFI.m:67."""
    return (1 - alpha) * (alpha / (r + delta)) ** (alpha / (1 - alpha))


def asset_grid(Na, alpha, beta, delta, b, s1):
    """Aiyagari_VFI.m:53-58."""
    wmin = (1 - alpha) * (alpha / ((1 / beta - 1) + delta)) ** (alpha / (1 - alpha))
    amin = min(b, wmin * s1)
    kmax = delta ** (1 / (alpha - 1))
    amax = kmax ** alpha + (1 - delta) * kmax
    x = matlab_linspace01(Na)
    return amin + (amax - amin) * (x * x), amin


def calib_aiyagari(Na=400, rho=0.75, sigma_e=0.75, beta=0.96, sigma=5.0, alpha=0.36,
                   delta=0.08, b=0.0, shocks="tauchen", N=7):
    """Aiyagari_VFI.m:7-63 (the other three Aiyagari scripts differ only in ρ, σe, extras)."""
    if shocks == "tauchen":
        l_grid, P = tauchen_reference(rho, sigma_e, N)
    else:
        l_grid, P = rouwenhorst(rho, sigma_e, N)
    pi = stationary_dist(P)
    s = np.exp(l_grid)
    labor = float(s @ pi)
    a_grid, amin = asset_grid(Na, alpha, beta, delta, b, s[0])
    return dict(P=P, s=s, labor=labor, a_grid=a_grid, amin=amin, beta=beta, sigma=sigma,
                alpha=alpha, delta=delta, N=N, Na=Na)


# ----------------------------------------------------------------------------------------
# A1/A2  Aiyagari VFI
# ----------------------------------------------------------------------------------------


def ev_rows(P, V, beta):
    """(β·P(i,:))·v_old for every i (Aiyagari_VFI.m:79; …Labor_VFI.m:69): sequential m-sum."""
    N = P.shape[0]
    bP = beta * P
    EV = np.zeros_like(V)
    for m in range(N):
        EV = EV + bP[:, m][:, None] * V[m][None, :]
    return EV


def vfi_sweep(v_old, a_grid, s, P, r, w, beta, sigma):
    """Aiyagari_VFI.m:70-83 for all (i, j).  Returns v_new, idx (0-based), policy_k, policy_c."""
    N, Na = v_old.shape
    EV = ev_rows(P, v_old, beta)
    v_new = np.zeros((N, Na))
    idx = np.zeros((N, Na), dtype=np.int64)
    pk = np.zeros((N, Na))
    pc = np.zeros((N, Na))
    for i in range(N):
        coh = (1 + r) * a_grid + w * s[i]                         # :72 (per j)
        C = coh[:, None] - a_grid[None, :]
        with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
            C = np.where(C <= 0, np.nan, C)                       # :73
            if sigma == 1:
                U = np.log(C)                                     # :75
            else:
                U = (crra_pow(C, sigma) - 1) / (1 - sigma)        # :77
            T = U + EV[i][None, :]                                # :79
        for j in range(Na):
            m, k = nan_first_argmax(T[j])
            v_new[i, j] = m
            idx[i, j] = k
        pk[i] = a_grid[idx[i]]                                    # :80
        pc[i] = coh - pk[i]                                       # :81
    return v_new, idx, pk, pc


def vfi_solve(v_old, a_grid, s, P, r, w, beta, sigma, tol=1e-5, max_iter=1000):
    """Aiyagari_VFI.m:65-90: break BEFORE v_old = v_new, so the caller keeps both."""
    v_old = np.array(v_old, dtype=np.float64)
    it = 0
    for it in range(1, max_iter + 1):
        v_new, idx, pk, pc = vfi_sweep(v_old, a_grid, s, P, r, w, beta, sigma)
        if nanmax_all(np.abs(v_new - v_old)) < tol:               # :85
            break
        v_old = v_new                                             # :88
    return dict(v_new=v_new, v_old=v_old, idx=idx, policy_k=pk, policy_c=pc, iters=it)


# ----------------------------------------------------------------------------------------
# A3  endogenous-labour VFI
# ----------------------------------------------------------------------------------------


def labor_vfi_sweep(v_old, v_prev, pol_prev, a_grid, s, P, r, w, beta, sigma, labor_choice,
                    psi, eta):
    """Aiyagari_Endogenous_Labor_VFI.m:69-112.  v_prev / pol_prev are the values left over
    from the previous sweep (states without a feasible choice keep them, :85)."""
    N, Na = v_old.shape
    L = np.asarray(labor_choice, dtype=np.float64)
    Nl = L.size
    EV = ev_rows(P, v_old, beta)                                  # :69
    v_new = np.array(v_prev, dtype=np.float64)
    pk, pl, pc, lin = (np.array(p) for p in pol_prev)
    if float(1 + eta).is_integer() and 1 + eta >= 1:
        Lp = ipow(L, int(1 + eta))
    else:
        Lp = np.power(L, 1 + eta)
    dis = psi * Lp / (1 + eta)                                    # :96
    for i in range(N):
        for j in range(Na):
            x = (1 + r) * a_grid[j]
            y = w * s[i]
            C = (x + (y * L)[:, None]) - a_grid[None, :]          # :81, rows l, cols k
            valid = C > 0
            if not valid.any():
                continue
            with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
                U = np.where(valid, (crra_pow(np.where(valid, C, 1.0), sigma) - 1) / (1 - sigma)
                             - dis[:, None], -np.inf)
                T = U + EV[i][None, :]
            flat = T.flatten(order="F")                            # column-major (:102)
            m, q = nan_first_argmax(flat)
            li, ki = q % Nl, q // Nl
            pl[i, j] = L[li]
            pk[i, j] = a_grid[ki]
            pc[i, j] = C[li, ki]
            lin[i, j] = q
            v_new[i, j] = m
    return v_new, (pk, pl, pc, lin)


def labor_vfi_solve(v_old, a_grid, s, P, r, w, beta, sigma, labor_choice, psi, eta, tol=1e-5,
                    max_iter=1000, v_prev=None, pol_prev=None):
    """Aiyagari_Endogenous_Labor_VFI.m:64-122."""
    N, Na = v_old.shape
    v_old = np.array(v_old, dtype=np.float64)
    v_new = np.zeros((N, Na)) if v_prev is None else np.array(v_prev)
    pol = pol_prev if pol_prev is not None else (np.zeros((N, Na)), np.zeros((N, Na)),
                                                 np.zeros((N, Na)), np.zeros((N, Na), np.int64))
    it = 0
    for it in range(1, max_iter + 1):
        v_new, pol = labor_vfi_sweep(v_old, v_new, pol, a_grid, s, P, r, w, beta, sigma,
                                     labor_choice, psi, eta)
        if nanmax_all(np.abs(v_new - v_old)) < tol:
            break
        v_old = v_new.copy()
    pk, pl, pc, lin = pol
    return dict(v_new=v_new, v_old=v_old, policy_k=pk, policy_l=pl, policy_c=pc, lin=lin,
                iters=it)


# ----------------------------------------------------------------------------------------
# interp1(x, y, xq, 'linear', 'extrap')
# ----------------------------------------------------------------------------------------


def interp1_linear_extrap(x, y, xq):
    """Segment i with x_i <= xq < x_{i+1}, clamped to the end segments for extrapolation;
    y = y_i + t·(y_{i+1}-y_i), t = (xq-x_i)/(x_{i+1}-x_i)."""
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    xq = np.asarray(xq, dtype=np.float64)
    n = x.size
    i = np.searchsorted(x, xq, side="right") - 1
    i = np.clip(i, 0, n - 2)
    t = (xq - x[i]) / (x[i + 1] - x[i])
    return y[i] + t * (y[i + 1] - y[i])


# ----------------------------------------------------------------------------------------
# A4/A5  EGM (policy_c layout Na x N, column j = productivity state)
# ----------------------------------------------------------------------------------------


def egm_rhs(policy_c, P, r, beta, sigma):
    """Aiyagari_EGM.m:80-85: RHS(:,j) += ((β(1+r))·P(j,m))·c_m^(-σ), m ascending."""
    Na, N = policy_c.shape
    RHS = np.zeros((Na, N))
    up = uprime_pow(policy_c, sigma)
    for j in range(N):
        for m in range(N):
            RHS[:, j] = RHS[:, j] + ((beta * (1 + r)) * P[j, m]) * up[:, m]
    return RHS


def egm_step(policy_c, a_grid, s, P, r, w, beta, sigma, amin):
    """Aiyagari_EGM.m:75-107 (one pass of the while loop)."""
    Na, N = policy_c.shape
    RHS = egm_rhs(policy_c, P, r, beta, sigma)
    c_next = np.power(RHS, -1.0 / sigma)                          # :88
    pk = np.zeros((Na, N))
    pcn = np.zeros((Na, N))
    for j in range(N):
        a_hat = ((c_next[:, j] + a_grid) - w * s[j]) / (1 + r)    # :92
        g = interp1_linear_extrap(a_hat, a_grid, a_grid)          # :95
        g = np.where(g < amin, amin, g)                           # :98
        pk[:, j] = g
        pcn[:, j] = ((1 + r) * a_grid + w * s[j]) - g             # :102
    dist = nanmax_all(np.abs(pcn - policy_c))                     # :106
    return pcn, pk, dist


def egm_solve(policy_c, a_grid, s, P, r, w, beta, sigma, amin, tol=1e-5, max_iter=1000):
    """Aiyagari_EGM.m:71-110."""
    dist, it = 1.0, 0
    pk = np.zeros_like(policy_c)
    while dist > tol and it < max_iter:
        it += 1
        policy_c, pk, dist = egm_step(policy_c, a_grid, s, P, r, w, beta, sigma, amin)
    return dict(policy_c=policy_c, policy_k=pk, dist=dist, iters=it)


def labor_egm_step(policy_c, a_grid, s, P, r, w, beta, sigma, phi, theta, amin):
    """Aiyagari_Endogenous_Labor_EGM.m:68-104."""
    Na, N = policy_c.shape
    RHS = egm_rhs(policy_c, P, r, beta, sigma)
    c_next = np.power(RHS, -1.0 / sigma)                          # :82
    pcn = np.zeros((Na, N))
    pl = np.zeros((Na, N))
    pk = np.zeros((Na, N))

    def lab(c, ws):                                               # u_prime_l_inv(ws·c^-σ)
        x = (ws * uprime_pow(c, sigma)) / phi
        return x if 1.0 / theta == 1.0 else np.power(x, 1.0 / theta)

    for j in range(N):
        ws = w * s[j]
        ls = lab(c_next[:, j], ws)                                # :86
        a_hat = ((c_next[:, j] + a_grid) - ws * ls) / (1 + r)     # :87
        g = interp1_linear_extrap(a_hat, c_next[:, j], a_grid)    # :90
        g = np.where(a_grid < amin, amin, g)                      # :91 (no-op)
        pcn[:, j] = g
        pl[:, j] = lab(g, ws)                                     # :95
        k = ((1 + r) * a_grid + ws * pl[:, j]) - g                # :98
        pk[:, j] = np.where(k < 0, 0.0, k)                        # :99
    dist = nanmax_all(np.abs(pcn - policy_c))
    return pcn, pk, pl, dist


def labor_egm_solve(policy_c, a_grid, s, P, r, w, beta, sigma, phi, theta, amin, tol=1e-5,
                    max_iter=1000):
    dist, it = 1.0, 0
    pk = np.zeros_like(policy_c)
    pl = np.zeros_like(policy_c)
    while dist > tol and it < max_iter:
        it += 1
        policy_c, pk, pl, dist = labor_egm_step(policy_c, a_grid, s, P, r, w, beta, sigma,
                                                phi, theta, amin)
    return dict(policy_c=policy_c, policy_k=pk, policy_l=pl, dist=dist, iters=it)


# ----------------------------------------------------------------------------------------
# A9  Monte-Carlo capital supply; A11 GE bisection
# ----------------------------------------------------------------------------------------


def sim_capital(policy_rows, a_grid, P, z1, k1, uniforms):
    """Aiyagari_VFI.m:104-129 (and :174-193).  policy_rows[z] is policy_k(z,:) (VFI layout);
    z1 is 0-based; uniforms has T-1 entries.  Returns (mean, sim_k, sim_z)."""
    T = len(uniforms) + 1
    sim_k = np.zeros(T)
    sim_z = np.zeros(T, dtype=np.int64)
    sim_z[0], sim_k[0] = z1, k1
    cs_rows = []
    for zz in range(P.shape[0]):
        acc, row = 0.0, []
        for m in range(P.shape[1]):
            acc = acc + P[zz, m]
            row.append(acc)
        cs_rows.append(np.array(row))
    for t in range(1, T):
        u = uniforms[t - 1]
        hit = np.nonzero(u < cs_rows[sim_z[t - 1]])[0]
        if hit.size == 0:
            raise ValueError("find(rand < cumsum(P)) returned empty (reference would error)")
        sim_z[t] = hit[0]
        sim_k[t] = interp1_linear_extrap(a_grid, policy_rows[sim_z[t]], np.array([sim_k[t - 1]]))[0]
    acc = 0.0
    for v in sim_k:
        acc += v
    return acc / T, sim_k, sim_z


def matlab_rand_stream(n, seed=5489):
    """Fresh-session MATLAB rand: MT19937(5489), 53-bit doubles."""
    return np.random.RandomState(seed).random_sample(n)


def ge_bisection_vfi(cal, T=10000, max_r_iter=10, r0=0.04, tol=1e-5, max_iter=1000,
                     solve=None, stream=None):
    """Aiyagari_VFI.m:63-206 end to end (initial VFI, MC, 10 bisection steps)."""
    P, s, a, beta, sigma = cal["P"], cal["s"], cal["a_grid"], cal["beta"], cal["sigma"]
    alpha, delta, N, Na = cal["alpha"], cal["delta"], cal["N"], cal["Na"]
    solve = solve or vfi_solve
    need = 2 + (T - 1) * (max_r_iter + 1)
    U = matlab_rand_stream(need) if stream is None else stream
    pos = 0
    z1 = int(math.ceil(N * U[pos])) - 1; pos += 1               # randi(N)
    k1 = a[int(math.ceil(Na * U[pos])) - 1]; pos += 1           # a_grid(randi(grid_size))
    v_old = np.zeros((N, Na))
    r = r0
    res = solve(v_old, a, s, P, r, wage(r, alpha, delta), beta, sigma, tol, max_iter)
    v_old = res["v_old"]
    Ks, _, _ = sim_capital(res["policy_k"], a, P, z1, k1, U[pos:pos + T - 1]); pos += T - 1
    r_low, r_high = -0.05, 1 / beta - 1
    hist = dict(r=[], k_supply=[], k_demand=[], iters=[res["iters"]])
    for _ in range(max_r_iter):
        r_guess = (r_low + r_high) / 2
        r = r_guess
        res = solve(v_old, a, s, P, r, wage(r, alpha, delta), beta, sigma, tol, max_iter)
        v_old = res["v_old"]
        Ks, _, _ = sim_capital(res["policy_k"], a, P, z1, k1, U[pos:pos + T - 1]); pos += T - 1
        Kd = cal["labor"] * (alpha / (r_guess + delta)) ** (1 / (1 - alpha))
        hist["r"].append(r); hist["k_supply"].append(Ks); hist["k_demand"].append(Kd)
        hist["iters"].append(res["iters"])
        if abs(Ks - Kd) < 1e-5:
            break
        elif Ks > Kd:
            r_high = r_guess
        else:
            r_low = r_guess
    hist["r_final"] = r
    return hist


# ----------------------------------------------------------------------------------------
# A10  histogram stationary distribution (new; no reference code → restated from its
#      definition in SURVEY.md §8(a) A10, scatter form)
# ----------------------------------------------------------------------------------------


def dist_update_ongrid(lam, idx, P):
    """λ'(m,k) = Σ_i P(i,m) Σ_{j: idx(i,j)=k} λ(i,j)."""
    N, Na = lam.shape
    mass = np.zeros((N, Na))
    for i in range(N):
        np.add.at(mass[i], idx[i], lam[i])
    return P.T @ mass


def dist_update_lottery(lam, kp, a_grid, P):
    """Off-grid policy: mass at a' split between the bracketing nodes."""
    N, Na = lam.shape
    mass = np.zeros((N, Na))
    for i in range(N):
        x = np.clip(kp[i], a_grid[0], a_grid[-1])
        k = np.clip(np.searchsorted(a_grid, x, side="right") - 1, 0, Na - 2)
        wr = (x - a_grid[k]) / (a_grid[k + 1] - a_grid[k])
        np.add.at(mass[i], k, lam[i] * (1 - wr))
        np.add.at(mass[i], k + 1, lam[i] * wr)
    return P.T @ mass


# ----------------------------------------------------------------------------------------
# A6/A7  Krusell-Smith VFI pieces (pchip, fminbnd, bellman_value, Howard)
# ----------------------------------------------------------------------------------------


def _sign(x):
    x = float(x)
    return int(x > 0) - int(x < 0)


def pchip_slopes(x, y):
    """MATLAB pchip slopes (Fritsch–Butland weighted harmonic mean; 3-point end rule)."""
    n = len(x)
    h = np.diff(x)
    dl = np.diff(y) / h
    d = np.zeros(n)
    for k in range(n - 2):
        if _sign(dl[k]) * _sign(dl[k + 1]) > 0:
            h1, h2 = h[k], h[k + 1]
            hs = h1 + h2
            w1 = (h1 + hs) / (3 * hs)
            w2 = (hs + h2) / (3 * hs)
            dmax = max(abs(dl[k]), abs(dl[k + 1]))
            dmin = min(abs(dl[k]), abs(dl[k + 1]))
            d[k + 1] = dmin / (w1 * (dl[k] / dmax) + w2 * (dl[k + 1] / dmax))
    d0 = ((2 * h[0] + h[1]) * dl[0] - h[0] * dl[1]) / (h[0] + h[1])
    if _sign(d0) != _sign(dl[0]):
        d0 = 0.0
    elif _sign(dl[0]) != _sign(dl[1]) and abs(d0) > abs(3 * dl[0]):
        d0 = 3 * dl[0]
    d[0] = d0
    dn = ((2 * h[n - 2] + h[n - 3]) * dl[n - 2] - h[n - 2] * dl[n - 3]) / (h[n - 2] + h[n - 3])
    if _sign(dn) != _sign(dl[n - 2]):
        dn = 0.0
    elif _sign(dl[n - 2]) != _sign(dl[n - 3]) and abs(dn) > abs(3 * dl[n - 2]):
        dn = 3 * dl[n - 2]
    d[n - 1] = dn
    return d


def pchip_eval(x, y, d, xq):
    """pwch/ppval: c3=(dzdxdx-dzzdx)/h, c2=2dzzdx-dzdxdx, c1=d_i, c0=y_i, Horner in s=xq-x_i."""
    n = len(x)
    i = int(np.searchsorted(x, xq, side="right") - 1)
    i = min(max(i, 0), n - 2)
    h = x[i + 1] - x[i]
    dl = (y[i + 1] - y[i]) / h
    dzzdx = (dl - d[i]) / h
    dzdxdx = (d[i + 1] - dl) / h
    c3 = (dzdxdx - dzzdx) / h
    c2 = 2 * dzzdx - dzdxdx
    sx = xq - x[i]
    v = c3
    v = sx * v + c2
    v = sx * v + d[i]
    v = sx * v + y[i]
    return v


def fminbnd(f, ax, bx, tolx=1e-4, maxfun=500, maxiter=500):
    """MATLAB fminbnd (Brent/FMM) with MATLAB's constants: seps = sqrt(eps), TolX 1e-4."""
    seps = math.sqrt(2.220446049250313e-16)
    c = 0.5 * (3.0 - math.sqrt(5.0))
    a, b = ax, bx
    v = a + c * (b - a)
    w = v
    xf = v
    d = 0.0
    e = 0.0
    x = xf
    fx = f(x)
    num = 1
    it = 0
    fv = fx
    fw = fx
    xm = 0.5 * (a + b)
    tol1 = seps * abs(xf) + tolx / 3.0
    tol2 = 2.0 * tol1
    while abs(xf - xm) > (tol2 - 0.5 * (b - a)):
        gs = 1
        if abs(e) > tol1:
            gs = 0
            r = (xf - w) * (fx - fv)
            q = (xf - v) * (fx - fw)
            p = (xf - v) * q - (xf - w) * r
            q = 2.0 * (q - r)
            if q > 0.0:
                p = -p
            q = abs(q)
            r = e
            e = d
            if abs(p) < abs(0.5 * q * r) and p > q * (a - xf) and p < q * (b - xf):
                d = p / q
                x = xf + d
                if (x - a) < tol2 or (b - x) < tol2:
                    si = _sign(xm - xf) + ((xm - xf) == 0)
                    d = tol1 * si
            else:
                gs = 1
        if gs:
            e = (a - xf) if xf >= xm else (b - xf)
            d = c * e
        si = _sign(d) + (d == 0)
        x = xf + si * max(abs(d), tol1)
        fu = f(x)
        num += 1
        it += 1
        if fu <= fx:
            if x >= xf:
                a = xf
            else:
                b = xf
            v, fv = w, fw
            w, fw = xf, fx
            xf, fx = x, fu
        else:
            if x < xf:
                a = x
            else:
                b = x
            if fu <= fw or w == xf:
                v, fv = w, fw
                w, fw = x, fu
            elif fu <= fv or v == xf or v == w:
                v, fv = x, fu
        xm = 0.5 * (a + b)
        tol1 = seps * abs(xf) + tolx / 3.0
        tol2 = 2.0 * tol1
        if num >= maxfun or it >= maxiter:
            break
    return xf, fx, num


def fdlibm_log(x: float) -> float:
    """Python transcription of the fdlibm log that aiy_math.h (aiy_log) uses, so that the KS
    restatement evaluates exactly the same function values as the C oracle and the kernels."""
    import struct
    ln2_hi, ln2_lo, two54 = 6.93147180369123816490e-01, 1.90821492927058770002e-10, 1.80143985094819840000e+16
    Lg1, Lg2, Lg3, Lg4 = 6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01, 2.222219843214978396e-01
    Lg5, Lg6, Lg7 = 1.818357216161805012e-01, 1.531383769920937332e-01, 1.479819860511658591e-01
    u = struct.unpack("<Q", struct.pack("<d", x))[0]
    hx = u >> 32
    if hx >= 0x80000000:
        hx -= 1 << 32
    lx = u & 0xFFFFFFFF
    k = 0
    if hx < 0x00100000:
        if ((hx & 0x7FFFFFFF) | lx) == 0:
            return -math.inf
        if hx < 0:
            return math.nan
        k -= 54
        x *= two54
        u = struct.unpack("<Q", struct.pack("<d", x))[0]
        hx = u >> 32
    if hx >= 0x7FF00000:
        return x + x
    k += (hx >> 20) - 1023
    hx &= 0x000FFFFF
    i = (hx + 0x95F64) & 0x100000
    u = struct.unpack("<Q", struct.pack("<d", x))[0]
    u = ((hx | (i ^ 0x3FF00000)) << 32) | (u & 0xFFFFFFFF)
    x = struct.unpack("<d", struct.pack("<Q", u))[0]
    k += i >> 20
    f = x - 1.0
    if (0x000FFFFF & (2 + hx)) < 3:
        if f == 0.0:
            if k == 0:
                return 0.0
            dk = float(k)
            return dk * ln2_hi + dk * ln2_lo
        R = f * f * (0.5 - 0.33333333333333333 * f)
        if k == 0:
            return f - R
        dk = float(k)
        return dk * ln2_hi - ((R - dk * ln2_lo) - f)
    s = f / (2.0 + f)
    dk = float(k)
    z = s * s
    i = hx - 0x6147A
    w = z * z
    j = 0x6B851 - hx
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6))
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)))
    i |= j
    R = t2 + t1
    if i > 0:
        hfsq = 0.5 * f * f
        if k == 0:
            return f - (hfsq - s * (hfsq + R))
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f)
    if k == 0:
        return f - s * (f - R)
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f)


def ks_setup(k_size=100, K_size=4, K_min=30.0, K_max=50.0):
    """Krusell_Smith_VFI.m:5-55, :97-99 (grids, 4x4 P, initial value, B)."""
    p = dict(beta=0.99, alpha=0.36, delta=0.025, k_min=0.0001, k_max=1000.0, ug=0.04, ub=0.10,
             mu=0.0, z_grid=(1.01, 0.99), eps_grid=(1.0, 0.0))
    p["l_bar"] = 1 / (1 - p["ub"])
    x = matlab_linspace01(k_size)
    k_grid = (x ** 7) * (p["k_max"] - p["k_min"]) + p["k_min"]   # :16 (x.^7)
    k_grid[0], k_grid[-1] = p["k_min"], p["k_max"]               # :17
    K_grid = K_min + (K_max - K_min) * matlab_linspace01(K_size)
    pgg = 1 - 1 / 8; pbb = 1 - 1 / 8; pgb = 1 - pgg; pbg = 1 - pbb
    p00_gg = 1 - 1 / 1.5; p00_bb = 1 - 1 / 2.5
    p00_gb = 1.25 * p00_bb; p00_bg = 0.75 * p00_gg
    p01_gg = 1 - p00_gg; p01_bb = 1 - p00_bb; p01_gb = 1 - p00_gb; p01_bg = 1 - p00_bg
    ug, ub = p["ug"], p["ub"]
    p10_gg = (ug - ug * p00_gg) / (1 - ug); p10_bb = (ub - ub * p00_bb) / (1 - ub)
    p10_gb = (ub - ug * p00_gb) / (1 - ug); p10_bg = (ug - ub * p00_bg) / (1 - ub)
    p11_gg = 1 - p10_gg; p11_bb = 1 - p10_bb; p11_gb = 1 - p10_gb; p11_bg = 1 - p10_bg
    P = np.array([[pgg * p11_gg, pgb * p11_gb, pgg * p10_gg, pgb * p10_gb],
                  [pbg * p11_bg, pbb * p11_bb, pbg * p10_bg, pbb * p10_bb],
                  [pgg * p01_gg, pgb * p01_gb, pgg * p00_gg, pgb * p00_gb],
                  [pbg * p01_bg, pbb * p01_bb, pbg * p00_bg, pbb * p00_bb]])   # :47-55
    k_opt0 = 0.9 * np.repeat(np.repeat(k_grid[:, None, None], K_size, 1), 4, 2)  # :97
    V0 = np.log(0.1 / 0.9 * k_opt0) / (1 - p["beta"])                           # :98
    B = np.array([0.0, 1.0, 0.0, 1.0])
    return p, k_grid, K_grid, P, V0, B


def ks_bellman(p, k_grid, K_grid, V, dV, B, P, kp, k_i, K_i, s_i):
    """bellman_value, Krusell_Smith_VFI.m:329-364 (V, dV indexed [k, K, s])."""
    zg = p["z_grid"]
    z = zg[1] if (s_i + 1) <= 2 else zg[0]
    K, k = K_grid[K_i], k_grid[k_i]
    if z == zg[0]:
        Kp = math.exp(B[0] + B[1] * math.log(max(K, 1e-8)))
    else:
        Kp = math.exp(B[2] + B[3] * math.log(max(K, 1e-8)))
    Kp = max(min(Kp, K_grid[-1]), K_grid[0])
    Kp_idx = int(np.argmin(np.abs(K_grid - Kp)))
    kq = max(min(kp, k_grid[-1]), k_grid[0])
    expec = 0.0
    for sn in range(4):
        expec = expec + P[s_i, sn] * pchip_eval(k_grid, V[:, Kp_idx, sn], dV[:, Kp_idx, sn], kq)
    L = p["l_bar"] * (1 - p["ug"] * float(z == zg[0]) - p["ub"] * float(z == zg[1]))
    a = p["alpha"]
    r_val = a * z * math.pow(K, a - 1) * math.pow(L, 1 - a)
    w_val = (1 - a) * z * math.pow(K, a) * math.pow(L, -a)
    eps = p["eps_grid"][0] if s_i % 2 == 0 else p["eps_grid"][1]
    c = (r_val + 1 - p["delta"]) * k + w_val * (eps * p["l_bar"]) - kp
    c = max(c, 1e-10)
    return fdlibm_log(c) + p["beta"] * expec


def ks_slopes(k_grid, V):
    dV = np.zeros_like(V)
    for Ki in range(V.shape[1]):
        for sn in range(V.shape[2]):
            dV[:, Ki, sn] = pchip_slopes(k_grid, V[:, Ki, sn])
    return dV


def ks_policy_improve(p, k_grid, K_grid, V, B, P):
    """Krusell_Smith_VFI.m:149-168."""
    nk, nK, nS = V.shape
    dV = ks_slopes(k_grid, V)
    k_opt = np.zeros_like(V)
    nfev = np.zeros(V.shape, np.int32)
    a = p["alpha"]
    for s_i in range(nS):
        zt = p["z_grid"][0] if s_i < 2 else p["z_grid"][1]
        eps = p["eps_grid"][0] if s_i % 2 == 0 else p["eps_grid"][1]
        for K_i in range(nK):
            K = K_grid[K_i]
            L = p["l_bar"] * (1 - p["ug"] * float(zt == p["z_grid"][0]) - p["ub"] * float(zt == p["z_grid"][1]))
            wt = (1 - a) * zt * math.pow(K, a) * math.pow(L, -a)
            rt = a * zt * math.pow(K, a - 1) * math.pow(L, 1 - a)
            for k_i in range(nk):
                res = (rt + 1 - p["delta"]) * k_grid[k_i] + wt * (eps * p["l_bar"] + (1 - eps) * p["mu"])
                kpmax = min(res, p["k_max"])
                f = lambda x: -ks_bellman(p, k_grid, K_grid, V, dV, B, P, x, k_i, K_i, s_i)
                xf, _, nf = fminbnd(f, p["k_min"], kpmax)
                k_opt[k_i, K_i, s_i] = xf
                nfev[k_i, K_i, s_i] = nf
    return k_opt, nfev


def ks_howard(p, k_grid, K_grid, V, k_opt, B, P, steps):
    """Krusell_Smith_VFI.m:172-192 (Jacobi sweeps, slopes rebuilt after each)."""
    V = np.array(V, dtype=np.float64)
    nk, nK, nS = V.shape
    for _ in range(steps):
        dV = ks_slopes(k_grid, V)
        Vn = np.empty_like(V)
        for s_i in range(nS):
            for K_i in range(nK):
                for k_i in range(nk):
                    Vn[k_i, K_i, s_i] = ks_bellman(p, k_grid, K_grid, V, dV, B, P,
                                                   k_opt[k_i, K_i, s_i], k_i, K_i, s_i)
        V = Vn
    return V


# ----------------------------------------------------------------------------------------
# A8  Krusell-Smith EGM (Krusell_Smith_EGM.m:101-112, :129-209)
# ----------------------------------------------------------------------------------------


def ks_egm_pairs(p, K_grid, B):
    """Per (s_i, K_i) scalars of the EGM step, in the script's operation order (libm
    pow/exp/log via math.*).  s_grid = [Z(:), Eps(:)] of meshgrid(z_grid, eps_grid)
    (:18-19): s = (z1,e1), (z1,e2), (z2,e1), (z2,e2).  Returns a list indexed s_i*nK + K_i of
    dicts {kd: [K''_idx per s_j], Rn: [(1 + r_next) - delta], Wn: [w_next*eps_next*l_bar],
    R: (1 + r) - delta, We: w*eps*l_bar}."""
    zg, eg = p["z_grid"], p["eps_grid"]
    a, dl, lb = p["alpha"], p["delta"], p["l_bar"]
    s_grid = [(zg[0], eg[0]), (zg[0], eg[1]), (zg[1], eg[0]), (zg[1], eg[1])]

    def labour(z):  # L = l_bar*(1 - ug*(z==z_grid(1)) - ub*(z==z_grid(2)))  (:108, :149)
        return lb * (1 - p["ug"] * float(z == zg[0]) - p["ub"] * float(z == zg[1]))

    def alm(z, K):  # :140-145 / :164-169 (no clamp, no floor in the EGM script)
        if z == zg[0]:
            return math.exp(B[0] + B[1] * math.log(K))
        return math.exp(B[2] + B[3] * math.log(K))

    out = []
    nK = len(K_grid)
    for s_i in range(4):
        z, e = s_grid[s_i]
        for K_i in range(nK):
            K = float(K_grid[K_i])
            L = labour(z)
            r = a * z * math.pow(K, a - 1) * math.pow(L, 1 - a)          # r_table  (:110)
            w = (1 - a) * z * math.pow(K, a) * math.pow(L, -a)          # w_table  (:109)
            Kp = alm(z, K)
            kd, Rn, Wn = [], [], []
            for s_j in range(4):
                zn, en = s_grid[s_j]
                Kdp = alm(zn, Kp)
                kd.append(int(np.argmin(np.abs(np.asarray(K_grid) - Kdp))))  # first on ties
                Ln = labour(zn)
                rn = a * zn * math.pow(Kdp, a - 1) * math.pow(Ln, 1 - a)   # :174
                wn = (1 - a) * zn * math.pow(Kdp, a) * math.pow(Ln, -a)    # :175
                Rn.append((1 + rn) - dl)
                Wn.append((wn * en) * lb)
            out.append(dict(kd=kd, Rn=Rn, Wn=Wn, R=(1 + r) - dl, We=(w * e) * lb))
    return out


def _pchip_slopes_n(x, y):
    """pchip.m slopes for n >= 2 (n == 2: the secant, i.e. linear interpolation)."""
    if len(x) == 2:
        s = (y[1] - y[0]) / (x[1] - x[0])
        return np.array([s, s])
    return pchip_slopes(x, y)


def ks_egm_sweep(p, k_grid, K_grid, B, P, k_opt, pairs=None, src=None):
    """One Gauss-Seidel sweep of Krusell_Smith_EGM.m:133-200: k_opt(:,K_i,s_i) is overwritten
    as soon as it is computed and read by later (s, K) pairs.  k_opt is [k, K, s] (modified in
    place and returned).  src (F1, not the reference): read the next-period policy from this
    array instead — src = a copy of the sweep's input gives the Jacobi variant."""
    nk, nK, _ = k_opt.shape
    src = k_opt if src is None else src
    pairs = pairs or ks_egm_pairs(p, K_grid, B)
    k_min, k_max, beta = p["k_min"], p["k_max"], p["beta"]
    for s_i in range(4):
        for K_i in range(nK):
            q = pairs[s_i * nK + K_i]
            cols = [src[:, q["kd"][s_j], s_j].copy() for s_j in range(4)]
            slopes = [pchip_slopes(k_grid, c) for c in cols]
            kc = np.empty(nk)
            for kp_i in range(nk):
                kp = float(k_grid[kp_i])
                em = 0.0
                for s_j in range(4):
                    kpn = pchip_eval(k_grid, cols[s_j], slopes[s_j], kp)        # :179
                    c_next = (q["Rn"][s_j] * kp + q["Wn"][s_j]) - kpn            # :178, :180
                    c_next = c_next if c_next > 1e-8 else 1e-8                   # :181 (NaN → 1e-8)
                    em = em + (P[s_i, s_j] * q["Rn"][s_j]) / c_next              # :183
                c = 1 / (beta * em)                                              # :187
                kc[kp_i] = ((c + kp) - q["We"]) / q["R"]                         # :188
            order = np.argsort(kc, kind="stable")                                 # :193 (NaN last)
            xs, ys = kc[order], k_grid[order]
            valid = (xs >= k_min) & (xs <= k_max)                                 # :195
            xs, ys = xs[valid], ys[valid]
            if len(xs) < 2:
                raise ValueError("fewer than 2 valid EGM points (griddedInterpolant would fail)")
            d = _pchip_slopes_n(xs, ys)
            new = np.empty(nk)
            for t in range(nk):                                                   # :196-197
                kq = float(k_grid[t])
                if kq < xs[0]:
                    v = ys[0]                                                     # 'nearest'
                elif kq > xs[-1]:
                    v = ys[-1]
                else:
                    v = pchip_eval(xs, ys, d, kq)
                v = k_max if not (v <= k_max) else v                              # min(v, k_max)
                new[t] = k_min if not (v >= k_min) else v                         # max(., k_min)
            k_opt[:, K_i, s_i] = new                                              # :199
    return k_opt


def ks_egm_solve(p, k_grid, K_grid, B, P, k_opt, tol=1e-6, max_iter=10000, jacobi=False):
    """Krusell_Smith_EGM.m:130-209 for one B: sweeps until max|Δk_opt| < tol (jacobi=True:
    the F1 Jacobi variant, every pair reads the previous sweep's k_opt — not the reference)."""
    k_opt = np.array(k_opt, dtype=np.float64, copy=True)
    pairs = ks_egm_pairs(p, K_grid, B)
    diff = float("nan")
    it = 0
    for it in range(1, max_iter + 1):
        old = k_opt.copy()
        ks_egm_sweep(p, k_grid, K_grid, B, P, k_opt, pairs, src=old if jacobi else None)
        dd = np.abs(k_opt - old)
        diff = float(np.nanmax(dd)) if not np.all(np.isnan(dd)) else float("nan")
        if diff < tol:
            break
    return dict(k_opt=k_opt, iters=it, diff=diff)


# ----------------------------------------------------------------------------------------
# F3  Krusell-Smith shock panel (Krusell_Smith_VFI.m:57-94) and F2 panel simulation
#     (:206-248).  Vectorised over agents; every operation is an IEEE basic operation or a
#     comparison, so the results are exact restatements (no libm).
# ----------------------------------------------------------------------------------------


def ks_eps_probs(p):
    """The idiosyncratic transition probabilities of Krusell_Smith_VFI.m:24-45, returned as
    thr[cur_z, prev_z, prev_e] = Peps(prev_e, 1) of :78-92 (z: 0 good / 1 bad after the
    `zi_shock - 1` of :68; e: 0 employed / 1 unemployed = epsi_shock - 1)."""
    pgg = 1 - 1 / 8; pbb = 1 - 1 / 8
    p00_gg = 1 - 1 / 1.5; p00_bb = 1 - 1 / 2.5
    p00_gb = 1.25 * p00_bb; p00_bg = 0.75 * p00_gg
    p01_gg = 1 - p00_gg; p01_bb = 1 - p00_bb; p01_gb = 1 - p00_gb; p01_bg = 1 - p00_bg
    ug, ub = p["ug"], p["ub"]
    p10_gg = (ug - ug * p00_gg) / (1 - ug); p10_bb = (ub - ub * p00_bb) / (1 - ub)
    p10_gb = (ub - ug * p00_gb) / (1 - ug); p10_bg = (ug - ub * p00_bg) / (1 - ub)
    p11_gg = 1 - p10_gg; p11_bb = 1 - p10_bb; p11_gb = 1 - p10_gb; p11_bg = 1 - p10_bg
    thr = np.zeros((2, 2, 2))
    # (cur, prev) -> matrix: (0,0) gg, (0,1) bg, (1,0) gb, else bb  (:78-86)
    for cz, pz, (p11, p01) in ((0, 0, (p11_gg, p01_gg)), (0, 1, (p11_bg, p01_bg)),
                               (1, 0, (p11_gb, p01_gb)), (1, 1, (p11_bb, p01_bb))):
        thr[cz, pz, 0] = p11   # prev_eps == 1 -> Peps(1,1)  (:88-89)
        thr[cz, pz, 1] = p01   # else          -> Peps(2,1)  (:90-91)
    return dict(pgg=pgg, pbb=pbb, thr=thr)


def ks_shock_draws(T, population):
    """Number of `rand` draws :57-94 consumes: T-1 aggregate, `population` initial, then
    (T-1)*population idiosyncratic (t outer, i inner)."""
    return (T - 1) + population + (T - 1) * population


def ks_shocks(p, T, population, U):
    """Krusell_Smith_VFI.m:59-94.  U = the MATLAB rand stream (ks_shock_draws(T, pop) values).
    Returns zi (T,) int8 in {0 good, 1 bad} (= zi_shock after :68) and e (T, population) int8 in
    {0, 1} (= epsi_shock - 1: 0 employed, 1 unemployed)."""
    pr = ks_eps_probs(p)
    U = np.asarray(U, dtype=np.float64)
    zi = np.zeros(T, np.int8)
    z = 1                                                     # :60 zi_shock(1) = 1
    for t in range(1, T):                                     # :61-67
        u = U[t - 1]
        z = 1 + int(u > (pr["pgg"] if z == 1 else pr["pbb"]))
        zi[t] = z - 1
    pos = T - 1
    e = np.zeros((T, population), np.int8)
    e[0] = (U[pos:pos + population] > p["ug"]).astype(np.int8)   # :71 ((rand>ug)+1) - 1
    pos += population
    thr = pr["thr"]
    for t in range(1, T):                                     # :72-94
        th = thr[zi[t], zi[t - 1]][e[t - 1]]
        e[t] = (U[pos:pos + population] > th).astype(np.int8)
        pos += population
    return zi, e


def ks_panel_blocks(population, block=256, max_blocks=1024):
    """Reduction geometry of mean(k_population) shared with the HIP kernel (MATLAB's own sum
    order is unpinned): G blocks of `block` lanes; lane g of the grid sums agents g, g + G*block,
    ... in order; each block folds its lanes pairwise (h = block/2 ... 1); the G block sums,
    zero-padded to the next power of two, are folded pairwise the same way and the total is
    divided by the population."""
    return max(1, min(max_blocks, -(-population // block)))


def ks_mean_blocked(x, G, block=256):
    n = x.size
    L = G * block
    lanes = np.zeros(L)
    for m in range(0, n, L):
        seg = x[m:m + L]
        lanes[:seg.size] = lanes[:seg.size] + seg
    s = lanes.reshape(G, block)
    h = block // 2
    while h >= 1:
        s = s.copy()
        s[:, :h] = s[:, :h] + s[:, h:2 * h]
        h //= 2
    Gp = 1
    while Gp < G:
        Gp *= 2
    q = np.zeros(Gp)
    q[:G] = s[:, 0]
    h = Gp // 2
    while h >= 1:
        q = q.copy()
        q[:h] = q[:h] + q[h:2 * h]
        h //= 2
    return q[0] / n


def _bilin_seg(x, q):
    i = np.searchsorted(x, q, side="right") - 1
    return np.clip(i, 0, x.size - 2)


def ks_panel_simulate(k_grid, K_grid, k_opt, zi, e, k_pop, block=256, max_blocks=1024):
    """Krusell_Smith_VFI.m:206-248: K_ts(1) = mean(k_population); per period t the agents in
    state s = (z_t, eps_t,i) (s_grid order (g,e),(g,u),(b,e),(b,u), :19-20) move to
    griddedInterpolant({k_grid, K_grid}, k_opt(:,:,s)) at (k, K_ts(t)) — bilinear, linear
    extrapolation from the edge cells: segment = largest i with x_i <= q clamped to
    [0, n-2]; f0 = f(ik,iK) + tk*(f(ik+1,iK) - f(ik,iK)), f1 likewise at iK+1,
    value = f0 + tK*(f1 - f0).  k_opt indexed [k, K, s].  Returns (K_ts, k_pop)."""
    k_pop = np.array(k_pop, dtype=np.float64, copy=True)
    T = zi.size
    n = k_pop.size
    G = ks_panel_blocks(n, block, max_blocks)
    K_ts = np.zeros(T)
    K_ts[0] = ks_mean_blocked(k_pop, G, block)                     # :208
    for t in range(T - 1):                                         # :222
        K = K_ts[t]
        iK = int(_bilin_seg(K_grid, np.array([K]))[0])
        tK = (K - K_grid[iK]) / (K_grid[iK + 1] - K_grid[iK])
        s = 2 * int(zi[t]) + e[t].astype(np.int64)                 # :227-232
        ik = _bilin_seg(k_grid, k_pop)
        tk = (k_pop - k_grid[ik]) / (k_grid[ik + 1] - k_grid[ik])
        f00 = k_opt[ik, iK, s]; f10 = k_opt[ik + 1, iK, s]
        f01 = k_opt[ik, iK + 1, s]; f11 = k_opt[ik + 1, iK + 1, s]
        f0 = f00 + tk * (f10 - f00)
        f1 = f01 + tk * (f11 - f01)
        k_pop = f0 + tK * (f1 - f0)                                # :241-246
        K_ts[t + 1] = ks_mean_blocked(k_pop, G, block)             # :247
    return K_ts, k_pop


def ks_alm_regress(K_ts, zi, T_discard=100):
    """Krusell_Smith_VFI.m:252-285: OLS of log K(t+1) on [1, log K(t)] per aggregate state over
    t = T_discard..T-1 (MATLAB 1-based t).  Returns (B_new (4,), R2_g, R2_b).  MATLAB's `\\`
    is a QR solve; numpy's lstsq (SVD) agrees to rounding (ulp-level; not bit-pinned)."""
    T = K_ts.size
    ts = np.arange(T_discard - 1, T - 1)                           # 0-based t
    B = np.zeros(4)
    R2 = [0.0, 0.0]
    for g, zsel in ((0, 0), (1, 1)):
        sel = ts[zi[ts] == zsel]
        if sel.size == 0:
            continue
        X = np.stack([np.ones(sel.size), np.log(K_ts[sel])], 1)
        Y = np.log(K_ts[sel + 1])
        b = np.linalg.lstsq(X, Y, rcond=None)[0]
        B[2 * g:2 * g + 2] = b
        res = Y - X @ b
        R2[g] = 1 - np.sum(res ** 2) / np.sum((Y - Y.mean()) ** 2)
    return B, R2[0], R2[1]
