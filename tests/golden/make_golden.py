"""Generate the golden fixtures under tests/golden/ from the numpy restatement
(oracle/np_oracle.py).  The reference is MATLAB and cannot run in this image, and it ships no
fixtures, so these vectors pin the C oracle and the HIP kernels to ONE literal restatement of
the cited MATLAB lines; parity against MATLAB itself is unpinned.

Run:  python tests/golden/make_golden.py        (≈2 minutes on one core)
"""
from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
from oracle import np_oracle as no  # noqa: E402


def save(name, **arrs):
    path = HERE / f"{name}.npz"
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrs.items()})
    print(f"  wrote {path.name} ({path.stat().st_size/1024:.1f} KiB)")


def main():
    t0 = time.time()
    # ---------------------------------------------------------------- RNG pin
    # MATLAB documentation, fresh session: rand(3) = [0.8147 0.9134 0.2785; 0.9058 0.6324
    # 0.5469; 0.1270 0.0975 0.9575] (column-major stream below, 4 decimals).
    save("rng_mt5489", first10=no.matlab_rand_stream(10),
         matlab_doc_4dp=np.array([0.8147, 0.9058, 0.1270, 0.9134, 0.6324, 0.0975, 0.2785,
                                  0.5469, 0.9575]))

    # ---------------------------------------------------------------- A1/A2 defaults
    cal = no.calib_aiyagari()
    P, s, a = cal["P"], cal["s"], cal["a_grid"]
    r = 0.04
    w = no.wage(r, cal["alpha"], cal["delta"])
    warm = no.vfi_solve(np.zeros((7, 400)), a, s, P, r, w, 0.96, 5.0, 1e-5, 20)
    v20 = warm["v_new"]
    v21, idx21, pk21, pc21 = no.vfi_sweep(v20, a, s, P, r, w, 0.96, 5.0)
    full = no.vfi_solve(np.zeros((7, 400)), a, s, P, r, w, 0.96, 5.0, 1e-5, 1000)
    save("a1_vfi_defaults", P=P, s=s, a_grid=a, r=r, w=w, beta=0.96, sigma=5.0,
         labor=cal["labor"], v20=v20, v21=v21, idx21=idx21, policy_k21=pk21,
         policy_c21=pc21, solve_iters=full["iters"], solve_v_new=full["v_new"],
         solve_v_old=full["v_old"], solve_idx=full["idx"])
    print(f"  A1 done {time.time()-t0:.1f}s (iters {full['iters']})")

    # ---------------------------------------------------------------- A9 + A11 GE trace
    H = no.ge_bisection_vfi(cal)
    U = no.matlab_rand_stream(2)
    z1 = int(np.ceil(7 * U[0])) - 1
    k1 = a[int(np.ceil(400 * U[1])) - 1]
    Ks0, path0, zpath0 = no.sim_capital(full["policy_k"], a, P, z1, k1,
                                        no.matlab_rand_stream(2 + 9999)[2:])
    save("a11_ge_vfi_defaults", r_history=H["r"], k_supply=H["k_supply"],
         k_demand=H["k_demand"], iters=H["iters"], r_final=H["r_final"], z1=z1, k1=k1,
         Ks0=Ks0, sim_k0=path0, sim_z0=zpath0)
    print(f"  GE done {time.time()-t0:.1f}s r_final={H['r_final']:.10f}")

    # ---------------------------------------------------------------- A3 labour VFI Na=100
    calL = no.calib_aiyagari(Na=100, rho=0.6, sigma_e=0.2)
    L = 0.01 + (1.5 - 0.01) * no.matlab_linspace01(10)
    rL = no.labor_vfi_solve(np.zeros((7, 100)), calL["a_grid"], calL["s"], calL["P"], r, w,
                            0.96, 5.0, L, 1.0, 2.0, 1e-5, 1000)
    save("a3_labor_vfi_na100", P=calL["P"], s=calL["s"], a_grid=calL["a_grid"], L=L, r=r, w=w,
         beta=0.96, sigma=5.0, psi=1.0, eta=2.0, iters=rL["iters"], v_new=rL["v_new"],
         v_old=rL["v_old"], policy_k=rL["policy_k"], policy_l=rL["policy_l"],
         policy_c=rL["policy_c"], lin=rL["lin"])
    print(f"  A3 done {time.time()-t0:.1f}s (iters {rL['iters']})")

    # ---------------------------------------------------------------- A4/A5 EGM defaults
    pc0 = np.tile(((1 + r) * a + w * np.mean(s))[:, None], (1, 7))       # Aiyagari_EGM.m:64
    E = no.egm_solve(pc0, a, s, P, r, w, 0.96, 5.0, cal["amin"])
    E1c, E1k, E1d = no.egm_step(pc0, a, s, P, r, w, 0.96, 5.0, cal["amin"])
    save("a4_egm_defaults", P=P, s=s, a_grid=a, r=r, w=w, amin=cal["amin"], policy_c0=pc0,
         step1_c=E1c, step1_k=E1k, step1_dist=E1d, iters=E["iters"], policy_c=E["policy_c"],
         policy_k=E["policy_k"], dist=E["dist"])
    calE = no.calib_aiyagari(rho=0.6, sigma_e=0.2)
    aE, sE = calE["a_grid"], calE["s"]
    pc0L = np.tile(((1 + r) * aE + w * np.mean(sE))[:, None], (1, 7))
    EL = no.labor_egm_solve(pc0L, aE, sE, calE["P"], r, w, 0.96, 5.0, 1.0, 1.0, calE["amin"])
    save("a5_labor_egm_defaults", P=calE["P"], s=sE, a_grid=aE, r=r, w=w, amin=calE["amin"],
         phi=1.0, theta=1.0, policy_c0=pc0L, iters=EL["iters"], policy_c=EL["policy_c"],
         policy_k=EL["policy_k"], policy_l=EL["policy_l"], dist=EL["dist"])
    print(f"  A4/A5 done {time.time()-t0:.1f}s (iters {E['iters']}, {EL['iters']})")

    # ---------------------------------------------------------------- A10 histogram push
    lam0 = np.full((7, 400), 1.0 / 2800)
    lam1 = no.dist_update_ongrid(lam0, full["idx"], P)
    lamL = no.dist_update_lottery(lam0, E["policy_k"].T, a, P)
    save("a10_dist_defaults", lam0=lam0, idx=full["idx"], lam1=lam1, kp_egm=E["policy_k"].T,
         lam1_lottery=lamL)

    # ---------------------------------------------------------------- A6/A7 KS
    p, kg, Kg, Pk, V0, B = no.ks_setup()
    kopt, nfev = no.ks_policy_improve(p, kg, Kg, V0, B, Pk)
    V2 = no.ks_howard(p, kg, Kg, V0, kopt, B, Pk, 2)
    save("ks_defaults", k_grid=kg, K_grid=Kg, P=Pk, V0=V0, B=B, k_opt=kopt, nfev=nfev,
         V_howard2=V2, beta=p["beta"], alpha=p["alpha"], delta=p["delta"], k_min=p["k_min"],
         k_max=p["k_max"], ug=p["ug"], ub=p["ub"], l_bar=p["l_bar"], mu=p["mu"])
    print(f"  KS done {time.time()-t0:.1f}s")
    make_ks_egm()


def make_ks_egm():
    """A8: Krusell_Smith_EGM.m:129-209 at the reference defaults (k=100, K=4, S=4), from the
    script's initial k_opt = 0.9*k_grid (:96): 1 and 3 Gauss-Seidel sweeps, and the full solve
    to tol_egm = 1e-6 (numpy restatement, ~75 s)."""
    t0 = time.time()
    p, kg, Kg, Pk, _, B = no.ks_setup()
    k0 = 0.9 * np.repeat(np.repeat(kg[:, None, None], len(Kg), 1), 4, 2)
    s1 = no.ks_egm_solve(p, kg, Kg, B, Pk, k0, max_iter=1)
    s3 = no.ks_egm_solve(p, kg, Kg, B, Pk, k0, max_iter=3)
    full = no.ks_egm_solve(p, kg, Kg, B, Pk, k0, tol=1e-6, max_iter=10000)
    save("ks_egm_defaults", k_grid=kg, K_grid=Kg, P=Pk, B=B, k_opt0=k0, k_opt1=s1["k_opt"],
         k_opt3=s3["k_opt"], diff3=s3["diff"], k_opt_final=full["k_opt"], iters=full["iters"],
         diff_final=full["diff"], beta=p["beta"], alpha=p["alpha"], delta=p["delta"],
         k_min=p["k_min"], k_max=p["k_max"], ug=p["ug"], ub=p["ub"], l_bar=p["l_bar"],
         mu=p["mu"])
    print(f"  KS EGM done {time.time()-t0:.1f}s ({full['iters']} sweeps)")


def make_ks_panel():
    """F3/F2: Krusell_Smith_VFI.m:57-94 shock panel and :206-248 capital simulation at a
    reduced panel (T = 120 periods, 700 agents: three reduction blocks, the last one ragged),
    MATLAB's fresh-session rand stream, the policy k_opt of ks_defaults (one improvement) and
    the script's initial population k = K_grid(1) (:101)."""
    p, kg, Kg, Pk, _, B = no.ks_setup()
    g = np.load(Path(__file__).resolve().parent / "ks_defaults.npz")
    T, pop = 120, 700
    U = no.matlab_rand_stream(no.ks_shock_draws(T, pop))
    zi, e = no.ks_shocks(p, T, pop, U)
    k0 = np.full(pop, Kg[0])
    K_ts, k_fin = no.ks_panel_simulate(kg, Kg, g["k_opt"], zi, e, k0)
    save("ks_panel_small", T=T, population=pop, zi=zi, eps=e, k_opt=g["k_opt"], k_grid=kg,
         K_grid=Kg, K_ts=K_ts, k_final=k_fin, ug=p["ug"], ub=p["ub"])
    print("  KS panel done")


if __name__ == "__main__":
    import sys as _sys
    if len(_sys.argv) > 1 and _sys.argv[1] == "ks_egm":
        make_ks_egm()
    elif len(_sys.argv) > 1 and _sys.argv[1] == "ks_panel":
        make_ks_panel()
    else:
        main()
