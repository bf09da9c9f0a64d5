"""Workloads for the round-5 PMC passes (tools/pmc.sh with PMC_CMD set to this script and
BENCH_ARGS = one workload name), one workload per process so every pass set sees only the
launches of the kernel it is about (VERDICT r4 "do this" 1):

  batch     bell_tree_kernel  — config-4 batched launch: 8 rates x 25 sweeps from v = 0 at
                                Na = 20,000 (bench `batch_config4_share`); take 25
  labor400  bell_wide_kernel  — labour VFI at Na = 400 (Nl = 10), 5 warm-up + 10 sweeps in one
                                C call (bench `labor_vfi.Na400`): skip 5 take 10
  labor20k  bell_tree_kernel  — labour VFI at Na = 20,000: 5 warm-up + 5 sweeps (bench
                                `labor_vfi.Na20000`): skip 5 take 5
  a1_400    bell_wide_kernel  — A1 solve at Na = 400 from v = 0 (the GE loop's solves): all
  ks        ks_howard_slopes_kernel — one rank's improvement + 10 fused Howard sweeps at the KS
                                scaling size (k = 32,768, K = 64, S = 4; bench `ks_sharded`)
  egm       egm_chain_kernel  — A4 then A5 solve loops at Na = 20,000, 200 chained steps each:
                                take 200 / skip 200 take 200
  dist      dist_push_kernel  — 64 pushes on the r = 0.04 policy at Na = 20,000 (bench `dist`)
  sim       sim_par_seg_kernel — (round 6) 20 capital-supply chains of T = 10,000 on the
                                Na = 400 policy at r = 0.04 (the GE loop's chain), K_s only
(round 6: the same workloads, tools/exp/r06_pmc.sh; `ks` now times ks_howard_slopes_xcd_kernel)
"""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

pkg = bench.load_pkg()
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
which = sys.argv[1] if len(sys.argv) > 1 else "batch"
r = 0.04


def a1_setup(Na):
    cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    return cal, w, t(cal["a_grid"]), t(cal["s"]), t(cal["P"])


if which == "batch":
    cal, w, a_t, s_t, P_t = a1_setup(20000)
    N, Na, C = cal["N"], 20000, 8
    rs = list(np.linspace(-0.03, 0.035, C))
    ws_b = [pkg.calibration.wage(x, cal["alpha"], cal["delta"]) for x in rs]
    bws = pkg.Workspace(N, Na)
    bv = [torch.zeros((C, N, Na), dtype=torch.float64, device=dev) for _ in range(2)]
    bidx = torch.zeros((C, N, Na), dtype=torch.int32, device=dev)
    bpk, bpc = torch.zeros_like(bv[0]), torch.zeros_like(bv[0])
    pkg.vfi.solve_batch_dev(bws, rs, ws_b, bv[0], bv[1], a_t, s_t, P_t, cal["beta"], cal["sigma"],
                            0.0, 25, bidx, bpk, bpc)
elif which in ("labor400", "labor20k"):
    Na = 400 if which == "labor400" else 20000
    steps = 10 if Na == 400 else 5
    lc = pkg.calibration.aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    L = t(0.01 + (1.5 - 0.01) * pkg.calibration.linspace01(10))
    ws = pkg.Workspace(lc["N"], Na, 10)
    v = [torch.zeros((lc["N"], Na), dtype=torch.float64, device=dev) for _ in range(2)]
    lin = torch.zeros((lc["N"], Na), dtype=torch.int32, device=dev)
    pk, pl, pc = (torch.zeros_like(v[0]) for _ in range(3))
    lw = pkg.calibration.wage(r, lc["alpha"], lc["delta"])
    a_t, s_t, P_t = t(lc["a_grid"]), t(lc["s"]), t(lc["P"])
    cur = 0
    for q in range(5 + steps):  # bench labor_leg's sweeps: 5 warm-up, then the timed ones
        ws.labor_vfi_sweep(v[cur], a_t, s_t, P_t, L, r, lw, lc["beta"], lc["sigma"], 1.0, 2.0,
                           v[1 - cur], lin, pk, pl, pc, hint=None if q == 0 else lin)
        cur = 1 - cur
elif which == "a1_400":
    cal, w, a_t, s_t, P_t = a1_setup(400)
    ws = pkg.Workspace(cal["N"], 400)
    va = torch.zeros((cal["N"], 400), dtype=torch.float64, device=dev)
    vb = torch.zeros_like(va)
    idx = torch.zeros((cal["N"], 400), dtype=torch.int32, device=dev)
    ws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5, 1000, idx)
elif which == "ks":
    kd = pkg.ks_dist
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=32768, K_size=64)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), 0, 64, 0, 4)
    V = t(V0.transpose(2, 1, 0))
    V2 = V.clone()
    ko = torch.ones_like(V)
    hs = kd.HowardSweeps(sh, 64, 0, 1, V)
    hs.improve(V, ko)
    hs.run(V, V2, ko, 10)
    torch.cuda.synchronize()
    hs.close()
    sh.close()
elif which == "egm":
    cal, w, a_t, s_t, P_t = a1_setup(20000)
    a = cal["a_grid"]
    pc0 = np.tile(((1 + r) * a + w * np.mean(cal["s"]))[None, :], (cal["N"], 1))
    for labor in (False, True):
        ws = pkg.Workspace(cal["N"], 20000)
        c = t(pc0)
        pk = torch.zeros_like(c)
        pl = torch.zeros_like(c) if labor else None
        pkg.egm_solve_dev(ws, c, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], cal["amin"], 0.0,
                          200, pk, labor=labor, phi=1.0, theta=1.0, policy_l=pl)
        torch.cuda.synchronize()
elif which == "dist":
    cal, w, a_t, s_t, P_t = a1_setup(20000)
    N, Na = cal["N"], 20000
    vws = pkg.Workspace(N, Na)
    va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
    vb = torch.zeros_like(va)
    idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    vws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5, 1000, idx)
    lam0 = torch.full((N, Na), 1.0 / (N * Na), dtype=torch.float64, device=dev)
    out = torch.empty_like(lam0)
    pkg.dist_stationary_dev(pkg.Workspace(N, Na), lam0, a_t, P_t, out, policy_idx=idx, tol=0.0,
                            max_iter=64)
elif which == "sim":
    cal, w, a_t, s_t, P_t = a1_setup(400)
    N, Na = cal["N"], 400
    vws = pkg.Workspace(N, Na)
    va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
    vb = torch.zeros_like(va)
    idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    pk = torch.zeros_like(va)
    vws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5, 1000, idx,
                  policy_k=pk)
    U = t(np.random.default_rng(0).random(9999))
    ks = torch.zeros(1, dtype=torch.float64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    for _ in range(20):
        pkg.sim_capital_dev(vws, pk, a_t, P_t, 3, float(cal["a_grid"][200]), U, ks, st)
else:
    raise SystemExit(f"unknown workload {which!r}")
torch.cuda.synchronize()
print(f"pmc workload {which} done")
