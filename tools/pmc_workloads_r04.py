"""Workloads for the round-4 PMC passes (tools/pmc.sh with PMC_CMD set to this script): the
kernels the bench legs actually time (VERDICT r3 "do this" 3).

  1. egm_chain_kernel  — aiy_egm_solve_dev at Na = 20,000 (Rouwenhorst Nz = 7, r = 0.04), 200
                         steps at tol = 0: one chained launch per step (bench `egm.Na20000`)
  2. egm_chain_kernel  — the labour EGM solve loop, same size (bench `labor_egm.Na20000`); it
                         runs after (1), so its launches are the second 200
  3. ks_howard_slopes_kernel — one rank's Howard sweeps at the KS scaling size (k = 32,768,
                         K = 64, S = 4): slopes once, then 10 fused sweeps (bench `ks_sharded`)
  4. dist_push_kernel  — 64 pushes on the r = 0.04 policy at Na = 20,000 (bench `dist`)
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
t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
cal = pkg.calibration.aiyagari(Na=20000, shocks="rouwenhorst")
N, Na = cal["N"], 20000
r = 0.04
w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
a = cal["a_grid"]
pc0 = np.tile(((1 + r) * a + w * np.mean(cal["s"]))[None, :], (N, 1))

# 1-2. EGM solve loops (chained launches)
for labor in (False, True):
    ws = pkg.Workspace(N, Na)
    c = t(pc0)
    pk = torch.zeros_like(c)
    pl = torch.zeros_like(c) if labor else None
    pkg.egm_solve_dev(ws, c, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], cal["amin"], 0.0, 200,
                      pk, labor=labor, phi=1.0, theta=1.0, policy_l=pl)
    torch.cuda.synchronize()

# 3. KS Howard sweeps at the scaling size, one rank (the bench leg's world = 1 schedule)
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

# 4. histogram pushes on the r = 0.04 policy
vws = pkg.Workspace(N, Na)
va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
vb = torch.zeros_like(va)
idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
vws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5, 1000, idx)
lam0 = torch.full((N, Na), 1.0 / (N * Na), dtype=torch.float64, device=dev)
out = torch.empty_like(lam0)
pkg.dist_stationary_dev(pkg.Workspace(N, Na), lam0, a_t, P_t, out, policy_idx=idx, tol=0.0,
                        max_iter=64)
torch.cuda.synchronize()
print("pmc workloads r04 done")
