"""Workloads for the PMC passes of the secondary kernels (tools/pmc.sh with PMC_CMD set to this
script): the config-4 batched multi-rate launch (8 rates, Na = 20,000, sweeps 1-25 from v = 0),
labour VFI sweeps (Na = 400 and 20,000, sweeps 1-15 / 1-8), EGM steps (Na = 20,000, two
launches, 40 steps), histogram pushes (Na = 20,000 policy of the r = 0.04 solve, 64 pushes).
The kernel names separate them in the counter files except the batched A1 launch: it runs
first, so its 25 launches are the first 25 bell_tree_kernel<4, false, 1, 1, 1> dispatches
(pmc_summary take = 25); the r = 0.04 solve that makes the pushes' policy follows."""
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

# 1. config-4 batch: 8 rates x 25 sweeps from v = 0, one tree launch per sweep over all rates
C = 8
rs = list(np.linspace(-0.03, 0.035, C))
ws_b = [pkg.calibration.wage(x, cal["alpha"], cal["delta"]) for x in rs]
bws = pkg.Workspace(N, Na)
bv = [torch.zeros((C, N, Na), dtype=torch.float64, device=dev) for _ in range(2)]
bidx = torch.zeros((C, N, Na), dtype=torch.int32, device=dev)
bpk, bpc = torch.zeros_like(bv[0]), torch.zeros_like(bv[0])
pkg.vfi.solve_batch_dev(bws, rs, ws_b, bv[0], bv[1], a_t, s_t, P_t, cal["beta"], cal["sigma"],
                        0.0, 25, bidx, bpk, bpc)
torch.cuda.synchronize()

# 2. the r = 0.04 solve (the pushes' policy)
ws = pkg.Workspace(N, Na)
va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
vb = torch.zeros_like(va)
idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
ws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5, 1000, idx)
torch.cuda.synchronize()

# 3. histogram pushes
lam0 = torch.full((N, Na), 1.0 / (N * Na), dtype=torch.float64, device=dev)
out = torch.empty_like(lam0)
pkg.dist_stationary_dev(pkg.Workspace(N, Na), lam0, a_t, P_t, out, policy_idx=idx, tol=0.0,
                        max_iter=64)

# 4. EGM steps (two launches each)
ew = pkg.Workspace(N, Na)
a = cal["a_grid"]
c = [t(np.tile(((1 + r) * a + w * np.mean(cal["s"]))[None, :], (N, 1))), torch.zeros_like(va)]
pk = torch.zeros_like(va)
for q in range(40):
    pkg.egm_step_dev(ew, c[q & 1], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], cal["amin"],
                     c[1 - (q & 1)], pk)
torch.cuda.synchronize()

# 5. labour VFI sweeps (the labour script's calibration, Nl = 10), from v = 0
L = 0.01 + (1.5 - 0.01) * pkg.calibration.linspace01(10)
for lna, sweeps in ((400, 15), (20000, 8)):
    lc = pkg.calibration.aiyagari(Na=lna, rho=0.6, sigma_e=0.2)
    lws = pkg.Workspace(lc["N"], lna, 10)
    lv = [torch.zeros((lc["N"], lna), dtype=torch.float64, device=dev) for _ in range(2)]
    lin = torch.zeros((lc["N"], lna), dtype=torch.int32, device=dev)
    lpk, lpl, lpc = (torch.zeros_like(lv[0]) for _ in range(3))
    lw = pkg.calibration.wage(r, lc["alpha"], lc["delta"])
    for q in range(sweeps):
        lws.labor_vfi_sweep(lv[q & 1], t(lc["a_grid"]), t(lc["s"]), t(lc["P"]), t(L), r, lw,
                            lc["beta"], lc["sigma"], 1.0, 2.0, lv[1 - (q & 1)], lin, lpk, lpl, lpc,
                            hint=None if q == 0 else lin)
    torch.cuda.synchronize()
print("pmc workloads done")
