"""Per-wave phase trace of the EGM interp1 kernel (two-launch step) and of the chained step
(egm_chain_kernel) at Na = 20,000 (aiy_ws_set_timing bit 2): shader cycles in the 64-ary search,
the LDS-window count, the interpolation loads + stores, and the rest (the RHS of step t+1 and
the reduction in the chained kernel), plus wave durations and start offsets.
    python tools/egm_trace.py [out.txt]"""
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
Na = 20000
cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
N, r = cal["N"], 0.04
w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
a = cal["a_grid"]
a_t, s_t, P_t = t(a), t(cal["s"]), t(cal["P"])
pc0 = np.tile(((1 + r) * a + w * np.mean(cal["s"]))[None, :], (N, 1))
lines = []


def summarize(name, tr):
    tr = tr[tr[:, 1] > 0]
    span = (tr[:, 1].max() - tr[:, 0].min()) / 100.0
    dur = (tr[:, 1] - tr[:, 0]) / 100.0
    start = (tr[:, 0] - tr[:, 0].min()) / 100.0
    lines.append(f"{name}: {len(tr)} waves, wall span {span:.2f} us")
    lines.append(f"  wave duration us p50/p90/p99/max {np.percentile(dur, [50, 90, 99, 100]).round(2).tolist()}")
    lines.append(f"  wave start offset us p50/p90/max {np.percentile(start, [50, 90, 100]).round(2).tolist()}")
    for p, nm in enumerate(("search (3 rounds)", "window count", "interp loads+stores", "rest")):
        col = tr[:, 3 + p]
        lines.append(f"  {nm:20s} cycles p50 {np.median(col):8.0f}  p99 {np.percentile(col, 99):8.0f}  max {col.max():8.0f}")


# two-launch step after 30 steps
ws = pkg.Workspace(N, Na)
c = [t(pc0), torch.zeros((N, Na), dtype=torch.float64, device=dev)]
pk = torch.zeros_like(c[0])
for q in range(31):
    if q == 30:
        ws.set_timing(True, trace=True)
    pkg.egm_step_dev(ws, c[q & 1], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], cal["amin"],
                     c[1 - (q & 1)], pk)
torch.cuda.synchronize()
summarize("egm_interp_kernel (two-launch step 31)", ws.trace())
ws.set_timing(False)
# chained solve: 31 steps at tol = 0, the last launch traced
ws2 = pkg.Workspace(N, Na)
c2 = t(pc0)
pk2 = torch.zeros_like(c2)
ws2.set_timing(True, trace=True)
pkg.egm_solve_dev(ws2, c2, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], cal["amin"], 0.0, 31, pk2)
torch.cuda.synchronize()
summarize("egm_chain_kernel (chained step 31)", ws2.trace())
txt = "\n".join(lines)
print(txt)
if len(sys.argv) > 1:
    Path(sys.argv[1]).write_text(txt + "\n")
