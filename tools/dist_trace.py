"""Per-wave phase trace of the A10 push (dist_push_kernel, aiy_ws_set_timing bit 2) on the
config-2 policy (Na = 20,000, r = 0.04 VFI argmax) and on a synthetic near-identity policy:
for the last push of a short run, each wave's staged range S, long-run lanes, and shader
cycles in: off loads, staging, mass sums, barrier + projection, diff reduction.
    python tools/dist_trace.py [out.txt]"""
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
a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
vws = pkg.Workspace(N, Na)
va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
vb = torch.zeros_like(va)
idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
vws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5, 1000, idx)
j = np.arange(Na)
synth = np.stack([np.clip((j * (0.9 + 0.02 * i)).astype(np.int32), 0, Na - 1) for i in range(N)])
lines = []
for name, pol in (("vfi_policy", idx), ("synthetic", t(synth.astype(np.int32)))):
    ws = pkg.Workspace(N, Na)
    lam0 = torch.full((N, Na), 1.0 / (N * Na), dtype=torch.float64, device=dev)
    out = torch.empty_like(lam0)
    pkg.dist_stationary_dev(ws, lam0, a_t, P_t, out, policy_idx=pol, tol=0.0, max_iter=64)
    ws.set_timing(True, trace=True)
    pkg.dist_stationary_dev(ws, out.clone(), a_t, P_t, out, policy_idx=pol, tol=0.0, max_iter=1)
    torch.cuda.synchronize()
    tr = ws.trace()
    ws.set_timing(False)
    span = (tr[:, 1].max() - tr[:, 0].min()) / 100.0
    ph = tr[:, 5:10]
    lines.append(f"{name}: {len(tr)} waves, wall span {span:.2f} us (100 MHz clock)")
    lines.append(f"  S p50/p99/max {np.percentile(tr[:, 3], [50, 99]).tolist()} {tr[:, 3].max()}; "
                 f"waves with long runs {int((tr[:, 4] > 0).sum())}")
    for p, nm in enumerate(("off loads", "staging", "mass", "barrier+proj", "diff+atomics")):
        lines.append(f"  {nm:14s} cycles p50 {np.median(ph[:, p]):8.0f}  p99 "
                     f"{np.percentile(ph[:, p], 99):8.0f}  max {ph[:, p].max():8.0f}")
    dur = (tr[:, 1] - tr[:, 0]) / 100.0
    lines.append(f"  wave duration us p50/p90/p99/max {np.percentile(dur, [50, 90, 99, 100]).round(2).tolist()}")
    start = (tr[:, 0] - tr[:, 0].min()) / 100.0
    lines.append(f"  wave start offset us p50/p90/max {np.percentile(start, [50, 90, 100]).round(2).tolist()}")
    slow = np.argsort(-(tr[:, 1] - tr[:, 0]))[:6]
    lines.append("  slowest (block, row, S, long, off/stage/mass/proj/out cycles):")
    for q in slow:
        lines.append(f"    {q // N} {q % N} {tr[q, 3]} {tr[q, 4]} {tr[q, 5:10].tolist()}")
txt = "\n".join(lines)
print(txt)
if len(sys.argv) > 1:
    Path(sys.argv[1]).write_text(txt + "\n")
