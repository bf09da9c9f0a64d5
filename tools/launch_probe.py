"""Workloads for the launch-floor attribution (run under rocprofv3 --kernel-trace, then
tools/launch_gaps.py): a chain of trivial kernels, EGM steps at Na = 400 and 20,000 (two
launches per step), headline sweeps (table + tree) and histogram pushes, each back to back on
one stream with no host synchronisation inside the chain."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

pkg = bench.load_pkg()
dev = torch.device("cuda:0")
x = torch.zeros(1, dtype=torch.float64, device=dev)
for _ in range(300):  # trivial one-wave kernels, dependent through x
    x.add_(1.0)
torch.cuda.synchronize()
t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)
for Na, variant in ((400, 2048), (20000, 4096), (20000, -1)):
    cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
    N, r = cal["N"], 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    a = cal["a_grid"]
    ws = pkg.Workspace(N, Na)
    ws.set_variant(variant)
    c = [t(np.tile(((1 + r) * a + w * np.mean(cal["s"]))[None, :], (N, 1))),
         torch.zeros((N, Na), dtype=torch.float64, device=dev)]
    pk = torch.zeros_like(c[0])
    a_t, s_t, P_t = t(a), t(cal["s"]), t(cal["P"])
    for q in range(200):
        pkg.egm_step_dev(ws, c[q & 1], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"],
                         cal["amin"], c[1 - (q & 1)], pk)
    torch.cuda.synchronize()
print("probe done")
