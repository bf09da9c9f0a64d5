"""Instrumented look at labour tree sweeps (A3, labour script calibration, Nl = 10): per-item
start-up / tree-phase split and work counts.  Tuning aid only.
    python tools/labor_trace.py Na [variant ...]"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    import torch
    pkg = bench.load_pkg()
    Na = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    variants = [int(v) for v in sys.argv[2:]] or [-1]
    cal = pkg.calibration.aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    N = cal["N"]
    L = 0.01 + (1.5 - 0.01) * pkg.calibration.linspace01(10)
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    dev = torch.device("cuda", 0)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t, L_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"]), t(L)
    for var in variants:
        ws = pkg.Workspace(N, Na, 10)
        if var >= 0:
            ws.set_variant(var)
        v = [torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(2)]
        lin = torch.zeros((N, Na), dtype=torch.int32, device=dev)
        pk, pl, pc = (torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(3))
        cur = 0
        for q in range(101):
            tr = q in (3, 10, 100)
            if tr:
                ws.set_timing(True, trace=True)
            ws.labor_vfi_sweep(v[cur], a_t, s_t, P_t, L_t, r, w, cal["beta"], cal["sigma"], 1.0,
                               2.0, v[1 - cur], lin, pk, pl, pc, hint=None if q == 0 else lin)
            cur = 1 - cur
            if not tr:
                continue
            torch.cuda.synchronize()
            ms, _, _ = ws.timing()
            ws.set_timing(False)
            T = ws.trace()
            dur = (T[:, 1] - T[:, 0]) / 100.0
            boot = (T[:, 0] - T[:, 12]) / 100.0
            t0 = T[:, 12].min()
            print(f"variant {var} sweep {q}: kernel {ms*1e3:.1f} us, items {len(T)}, last end "
                  f"{(T[:, 1].max() - t0) / 100.0:.1f} us after the first entry")
            print("  tree phase us p50/max:", np.percentile(dur, [50, 100]).round(1),
                  " entry->start us p50/max:", np.percentile(boot, [50, 100]).round(1))
            print("  start-up cycles mean %.0f, output cycles mean %.0f" % (T[:, 13].mean(), T[:, 14].mean()))
            for name, col in (("sup", 3), ("blk", 4), ("cand", 5), ("exact", 6)):
                x = T[:, col].astype(float)
                print(f"  {name}: mean {x.mean():.1f} max {x.max():.0f}")
            cy = T[:, 8:12].astype(float)
            print("  wave-0 cycles mean: top/sup-tests %.0f  block-tests %.0f  fine %.0f  exact %.0f"
                  % tuple(cy.mean(0)))


if __name__ == "__main__":
    main()
