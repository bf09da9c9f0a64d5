"""GE wall time at the script's defaults and a Na = 400 solve from v = 0, with the persistent
small-grid solve on (default) and off (tuning aid): python tools/ge_timing.py."""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    import torch
    pkg = bench.load_pkg()
    dev = torch.device("cuda", 0)
    cal = pkg.calibration.aiyagari(Na=400)
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    out = {}
    for persist in (True, False):
        ws = pkg.Workspace(cal["N"], 400)
        ws.set_persistent(persist)
        walls = []
        for _ in range(5):
            va = torch.zeros((cal["N"], 400), dtype=torch.float64, device=dev)
            vb = torch.zeros_like(va)
            idx = torch.zeros((cal["N"], 400), dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            it, _ = ws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5,
                                 1000, idx)
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
        out[f"solve_na400_persist{int(persist)}"] = {"iters": it, "ms": sorted(walls)[2] * 1e3,
                                                     "us_per_sweep": sorted(walls)[2] / it * 1e6}
        ws.close()
    for name, fn in (("ge_overlapped", pkg.ge.aiyagari_vfi_overlapped), ("ge_sequential", pkg.ge.aiyagari_vfi)):
        fn()  # warm
        walls = []
        for _ in range(3):
            t0 = time.perf_counter()
            R = fn()
            walls.append(time.perf_counter() - t0)
        out[name] = {"ms": sorted(walls)[1] * 1e3, "r": R["r"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
