"""A/B of chained sweeps (aiy_ws_set_chain) against a table launch per sweep, by grid size:
the solve to tol from v = 0 (A2, Aiyagari_VFI.m:65-90) and warm fixed-count sweeps
(aiy_vfi_sweeps_dev), best of `reps`, default geometry and one wave per tile (variant 0/16).
Prints one JSON line per (Na, variant, chain)."""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from conftest import load_pkg  # noqa: E402
from oracle import np_oracle as no  # noqa: E402


def main():
    pkg = load_pkg()
    dev = torch.device("cuda:0")
    reps = 5
    for Na in (400, 1000, 4096, 20000):
        cal = no.calib_aiyagari(Na=Na, shocks="tauchen" if Na <= 1000 else "rouwenhorst")
        N = cal["N"]
        t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
        a, s, P = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
        r = 0.04
        w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
        for variant in (-1, 0 if Na <= 4096 else 16):
            for chain in (False, True):
                ws = pkg.Workspace(N, Na)
                ws.set_chain(chain)
                if variant >= 0:
                    ws.set_variant(variant)
                va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
                vb = torch.zeros_like(va)
                idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
                pk, pc = torch.empty_like(va), torch.empty_like(va)
                solve = []
                for _ in range(reps):
                    va.zero_(); vb.zero_()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    it, which = ws.vfi_solve(va, vb, a, s, P, r, w, cal["beta"], cal["sigma"],
                                             1e-5, 1000, idx, pk, pc, mode=1)
                    torch.cuda.synchronize()
                    solve.append(time.perf_counter() - t0)
                sw = []
                n = 100
                for _ in range(reps):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    ws.vfi_sweeps(va, vb, a, s, P, r, w, cal["beta"], cal["sigma"], n, idx, pk,
                                  pc, hint=idx, mode=1)
                    torch.cuda.synchronize()
                    sw.append((time.perf_counter() - t0) / n)
                print(json.dumps({"Na": Na, "variant": variant, "chain": chain, "iters": it,
                                  "solve_ms": min(solve) * 1e3,
                                  "solve_us_per_sweep": min(solve) / it * 1e6,
                                  "warm_us_per_sweep": min(sw) * 1e6}), flush=True)


if __name__ == "__main__":
    main()
