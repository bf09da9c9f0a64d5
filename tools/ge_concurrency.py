"""Why do the GE driver's solves slow down when they overlap?  Times one warm A1 solve at
Na = 400 (the GE loop's shape) alone, then k copies at once on k host threads / streams, with and
without MC chains running beside them, for a few speculation caps (aiy_ws_set_speculation).

    python tools/ge_concurrency.py [--out gpurun_out/ge_conc.json]
"""
import argparse
import concurrent.futures as cf
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "ge_conc.json"))
    ap.add_argument("--cases", default="1:0,2:0,4:0,8:0,1:1,2:2,4:2,0:1",
                    help="solves:chains pairs")
    ap.add_argument("--specs", default="16,64")
    ap.add_argument("--queues", type=int, default=0, help="GPU_MAX_HW_QUEUES (0: inherited)")
    ap.add_argument("--prio", action="store_true", help="solve streams at high priority")
    ap.add_argument("--excl", action="store_true", help="CU-exclusive sweep workgroups")
    ap.add_argument("--geo", default="", help="wide geometry S,NW,SB for the solve slots")
    ap.add_argument("--chain-shared", action="store_true",
                    help="chains without CU exclusivity (the GE driver sets it, round 6)")
    ap.add_argument("--chain-nap", type=float, default=2e-4, help="host poll interval of a chain")
    args = ap.parse_args()
    import os
    if args.queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.queues)  # before the HIP runtime starts
    torch.cuda.set_device(0)
    pkg = bench.load_pkg()
    ge = pkg.ge
    dev = torch.device("cuda:0")
    cal = pkg.calibration.aiyagari(Na=400)
    N, Na = cal["N"], 400
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=dev)
    a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    # the warm start: v_old of the r = 0.04 solve (what the bisection's first step starts from)
    root = ge._GESlot(N, Na, dev)
    w0 = pkg.calibration.wage(0.04, cal["alpha"], cal["delta"])
    it, which = root.ws.vfi_solve(root.va, root.vb, a_t, s_t, P_t, 0.04, w0, cal["beta"],
                                  cal["sigma"], 1e-5, 1000, root.idx, root.pk, root.pc)
    torch.cuda.synchronize()
    v_warm = (root.vb if which == 0 else root.va).clone()
    rs = [-0.004167, 0.018750, -0.027083, 0.007292, 0.030208, -0.015625, -0.038542, -0.009896]
    slots = [ge._GESlot(N, Na, dev) for _ in range(8)]
    for sl in slots:
        if args.geo:
            S_, NW_, SB_ = (int(x) for x in args.geo.split(","))
            sl.ws.set_wide(-1, S_, NW_, SB_)
        if args.excl:
            sl.ws.set_cu_exclusive(True)
    sims = [ge._GESim(N, Na, dev) for _ in range(4)]
    if args.chain_shared:
        for sm in sims:
            sm.ws.set_cu_exclusive(False)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    streams = [torch.cuda.Stream(device=dev, priority=(-1 if args.prio and q < 8 else 0))
               for q in range(12)]
    U = t(np.random.default_rng(5).random(9999))

    def solve(q):
        sl, st = slots[q], streams[q]
        r = rs[q]
        with torch.cuda.stream(st):
            sl.va.copy_(v_warm)
            sl.vb.zero_()
            t0 = time.perf_counter()
            it, _ = sl.ws.vfi_solve(sl.va, sl.vb, a_t, s_t, P_t, r,
                                    pkg.calibration.wage(r, cal["alpha"], cal["delta"]),
                                    cal["beta"], cal["sigma"], 1e-5, 1000, sl.idx, sl.pk, sl.pc,
                                    stream=st)
        ge._wait_polled(st)
        return time.perf_counter() - t0, it

    def chain(q):
        sm, st = sims[q], streams[8 + q]
        with torch.cuda.stream(st):
            t0 = time.perf_counter()
            pkg.sim.sim_capital_dev(sm.ws, root.pk, a_t, P_t, 2, float(cal["a_grid"][100]), U,
                                    sm.k, sm.status, stream=st)
        ge._wait_polled(st, nap=args.chain_nap)
        return time.perf_counter() - t0, 0

    res = {}
    with cf.ThreadPoolExecutor(max_workers=16) as pool:
        for spec in [int(x) for x in args.specs.split(",")]:
            for s in slots:
                s.ws.set_speculation(spec)
            for nsolve, nchain in [tuple(int(y) for y in x.split(":")) for x in args.cases.split(",")]:
                runs = []
                for rep in range(5):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    fs = [pool.submit(solve, q) for q in range(nsolve)]
                    fs += [pool.submit(chain, q) for q in range(nchain)]
                    out = [f.result() for f in fs]
                    runs.append((time.perf_counter() - t0, out))
                runs.sort(key=lambda x: x[0])
                wall, out = runs[len(runs) // 2]
                key = f"spec{spec}_solves{nsolve}_chains{nchain}"
                res[key] = {"wall_ms": wall * 1e3,
                            "solve_ms": [o[0] * 1e3 for o in out[:nsolve]],
                            "iters": [o[1] for o in out[:nsolve]],
                            "chain_ms": [o[0] * 1e3 for o in out[nsolve:]]}
                print(key, json.dumps({k: (np.round(v, 3).tolist() if isinstance(v, list) else round(v, 3))
                                       for k, v in res[key].items()}), flush=True)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
