"""BASELINE config 4: the GE r search of Aiyagari_VFI.m with candidate rates solved in
parallel, one process per GPU (torch.distributed; RCCL on GPUs), two multisection rounds of
the bisection tree (63 + 15 candidates) instead of 10 sequential steps.

    python bench_ge.py [--na 400] [--levels 6]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench_ge.py

Prints one JSON line: wall time to the final r (max over ranks), the trace length, the
candidates solved, and the sequential bisection's wall time on the same GPU for comparison
(rank 0, world 1 only)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--na", type=int, default=400)
    ap.add_argument("--levels", type=int, default=6,
                    help="bisection-tree levels per round (6: BASELINE's 63+1 candidates; 0: auto)")
    ap.add_argument("--no-sequential", action="store_true")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (started here when no launcher)")
    args = ap.parse_args()
    import bench_launch
    bench_launch.relaunch(args.gpus, str(Path(__file__).resolve()), sys.argv[1:])
    world, rank, local = bench_launch.check_world(args.gpus)
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    torch.cuda.set_device(local)  # before the process group: RCCL binds the current device
    if world > 1:
        dist.init_process_group("nccl")
    pkg = bench.load_pkg()
    gb = pkg.ge_batch
    pkg.ge_batch.aiyagari_vfi_multisection(Na=args.na, levels=1, rank=0, world=1)  # warm-up
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    A = gb.aiyagari_vfi_multisection(Na=args.na, levels=args.levels or None, rank=rank,
                                     world=world)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t[0])
    if rank == 0:
        out = {"metric": "wall time to GE equilibrium r (Aiyagari_VFI.m, multisection)",
               "value": dt, "unit": "s", "n_gpus": world, "higher_is_better": False,
               "r": A.r, "steps": len(A.r_history), "rounds": A.rounds,
               "candidates": A.candidates, "sweeps_rank0": int(sum(A.iters)),
               "config": {"workload": f"Aiyagari_VFI.m GE, Na={args.na}, Tauchen N=7, MC T=1e4, "
                                      f"warm start from the r0=0.04 solution",
                          "levels_per_round": args.levels,
                          "parallelism": f"{world} ranks x candidates round-robin"}}
        if world == 1 and not args.no_sequential:
            cal = pkg.calibration.aiyagari(Na=args.na)
            w0 = pkg.calibration.wage(0.04, cal["alpha"], cal["delta"])
            t1 = time.perf_counter()
            v0 = pkg.vfi_solve(np.zeros((cal["N"], args.na)), cal["a_grid"], cal["s"], cal["P"],
                               0.04, w0, cal["beta"], cal["sigma"])["v_old"]
            S = gb.bisection(gb.hip_vfi_evaluator(cal, v0), -0.05, 1 / cal["beta"] - 1)
            out["sequential_s"] = time.perf_counter() - t1
            out["identical_trace"] = S.r_history == A.r_history
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
