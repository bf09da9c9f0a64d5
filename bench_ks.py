"""BASELINE config 5: the Krusell-Smith VFI (Krusell_Smith_VFI.m:141-204) at the scaling size
of SURVEY §8(d) D6 (k = 32,768, K = 64 on [30, 50], S = 4: 8.4 M nodes), sharded over ranks by
K range, one process per GPU (ks_dist.py; RCCL all-gather of the value slices after every
Howard sweep).

    python bench_ks.py [--nk 32768] [--nK 64] [--howard 20]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench_ks.py

Unit = one bellman_value evaluation (:329-364): 4 pchip evaluations + 1 log.  Timed: one
policy improvement (fminbnd on every node) and `howard` Jacobi sweeps with their exchanges,
max over ranks.  Prints one JSON line (rank 0)."""
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
    ap.add_argument("--nk", type=int, default=32768)
    ap.add_argument("--nK", type=int, default=64)
    ap.add_argument("--howard", type=int, default=20)
    args = ap.parse_args()
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    from oracle import np_oracle as no  # grids/calibration only (Krusell_Smith_VFI.m:5-99)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pkg = bench.load_pkg()
    kd = pkg.ks_dist
    p, kg, Kg, P, V0, B = no.ks_setup(k_size=args.nk, K_size=args.nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    K0, K1 = kd.shard_range(args.nK, rank, world)
    sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), K0, K1)
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
    V2 = V.clone()
    ko = torch.ones_like(V)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def howard_sweeps(n):
        nonlocal V, V2
        for _ in range(n):
            sh.howard(V, ko, V2)
            V2[:, :K0, :] = V[:, :K0, :]
            V2[:, K1:, :] = V[:, K1:, :]
            V, V2 = V2, V
            if world > 1:
                kd._exchange(V, K0, K1, rank, world, args.nK)

    sh.improve(V, ko)  # warm-up (kernels, caches)
    howard_sweeps(2)
    sync()
    t0 = time.perf_counter()
    sh.improve(V, ko)
    sync()
    t1 = time.perf_counter()
    howard_sweeps(args.howard)
    sync()
    t2 = time.perf_counter()
    ti, th = t1 - t0, t2 - t1
    if world > 1:
        t = torch.tensor([ti, th], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ti, th = float(t[0]), float(t[1])
    nodes = args.nk * args.nK * 4
    if rank == 0:
        print(json.dumps({
            "metric": "Krusell-Smith bellman_value evals/sec (Howard sweeps, fp64)",
            "value": nodes * args.howard / th, "unit": "evals/s", "n_gpus": world,
            "scaling": "strong", "higher_is_better": True,
            "howard_ms_per_sweep": th / args.howard * 1e3, "improve_ms": ti * 1e3,
            "config": {"workload": f"Krusell_Smith_VFI k={args.nk} K={args.nK} S=4 "
                                   f"({nodes} nodes), ALM B={list(B)}",
                       "parallelism": f"K-range shards over {world} ranks, value all-gather "
                                      f"per Howard sweep"}}), flush=True)
    sh.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
