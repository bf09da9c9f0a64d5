"""BASELINE config 5: the Krusell-Smith VFI (Krusell_Smith_VFI.m:141-204) at the scaling size
of SURVEY §8(d) D6 (k = 32,768, K = 64 on [30, 50], S = 4: 8.4 M nodes), sharded over ranks by
K range, one process per GPU (ks_dist.py; after every Howard sweep each rank receives the halo
columns its nodes forecast into, RCCL point-to-point over xGMI).  bench.py runs the same leg
(`ks_sharded`) at every N.

    python bench_ks.py [--nk 32768] [--nK 64] [--howard 50] [--exchange halo|allgather]
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


def ks_leg(pkg, world, rank, dev, nk=32768, nK=64, howard=50, exchange="halo", reps=3):
    """Time one VFI iteration of the sharded solve (policy improvement + `howard` Jacobi
    sweeps with their exchanges, Krusell_Smith_VFI.m:148-192) at k = nk, K = nK, S = 4, max
    over ranks, median of `reps`.  Every rank must call it (collectives inside)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    kd = pkg.ks_dist
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    K0, K1, s0, s1 = kd.shard_slices(nK, rank, world)
    sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), K0, K1, s0, s1)
    own = torch.tensor(kd.owned_columns(nK, rank, world), device=dev)
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
    V2 = V.clone()
    ko = torch.ones_like(V)
    halo = None
    if world > 1:
        dist.barrier()
        if exchange == "halo":
            halo = kd.HaloExchange(kd.halo_plan(sh.kp_idx, nK, world), rank, world, dev, nk,
                                   V.dtype)

    def sweeps(n):
        nonlocal V, V2
        for _ in range(n):
            sh.howard(V, ko, V2)
            if halo is None and world > 1:
                fresh = V2.view(-1, nk).index_select(0, own)
                V2.copy_(V)
                V2.view(-1, nk).index_copy_(0, own, fresh)
            V, V2 = V2, V
            if halo is not None:
                halo(V)
            elif world > 1:
                kd._exchange(V, rank, world, nK)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    sh.improve(V, ko)  # warm-up (kernels, caches, communicators)
    sweeps(2)
    samples = []
    for _ in range(reps):
        sync()
        t0 = time.perf_counter()
        sh.improve(V, ko)
        sync()
        t1 = time.perf_counter()
        sweeps(howard)
        sync()
        t2 = time.perf_counter()
        samples.append((t1 - t0, t2 - t1))
    ti = sorted(x[0] for x in samples)[reps // 2]
    th = sorted(x[1] for x in samples)[reps // 2]
    if world > 1:
        t = torch.tensor([ti, th], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ti, th = float(t[0]), float(t[1])
    nodes = nk * nK * 4
    cols = halo.columns if halo is not None else (4 * nK - len(own) if world > 1 else 0)
    sh.close()
    # Algorithmic bytes per node and Howard sweep (each array touched once): the slope rebuild
    # reads V and writes dV (16 B); the sweep reads k_opt and the segment hint (12 B), the V/dV
    # columns its forecast reads (16 B, each column once) and writes V (8 B) -> 52 B.
    bpn = 52
    gbs = nodes * bpn / (th / howard) / 1e9 / world  # per GPU
    return {"metric": "Krusell-Smith bellman_value evals/sec (Howard sweeps, fp64)",
            "value": nodes * howard / th, "unit": "evals/s", "n_gpus": world,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s",
                         "frac": gbs / 8000.0,
                         "basis": f"{bpn} B algorithmic per node per Howard sweep (slopes: V in, dV "
                                  f"out; sweep: k_opt, segment hint, forecast V/dV columns in, V "
                                  f"out) x {nodes // world} nodes per GPU / sweep time; the "
                                  f"working set (V, dV, k_opt: 200 MB) is HBM-resident"},
            "scaling": "strong", "vfi_iteration_ms": (ti + th) * 1e3,
            "howard_ms_per_sweep": th / howard * 1e3, "improve_ms": ti * 1e3,
            "workload": f"Krusell_Smith_VFI k={nk} K={nK} S=4 ({nodes} nodes, BASELINE "
                        f"configs[4] scaling size), ALM B={[float(b) for b in B]}, one VFI "
                        f"iteration = improvement + {howard} Howard sweeps, median of {reps}",
            "parallelism": f"(K, Z) shards over {world} ranks (rank 0: K [{K0}, {K1}), s "
                           f"[{s0}, {s1})), {exchange} exchange per Howard sweep (rank 0 "
                           f"receives {cols} (s, K) columns of {nk} values)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nk", type=int, default=32768)
    ap.add_argument("--nK", type=int, default=64)
    ap.add_argument("--howard", type=int, default=50)
    ap.add_argument("--exchange", default="halo", choices=("halo", "allgather"))
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import bench
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    out = ks_leg(bench.load_pkg(), world, rank, dev, args.nk, args.nK, args.howard,
                 args.exchange)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
