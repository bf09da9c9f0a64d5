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
KS_FLOPS_PER_NODE = 126  # algorithmic fp64 flops of one fused Howard node (ks_leg)
sys.path.insert(0, str(ROOT))


def ks_leg(pkg, world, rank, dev, nk=32768, nK=64, howard=50, exchange="halo", reps=3,
           depth=None, balanced=True):
    """Time one VFI iteration of the sharded solve (policy improvement + `howard` Jacobi
    sweeps with their exchanges, Krusell_Smith_VFI.m:148-192) at k = nk, K = nK, S = 4, max
    over ranks, median of `reps`.  depth: Howard sweeps per exchange (ks_dist.HowardSweeps;
    default 4 on more than one rank); balanced: K ranges cut at ks_dist.balanced_bounds (equal
    ghost-block cost per rank) when depth > 1.  Every rank must call it (collectives inside)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    kd = pkg.ks_dist
    if depth is None:
        depth = 4 if world > 1 else 1
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    bounds = None
    if balanced and 1 < world <= nK and depth > 1 and exchange == "halo":
        bounds = kd.balanced_bounds(kd.forecast_index(Kg, B, pkg.ks_params()), nK, world, depth)
    K0, K1, s0, s1 = kd.shard_slices(nK, rank, world, bounds)
    sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), K0, K1, s0, s1)
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
    V2 = V.clone()
    ko = torch.ones_like(V)
    if world > 1:
        dist.barrier()
    hs = kd.HowardSweeps(sh, nK, rank, world, V, depth=depth, exchange=exchange, bounds=bounds)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    hs.improve(V, ko)  # warm-up (kernels, caches, communicators)
    V, V2 = hs.run(V, V2, ko, 2 * hs.depth)
    samples = []
    for _ in range(reps):
        sync()
        t0 = time.perf_counter()
        hs.improve(V, ko)
        sync()
        t1 = time.perf_counter()
        V, V2 = hs.run(V, V2, ko, howard)
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
    cols = hs.halo.columns if hs.halo is not None else 0
    gcols = hs.blocks[hs.depth].columns if hs.depth > 1 else cols
    ghost = [(r[1] - r[0]) * (r[3] - r[2]) for r in hs.rects]
    hs.close()
    sh.close()
    # Algorithmic bytes per node and Howard sweep (each array touched once): the slope rebuild
    # reads V and writes dV (16 B); the sweep reads k_opt and the segment hint (12 B), the V/dV
    # columns its forecast reads (16 B, each column once) and writes V (8 B) -> 52 B.
    bpn = 52
    gbs = nodes * bpn / (th / howard) / 1e9 / world  # per GPU
    # The sweep is VALU-bound (PMC: ~73 % VALU busy, 5 waves/SIMD; traffic ~1.6x algorithmic),
    # so the roof is fp64 vector throughput on the algorithmic flops of one node:
    #   bellman_value: 4 pchip evaluations (pwch coefficients + Horner, 16 flops each with 4
    #   divisions, + the shared h and x - x_i: 66), the expectation (8), the budget (3), aiy_log
    #   (fdlibm, 28 with 1 division), beta*E + u (2) = 107; the fused next-sweep slope
    #   (Fritsch-Butland interior rule, 19 with 7 divisions) -> 126 flops, divisions counted as
    #   one flop as in SURVEY D3.
    fpn = KS_FLOPS_PER_NODE
    tfs = nodes * fpn / (th / howard) / 1e12 / world
    pmc, pmc_src = _ks_pmc()
    return {"metric": "Krusell-Smith bellman_value evals/sec (Howard sweeps, fp64)",
            "value": nodes * howard / th, "unit": "evals/s", "n_gpus": world,
            "roofline": {"bound": "valu", "achieved": tfs, "peak": 78.6, "unit": "TFLOP/s",
                         "frac": tfs / 78.6,
                         "traffic": next(iter((pmc or {None: {}}).values())).get(
                             "hbm_bytes_per_launch"),
                         "basis": f"{fpn} fp64 flops per node per Howard sweep (4 pchip "
                                  f"evaluations 66, expectation 8, budget 3, aiy_log 28, "
                                  f"beta*E + u 2, fused pchip slope 19; 24 divisions counted "
                                  f"as one flop each, SURVEY D3) x {nodes // world} nodes per "
                                  f"GPU / sweep time; peak = fp64 vector 78.6 TF/s",
                         "hbm_secondary": {"achieved": gbs, "peak": 8000.0, "unit": "GB/s",
                                           "frac": gbs / 8000.0,
                                           "basis": f"{bpn} B algorithmic per node per sweep "
                                                    f"(slopes: V in, dV out; sweep: k_opt, "
                                                    f"segment hint, forecast V/dV columns in, "
                                                    f"V out)"}},
            "pmc": pmc,
            "pmc_source": pmc_src,
            "scaling": "strong", "vfi_iteration_ms": (ti + th) * 1e3,
            "howard_ms_per_sweep": th / howard * 1e3, "improve_ms": ti * 1e3,
            "workload": f"Krusell_Smith_VFI k={nk} K={nK} S=4 ({nodes} nodes, BASELINE "
                        f"configs[4] scaling size), ALM B={[float(b) for b in B]}, one VFI "
                        f"iteration = improvement + {howard} Howard sweeps, median of {reps}",
            "parallelism": f"(K, Z) shards over {world} ranks (rank 0: K [{K0}, {K1}), s "
                           f"[{s0}, {s1}); K bounds {bounds or 'even'}), {exchange} exchange "
                           + (f"every {hs.depth} Howard sweeps (ghost rectangles of rank 0: "
                              f"{ghost} columns; {gcols} columns received per block)"
                              if hs.depth > 1 else
                              f"per Howard sweep (rank 0 receives {cols} (s, K) columns of "
                              f"{nk} values)")}


def ks_direct_leg(pkg, world, rank, dev, nk=32768, nK=64, howard=50, reps=3, check_sweeps=6):
    """The direct schedule under one process per GPU (ks_dist.DirectPeers: forecast columns
    read in the owners' buffers through IPC mappings, a stream-ordered counter hand-off per
    sweep, no copies, no ghost sweeps): one VFI iteration (improvement + `howard`
    sweeps) at the scaling size, max over ranks, median of `reps`.  Before timing, the same
    short run (improvement + `check_sweeps` sweeps from the same start) through the halo
    schedule, which the tests pin bit-exact to the single-device solve, must give identical
    own columns on every rank (`bit_exact_vs_halo`).  Every rank must call it."""
    import numpy as np
    import torch
    import torch.distributed as dist
    kd = pkg.ks_dist
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    K0, K1, s0, s1 = kd.shard_slices(nK, rank, world)
    sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), K0, K1, s0, s1)
    Vs = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # the exactness check: halo schedule (depth 1) vs direct on the same start
    Vh, Vh2, koh = Vs.clone(), Vs.clone(), torch.ones_like(Vs)
    hs = kd.HowardSweeps(sh, nK, rank, world, Vh, depth=1)
    hs.improve(Vh, koh)
    Vh, Vh2 = hs.run(Vh, Vh2, koh, check_sweeps)
    hs.close()
    dp = kd.DirectPeers(sh, nK, rank, world, Vs)
    kod = torch.ones_like(Vs)
    dp.start(Vs)
    dp.improve(kod)
    dp.sweeps(kod, check_sweeps)
    sync()
    dp.check()
    flat = lambda t: t.view(-1, nk)
    same = all(torch.equal(flat(dp.current())[a:b], flat(Vh)[a:b]) and
               torch.equal(flat(kod)[a:b], flat(koh)[a:b]) for a, b in dp.own_runs())
    ok = torch.tensor([1.0 if same else 0.0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    del Vh, Vh2, koh
    # timing: improvement + howard sweeps, as ks_leg
    dp.sweeps(kod, 2)
    samples = []
    for _ in range(reps):
        sync()
        t0 = time.perf_counter()
        dp.improve(kod)
        sync()
        t1 = time.perf_counter()
        dp.sweeps(kod, howard)
        sync()
        t2 = time.perf_counter()
        samples.append((t1 - t0, t2 - t1))
    dp.check()
    ti = sorted(x[0] for x in samples)[reps // 2]
    th = sorted(x[1] for x in samples)[reps // 2]
    if world > 1:
        t = torch.tensor([ti, th], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ti, th = float(t[0]), float(t[1])
    nbr = len(dp.nbr)
    sh.set_columns(None)
    dp.close()
    sh.close()
    nodes = nk * nK * 4
    bpn = 52
    gbs = nodes * bpn / (th / howard) / 1e9 / world
    exact = bool(ok[0] > 0.5)
    out = {} if exact else {
        "error": "direct schedule differs from the halo schedule on the same start: value "
                 "withheld (multi-GPU parity of the direct schedule is pinned only by this check)"}
    return {**out, "metric": "Krusell-Smith bellman_value evals/sec (Howard sweeps, fp64)",
            "value": nodes * howard / th if exact else None, "unit": "evals/s", "n_gpus": world,
            "value_unchecked": nodes * howard / th,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s",
                         "frac": gbs / 8000.0,
                         "basis": f"{bpn} B algorithmic per node per Howard sweep x "
                                  f"{nodes // world} nodes per GPU / sweep time"},
            "scaling": "strong", "vfi_iteration_ms": (ti + th) * 1e3,
            "howard_ms_per_sweep": th / howard * 1e3, "improve_ms": ti * 1e3,
            "bit_exact_vs_halo": exact,
            "workload": f"Krusell_Smith_VFI k={nk} K={nK} S=4 ({nodes} nodes), one VFI iteration "
                        f"= improvement + {howard} Howard sweeps, median of {reps}",
            "parallelism": f"(K, Z) shards over {world} ranks (rank 0: K [{K0}, {K1}), s [{s0}, "
                           f"{s1})), direct schedule: forecast columns read in the owners' "
                           f"buffers (IPC), counter hand-off with {nbr} neighbour(s) per sweep"}


def _ks_pmc():
    """Counter summary of the kernel this leg times — one launch per Howard sweep at k = 32,768,
    K = 64 (rocprofv3 --pmc passes over tools/pmc_workloads_r05.py ks, tools/exp/r06_pmc.sh):
    ks_howard_slopes_xcd_kernel from round 6, ks_howard_slopes_kernel before — from the newest
    round's files committed under profiles/."""
    for rnd in ("r06", "r05", "r04"):
        name = "ks_howard_slopes_xcd_kernel" if rnd >= "r06" else "ks_howard_slopes_kernel"
        p = ROOT / "profiles" / f"{rnd}_pmc_ks_howard_slopes.json"
        q = ROOT / "profiles" / f"{rnd}_traffic_ks_howard_slopes.json"
        if not p.exists():
            continue
        d = json.loads(p.read_text())["derived"]
        out = {name: {k: d[k] for k in ("valu_busy", "waves_per_simd", "valu_per_wave",
                                        "wait_frac") if k in d}}
        if q.exists():
            out[name]["hbm_bytes_per_launch"] = json.loads(q.read_text())["bytes_per_launch"]
        return out, f"profiles/{p.name}, profiles/{q.name} (the timed kernel)"
    return None, None


def ghost_model(pkg, dev, world=8, nk=32768, nK=64, depths=(1, 2, 3, 4, 6, 8), sweeps=24):
    """Compute side of the communication-avoiding schedule on ONE GPU: for each emulated rank
    of `world` (K-range shards of the scaling grid), the time of `sweeps` Howard sweeps run as
    blocks of `depth` (one slopes launch over what R_{L-1} reads, then one fused Howard+slopes
    launch per sweep over the ghost rectangles R_{L-1} .. R_0, ks_dist.HowardSweeps) without the
    exchanges — what each rank's GPU does between exchanges at N = world.  Returns, per depth,
    the slowest emulated rank's ms per sweep, for even K ranges and for the ranges of
    ks_dist.balanced_bounds (equal ghost-block cost per rank; what ks_leg uses at depth > 1)."""
    import numpy as np
    import torch
    kd = pkg.ks_dist
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    kp = kd.forecast_index(Kg, B, pkg.ks_params())
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
    V2 = V.clone()
    dV, dV2 = torch.empty_like(V), torch.empty_like(V)
    ko = torch.ones_like(V)
    res = {}
    for part in ("even", "balanced"):
        out, gout, per_rank, bnds = {}, {}, {}, {}
        for d in depths:
            bounds = kd.balanced_bounds(kp, nK, world, d) if part == "balanced" else None
            bnds[str(d)] = bounds or [nK * r // world for r in range(world + 1)]
            per_rank[str(d)] = []
            for rank in range(world):
                K0, K1, s0, s1 = kd.shard_slices(nK, rank, world, bounds)
                sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), K0, K1, s0, s1)
                sh.improve(V, ko)
                rects = kd.ghost_rects(sh.kp_idx, nK, K0, K1, s0, s1, d)
                shards = [sh] + [sh.ghost(*r) for r in rects[1:d]]
                shards[-1].hints(ko)

                def run(n):  # ks_dist.HowardSweeps' fused block schedule without the exchanges
                    nonlocal V, V2, dV, dV2
                    done = 0
                    while done < n:
                        L = min(d, n - done)
                        shards[L - 1].slopes(V, dV)
                        for i in range(1, L + 1):
                            shards[L - i].howard_fused(V, dV, ko, V2, dV2)
                            V, V2 = V2, V
                            dV, dV2 = dV2, dV
                        done += L
                run(d)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record()
                run(sweeps)
                e1.record()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / sweeps * 1e3
                gms = e0.elapsed_time(e1) / sweeps
                out[d] = max(out.get(d, 0.0), ms)
                gout[d] = max(gout.get(d, 0.0), gms)
                per_rank[str(d)].append(gms)
                for g in shards[1:]:
                    g.close()
                sh._ghosts.clear()
                sh.close()
        res[part] = {"ms_per_sweep_by_depth": {str(d): out[d] for d in depths},
                     "gpu_ms_per_sweep_by_depth": {str(d): gout[d] for d in depths},
                     "gpu_ms_per_sweep_by_rank": per_rank, "K_bounds": bnds}
    return {"world": world, "sweeps": sweeps,
            "ms_per_sweep_by_depth": res["even"]["ms_per_sweep_by_depth"],
            "gpu_ms_per_sweep_by_depth": res["even"]["gpu_ms_per_sweep_by_depth"],
            "even": res["even"], "balanced": res["balanced"],
            "note": "slowest emulated rank, compute only (no exchanges): ghost overhead vs depth; "
                    "top level = even K ranges (as in round 2), `balanced` = balanced_bounds; "
                    "ms_per_sweep = host wall clock (Python issue included), gpu_ms_per_sweep = "
                    "HIP events on the stream (tools/ks_ghost_probe.py gives the per-kernel split)"}


def direct_model(pkg, dev, world=8, nk=32768, nK=64, sweeps=24, howard=50):
    """Compute side of the direct (peer-read) schedule — ks_vfi_solve_sharded(depth = 0) — on ONE
    GPU: `world` emulated shards ((K, Z) slices, even K ranges), each with its own double-buffered
    value / slope arrays; each shard's improvement and fused Howard sweeps read the forecast
    columns in the OTHER shards' buffers through its column table (ks_dev_set_columns), as on
    `world` devices with peer pointers.  Each shard is timed alone (HIP events on the stream):
    its GPU time per sweep and per improvement is what its device does at N = world between the
    stream-event waits on its neighbours.  Returns the slowest shard's figures and the projected
    VFI iteration (improvement + `howard` sweeps, waits not included)."""
    import numpy as np
    import torch
    kd = pkg.ks_dist
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
    owner = [0] * (4 * nK)
    slices = [kd.shard_slices(nK, q, world) for q in range(world)]
    for q, (K0, K1, s0, s1) in enumerate(slices):
        for sidx in range(s0, s1):
            for K in range(K0, K1):
                owner[sidx * nK + K] = q
    sh = [kd.HipShard(kg, Kg, B, P, pkg.ks_params(), *slices[q]) for q in range(world)]
    Vb = [[V.clone(), V.clone()] for _ in range(world)]
    dVb = [[torch.empty_like(V), torch.empty_like(V)] for _ in range(world)]
    for q in range(world):
        sh[q].slopes_own(Vb[q][0], dVb[q][0])
        dVb[q][1].copy_(dVb[q][0])
    ko = torch.ones_like(V)
    tabs = [[kd.column_table([Vb[p][b] for p in range(world)], [dVb[p][b] for p in range(world)],
                             owner, nk) for b in range(2)] for _ in range(world)]
    torch.cuda.synchronize()
    ev = lambda: torch.cuda.Event(enable_timing=True)
    imp, swp = [], []
    for q in range(world):
        sh[q].set_columns(tabs[q][0])
        sh[q].improve_direct(ko)  # warm-up
        e0, e1 = ev(), ev()
        e0.record()
        sh[q].improve_direct(ko)
        e1.record()
        torch.cuda.synchronize()
        imp.append(e0.elapsed_time(e1))
        cur = 0

        def run(n):
            nonlocal cur
            for _ in range(n):
                sh[q].set_columns(tabs[q][cur])
                sh[q].howard_fused(Vb[q][cur], dVb[q][cur], ko, Vb[q][cur ^ 1], dVb[q][cur ^ 1])
                cur ^= 1
        run(2)
        e0, e1 = ev(), ev()
        e0.record()
        run(sweeps)
        e1.record()
        torch.cuda.synchronize()
        swp.append(e0.elapsed_time(e1) / sweeps)
    # the cross-process schedule's own cost (ks_dist.DirectPeers, staged): the slowest shard's
    # sweeps through ks_dev_direct_sweeps — ONE launch per sweep that publishes the previous
    # version in its slot of a mapped host page, copies the peers' forecast columns into a local
    # halo once the neighbours' slots allow it (its own slot here: self-satisfied), sweeps the
    # interior columns meanwhile and the boundary columns after the copies, on three buffers.
    # The copies here are device-local (the peers' buffers are on this GPU), so their time is an
    # HBM lower bound on the xGMI copy (DESIGN.md §6 budgets the link).
    import ctypes as C
    import mmap
    check, lib = pkg._capi.check, pkg._capi.lib
    def plan_of(x):
        K0x, K1x, s0x, s1x = slices[x]
        ownx = [sidx * nK + K for sidx in range(s0x, s1x) for K in range(K0x, K1x)]
        return kd.staged_plan(ownx, sh[x].kp_idx, owner, nK, x)
    # the shard with the most peer-owned forecast columns (ties: the slowest sweep)
    q = max(range(world), key=lambda x: (len(plan_of(x)[0]), swp[x]))
    remote, interior, boundary = plan_of(q)
    interior = np.ascontiguousarray(interior, np.int32)
    boundary = np.ascontiguousarray(boundary, np.int32)
    check(lib().ks_dev_set_split(sh[q]._h, C.c_void_p(interior.ctypes.data),
                                 C.c_int32(interior.size), C.c_void_p(boundary.ctypes.data),
                                 C.c_int32(boundary.size)))
    nr = len(remote)
    hV = torch.empty((max(nr, 1), nk), dtype=torch.float64, device=dev)
    hdV = torch.empty_like(hV)
    cb = 8 * nk
    slot = {c: i for i, c in enumerate(remote)}
    # shard q's third buffer (the other shards keep two: only their buffer b of the version
    # being read matters to q's copies and tables)
    Vq = Vb[q] + [Vb[q][0].clone()]
    dVq = dVb[q] + [dVb[q][0].clone()]
    bufV = lambda o, b: Vq[b] if o == q else Vb[o][b % 2]
    bufD = lambda o, b: dVq[b] if o == q else dVb[o][b % 2]
    stab = []
    for b in range(3):
        a = [(hV.data_ptr() + cb * slot[c]) if c in slot else bufV(owner[c], b).data_ptr() + cb * c
             for c in range(4 * nK)]
        a += [(hdV.data_ptr() + cb * slot[c]) if c in slot else bufD(owner[c], b).data_ptr() + cb * c
              for c in range(4 * nK)]
        stab.append(torch.tensor(a, dtype=torch.int64, device=dev))
    darr = lambda xs: torch.tensor(xs or [0], dtype=torch.int64, device=dev)
    src = [darr([bufV(owner[c], b).data_ptr() + cb * c for c in remote] +
                [bufD(owner[c], b).data_ptr() + cb * c for c in remote]) for b in range(3)]
    dst = darr([hV.data_ptr() + cb * i for i in range(nr)] + [hdV.data_ptr() + cb * i for i in range(nr)])
    page = mmap.mmap(-1, 16384)
    host = C.c_char.from_buffer(page)
    hp = C.addressof(host)
    dptr = C.c_void_p()
    check(lib().aiy_host_register(C.c_void_p(hp), C.c_int64(16384), C.byref(dptr)))
    C.c_uint64.from_address(hp).value = 1
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    p3 = lambda ts: (C.c_void_p * 3)(*[t.data_ptr() for t in ts])
    tabs3, V3, dV3, src3 = p3(stab), p3(Vq), p3(dVq), p3(src)
    cur = [0]

    def run_direct(n, n0):
        check(lib().ks_dev_direct_sweeps(
            sh[q]._h, tabs3, V3, dV3, C.c_void_p(ko.data_ptr()), C.c_int32(cur[0]), C.c_int64(n),
            src3, C.c_void_p(dst.data_ptr()), C.c_int32(2 * nr), C.c_int64(cb), dptr,
            C.c_int32(0), C.c_uint64(1), C.c_uint64(n0), C.c_double(30.0),
            C.c_void_p(dptr.value + 8192), st))
        cur[0] = (cur[0] + n) % 3
    run_direct(2, 1)
    e0, e1 = ev(), ev()
    e0.record()
    run_direct(sweeps, 3)
    e1.record()
    torch.cuda.synchronize()
    hand = e0.elapsed_time(e1) / sweeps
    err = C.c_uint64.from_address(hp + 8192).value
    check(lib().aiy_host_unregister(C.c_void_p(hp)))
    del host
    page.close()
    for x in sh:
        x.close()
    remote_bytes = 2 * nr * cb
    it_ms = max(imp) + howard * max(swp)
    return {"world": world, "sweeps": sweeps, "improve_ms_by_shard": imp,
            "gpu_ms_per_sweep_by_shard": swp, "gpu_ms_per_sweep_slowest": max(swp),
            "improve_ms_slowest": max(imp), "projected_vfi_iteration_ms": it_ms,
            "handoff": {"shard": q, "gpu_ms_per_sweep_with_handoff": hand,
                        "handoff_us_per_sweep": (hand - swp[q]) * 1e3, "timeouts": err,
                        "projected_vfi_iteration_ms": max(imp) + howard * (max(swp) + hand - swp[q]),
                        "remote_columns": nr, "remote_bytes_per_sweep": remote_bytes,
                        "interior_columns": int(interior.size),
                        "boundary_columns": int(boundary.size),
                        "xgmi_us_per_sweep_at_link_rate": remote_bytes / 153e9 * 1e6,
                        "note": "ks_dev_direct_sweeps (staged, one launch per sweep, three "
                                "buffers) on the shard with the most peer columns: publish, "
                                "self-satisfied counter wait and halo copies in the copy blocks, "
                                "interior columns beside them, boundary columns after the copies; "
                                "the copies are device-local here (xGMI time at one link's "
                                "153 GB/s: xgmi_us_per_sweep_at_link_rate); the neighbours' skew is "
                                "not in it"},
            "note": f"direct schedule (ks_vfi_solve_sharded depth 0) emulated on one GPU: each of "
                    f"{world} shards timed alone, reading the other shards' buffers through its "
                    f"column table; projected iteration = slowest improvement + {howard} x "
                    f"slowest sweep; `handoff` adds the staged schedule's one-launch hand-off (publish, waits, copies)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nk", type=int, default=32768)
    ap.add_argument("--nK", type=int, default=64)
    ap.add_argument("--howard", type=int, default=50)
    ap.add_argument("--exchange", default="halo", choices=("halo", "allgather"))
    ap.add_argument("--depth", type=int, default=None, help="Howard sweeps per exchange")
    ap.add_argument("--ghost-model", action="store_true",
                    help="one GPU: compute time per sweep vs depth for emulated 8-rank shards")
    ap.add_argument("--direct-model", action="store_true",
                    help="one GPU: per-shard time of the direct (peer-read) schedule, 8 shards")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (started here when no launcher)")
    args = ap.parse_args()
    import bench_launch
    bench_launch.relaunch(args.gpus, str(Path(__file__).resolve()), sys.argv[1:])
    world, rank, local = bench_launch.check_world(args.gpus)
    import torch
    import torch.distributed as dist
    import bench
    torch.cuda.set_device(local)  # before the process group: RCCL binds the current device
    if world > 1:
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    if args.ghost_model:
        out = ghost_model(bench.load_pkg(), dev, nk=args.nk, nK=args.nK)
    elif args.direct_model:
        out = direct_model(bench.load_pkg(), dev, nk=args.nk, nK=args.nK)
    else:
        out = ks_leg(bench.load_pkg(), world, rank, dev, args.nk, args.nK, args.howard,
                     args.exchange, depth=args.depth)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
