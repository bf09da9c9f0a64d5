"""Headline benchmark: Bellman evals/s (Na·Na'·Nz per sweep, fp64) for BASELINE config 2 —
Aiyagari VFI, Na = 20,000, Nz = 7 Rouwenhorst, one exhaustive Bellman sweep per step
(Aiyagari_VFI.m:70-83) on the MI355X, inputs resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Multi-GPU: the Aiyagari sweep does not shard (replicas only), so every rank
runs the same sweeps (weak scaling, no collective on the data path; --distinct-r gives each
rank its own GE candidate r instead); the timing is max over ranks.  Rank 0 prints one JSON
line.  The line also carries `ks_sharded` (BASELINE configs[4]): one VFI iteration of the
Krusell-Smith solve at k = 32,768, K = 64 sharded over the same N ranks ((K, Z) slices, one
ghost-rectangle exchange per block of 4 Howard sweeps on > 1 rank; strong scaling), and
`ge_batch` (configs[3]: multisection GE, candidates round-robin over the ranks, one all-gather
per round), so the driver's N = 1, 2, 4, 8 runs give their speed-ups directly.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
# hardware queues per process (HIP's default is 4): the GE driver runs up to two speculative
# solves and two Monte-Carlo chains on their own streams, and with 4 queues streams share them —
# a solve queued behind a 1.6 ms chain waits for it (tools/ge_concurrency.py, profiles/
# r06_g14_hw_queues.txt: 2 solves + 2 chains 3.2 ms at 4 queues, 2.9 at 16; 4 solves 2.7 vs
# 1.8 ms).  More than ~4 busy queues degrade instead (6 solves: 5.9 ms at 16 queues, 3.1 at 4 —
# the driver's lookahead 2 keeps 4 solves + 1 chain).  Raised (never lowered) by bench.py's main only, before the
# HIP runtime starts; the GE leg reports the wall at the inherited value too.
HW_QUEUES_INHERITED = os.environ.get("GPU_MAX_HW_QUEUES")  # recorded in ge_equilibrium


def raise_hw_queues():
    """bench.py's own process only (called first in main, before the HIP runtime starts; an
    import of this module changes nothing — tools/ge_wall_probe.py measures the inherited
    value through that)."""
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 16:
        os.environ["GPU_MAX_HW_QUEUES"] = "16"

PEAK_FP64_TFLOPS = 78.6   # MI355X fp64 vector (= fp64 matrix) peak, datasheet
FLOPS_PER_CANDIDATE = 8  # sub, mul, mul, div, sub, mul, add, max
FLOPS_PER_TEST = 7       # bound / candidate screen test: sub, max, mul, mul, sub, mul, max


def load_pkg():
    name = "aiyagari_replication_amd"
    if name in sys.modules:
        return sys.modules[name]
    root = ROOT / "aiyagari-replication_amd"
    spec = importlib.util.spec_from_file_location(name, root / "__init__.py",
                                                  submodule_search_locations=[str(root)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def feasible_candidates(a, s, r, w):
    """Σ_{i,j} #{k : a_k < coh_ij}: the candidates that carry arithmetic (c <= 0 is NaN in
    the reference, Aiyagari_VFI.m:73)."""
    tot = 0
    for si in s:
        coh = (1 + r) * a + w * si
        tot += int(np.searchsorted(a, coh, side="left").sum())
    return tot


def cpu_baseline(cal, r, w, sweeps, threads, info):
    """The C restatement (oracle/liborc.so, exhaustive, reference op order) timed on the host:
    one sweep on one core, `sweeps` sweeps on the job's CPU share, from v = 0 at the full
    workload size.  `value` is the all-cores rate."""
    from oracle import corc
    N, Na = cal["N"], cal["Na"]
    per = N * Na * Na
    out = {}
    for th, n in ((1, 1), (threads, sweeps)):
        got = corc.num_threads(th)
        v = np.zeros((N, Na))
        t0 = time.perf_counter()
        for _ in range(n):
            v, _, _, _ = corc.vfi_sweep(v, cal["a_grid"], cal["s"], cal["P"], r, w, cal["beta"],
                                        cal["sigma"])
        dt = time.perf_counter() - t0
        out[th] = (n * per / dt, got, dt, n)
    allv = out[threads]
    return dict(value=allv[0], unit="evals/s", cores=allv[1], kind="port",
                one_core={"value": out[1][0], "cores": 1, "seconds": out[1][2]},
                cpu=info,
                sample=f"exhaustive sweeps from v=0 at Na={Na}, Nz={N} (C restatement "
                       f"oracle/aiy_oracle.c, OpenMP over states): {allv[3]} sweeps on {allv[1]} "
                       f"threads in {allv[2]:.2f} s; 1 sweep on 1 thread in {out[1][2]:.2f} s")


def ge_wall(pkg, threads):
    """Second half of the metric: wall time to the GE equilibrium r of Aiyagari_VFI.m at its
    own defaults (BASELINE configs[0]: Na = 400, Tauchen N = 7, 10 bisection steps, MC supply
    with MATLAB's rand stream), GPU pipeline vs the C restatement on the host."""
    from oracle import corc
    from oracle import np_oracle as no
    pkg.ge.aiyagari_vfi(max_iter=5)  # warm the library / context (not timed)
    pkg.ge.aiyagari_vfi_overlapped(max_iter=5)
    t0 = time.perf_counter()
    seq = pkg.ge.aiyagari_vfi()
    seq_s = time.perf_counter() - t0
    walls = []
    for _ in range(5):  # the same equilibrium computed 5 times: value = the median wall
        t0 = time.perf_counter()
        out = pkg.ge.aiyagari_vfi_overlapped()
        walls.append(time.perf_counter() - t0)
    gpu_s = sorted(walls)[len(walls) // 2]
    cal = no.calib_aiyagari()
    cpu = {}
    for th in sorted({1, threads}):
        corc.num_threads(th)
        t0 = time.perf_counter()
        H = no.ge_bisection_vfi(cal, solve=lambda *a: corc.vfi_solve(*a))
        cpu[th] = time.perf_counter() - t0
    cpu_s = cpu[threads]
    inherited = queues_probe()
    return {"hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"]),
            "hw_queues_inherited": HW_QUEUES_INHERITED, "at_inherited_queues": inherited,
            "wall_s_gpu_inherited_queues": inherited.get("wall_s_gpu"),"workload": "Aiyagari_VFI.m defaults (configs[0]): initial VFI + 10-step bisection + MC",
            "r_gpu": out["r"], "r_cpu": H["r_final"], "identical_trace": out["r_history"] == H["r"],
            "sweeps": int(sum(out["iters"])), "wall_s_gpu": gpu_s, "wall_s_cpu": cpu_s,
            "wall_s_gpu_runs": walls,
            "driver": f"ge.aiyagari_vfi_overlapped (solves speculated {out['lookahead']} "
                      f"bisection level(s) ahead of the pending MC chain; {out['solves']} solve "
                      f"slots)",
            "wall_s_gpu_sequential": seq_s, "sequential_trace_equal": seq["r_history"] == out["r_history"]
            and seq["k_supply"] == out["k_supply"] and seq["iters"] == out["iters"],
            "cpu_cores": threads, "wall_s_cpu_1core": cpu[1],
            "cpu_kind": "port (oracle/aiy_oracle.c)"}


def queues_probe():
    """The same GE wall in a child process under the inherited GPU_MAX_HW_QUEUES (the value a
    library caller or the test suite runs with; bench.py raised its own to 16) — ADVICE r5."""
    import subprocess
    env = dict(os.environ)
    if HW_QUEUES_INHERITED is None:
        env.pop("GPU_MAX_HW_QUEUES", None)
    else:
        env["GPU_MAX_HW_QUEUES"] = HW_QUEUES_INHERITED
    try:
        p = subprocess.run([sys.executable, str(ROOT / "tools" / "ge_wall_probe.py")], env=env,
                           capture_output=True, text=True, timeout=300)
        return json.loads(p.stdout.strip().splitlines()[-1])
    except Exception as e:  # reported, never fatal to the bench
        return {"error": repr(e)[:200]}


def solve_wall(pkg, ws, cal, r, w, a_t, s_t, P_t, dev):
    """Config 2's wall time to tol: the whole A2 loop (Aiyagari_VFI.m:65-90) at Na = 20,000
    from v = 0 on the device tier, every sweep's convergence test included."""
    import torch
    N, Na = cal["N"], cal["Na"]
    va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
    vb = torch.zeros_like(va)
    idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    pk, pc = torch.empty_like(va), torch.empty_like(va)
    ws.invalidate()  # the solve at a new (r, w) rebuilds its feasible prefixes and dispatch
    torch.cuda.synchronize()  # order (host round trip): that cost is inside the timed solve
    t0 = time.perf_counter()
    iters, _ = ws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5, 1000,
                            idx, pk, pc, mode=1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"iters": iters, "wall_ms": dt * 1e3, "evals_per_s": iters * N * Na * Na / dt,
            "workload": f"vfi_solve Na={Na} Nz={N} tol=1e-5 from v=0 (device tier)"}


def _json_profile(name):
    f = ROOT / "profiles" / name
    return json.loads(f.read_text()) if f.exists() else None


PMC_ROUNDS = ("r06", "r05", "r04", "r03")  # newest first: counter passes of the kernels at HEAD


def _counters(name, traffic_name=None):
    """(derived PMC, HBM bytes per launch, source note) of the newest round's counter passes of
    one kernel workload (profiles/<round>_pmc_<name>.json, <round>_traffic_<name>.json; made by
    tools/pmc.sh + tools/pmc_summary.py / pmc_traffic.py)."""
    traffic_name = traffic_name or name
    for rnd in PMC_ROUNDS:
        pmc = _json_profile(f"{rnd}_pmc_{name}.json")
        if pmc is None:
            continue
        tf = _json_profile(f"{rnd}_traffic_{traffic_name}.json")
        src = f"profiles/{rnd}_pmc_{name}.json" + (f", profiles/{rnd}_traffic_{traffic_name}.json"
                                                    if tf else "")
        return pmc.get("derived"), (tf or {}).get("bytes_per_launch"), src
    return None, None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--repeats", type=int, default=5, help="timed blocks for the median (D7)")
    ap.add_argument("--na", type=int, default=20000)
    ap.add_argument("--mode", type=int, default=1, help="1 screened exhaustive, 2 plain")
    ap.add_argument("--k-chunk", type=int, default=1024)
    ap.add_argument("--variant", type=int, default=-1, help="screen geometry (tuning sweep)")
    ap.add_argument("--cpu-sweeps", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ge", action="store_true", help="skip the GE wall-time legs")
    ap.add_argument("--no-solve", action="store_true", help="skip the solve-to-tol leg")
    ap.add_argument("--no-ks", action="store_true", help="skip the sharded Krusell-Smith leg")
    ap.add_argument("--distinct-r", action="store_true",
                    help="N > 1: one GE candidate r per rank instead of the same r on every rank")
    ap.add_argument("--no-panel", action="store_true", help="skip the KS panel (F2/F3) leg")
    ap.add_argument("--ks-depth", type=int, default=None,
                    help="KS Howard sweeps per halo exchange (default 4 on >1 rank)")
    ap.add_argument("--one-call", action="store_true",
                    help="issue the timed sweeps with one aiy_vfi_sweeps_dev call (C++ loop) "
                         "instead of one Python call per sweep; same kernels")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the labour/EGM/batch legs (D4, D5 per-GPU)")
    ap.add_argument("--detail", default=str(ROOT / "gpurun_out" / "bench_detail.json"),
                    help="file for the full result (every leg); stdout's last line is the "
                         "compact contract line")
    ap.add_argument("--dry-run-cpu", action="store_true",
                    help="launcher/contract check without a GPU: gloo ranks, a trivial timed "
                         "CPU loop, the same barrier/max-over-ranks/contract line")
    args = ap.parse_args()
    raise_hw_queues()

    import bench_launch
    # --gpus N without a launcher: start N ranks (child torch.distributed.run), exit with its rc
    bench_launch.relaunch(args.gpus, str(Path(__file__).resolve()), sys.argv[1:])
    world, rank, local = bench_launch.check_world(args.gpus)
    if args.dry_run_cpu:
        return dry_run_cpu(args, world, rank)

    import torch
    import torch.distributed as dist
    import bench_legs as BL

    torch.cuda.set_device(local)  # before the process group: RCCL binds the current device
    if world > 1:
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)

    pkg = load_pkg()
    cal = pkg.calibration.aiyagari(Na=args.na, shocks="rouwenhorst")
    N, Na = cal["N"], cal["Na"]
    # weak scaling: every rank sweeps the same problem (r = 0.04), so the work per GPU is fixed
    # as N grows and the driver's efficiency compares like with like; --distinct-r gives each
    # rank its own GE candidate of the bracket [-0.05, 1/beta-1] instead (per-rank cost varies
    # with r: the feasible set shrinks as r falls)
    r_lo, r_hi = -0.05, 1 / cal["beta"] - 1
    r = r_lo + (r_hi - r_lo) * (rank + 1) / (world + 1) if (world > 1 and args.distinct_r) else 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])

    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    v = [torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(2)]
    idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    pk = torch.empty((N, Na), dtype=torch.float64, device=dev)
    pc = torch.empty((N, Na), dtype=torch.float64, device=dev)
    ws = pkg.Workspace(N, Na)
    ws.set_search(0, args.k_chunk)
    if args.variant >= 0:
        ws.set_variant(args.variant)

    cur = 0

    def step(first=False):
        nonlocal cur
        ws.vfi_sweep(v[cur], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], v[1 - cur], idx,
                     pk, pc, hint=None if first else idx, mode=args.mode)
        cur = 1 - cur

    for q in range(max(args.warmup, 1)):
        step(first=(q == 0))
    torch.cuda.synchronize()
    snap = [x.clone() for x in (v[0], v[1], idx)]
    snap_cur = cur

    def sweeps(n):
        """n sweeps of the solve (hint = the previous argmax): n table + tree launch pairs, one
        Python call per sweep, or with --one-call one aiy_vfi_sweeps_dev call (C++ loop)."""
        nonlocal cur
        if not args.one_call or args.mode != 1:
            for _ in range(n):
                step()
            return
        ws.vfi_sweeps(v[cur], v[1 - cur], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], n,
                      idx, pk, pc, hint=idx, mode=args.mode)
        cur ^= n & 1

    def restore():
        nonlocal cur
        v[0].copy_(snap[0]); v[1].copy_(snap[1]); idx.copy_(snap[2])
        cur = snap_cur
        torch.cuda.synchronize()

    def timed_block(kernel_events):
        """Wall time of the same `steps` sweeps (barrier + synchronize on both sides); with
        kernel_events, HIP events bracket every launch of the dominant kernel on its stream
        (they add ~5 us of gap per launch, so the contract blocks run without them)."""
        ws.set_timing(bool(kernel_events))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sweeps(args.steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt_rep = time.perf_counter() - t0
        kern_ms, launches, _ = ws.timing()
        ws.set_timing(False)
        return dt_rep, (kern_ms / max(launches, 1) if kernel_events else None)

    blocks = []  # wall s per timed block of the same sweeps
    for rep in range(max(args.repeats, 1)):
        if rep:
            restore()
        blocks.append(timed_block(False)[0])
    # value: the median block (median of >= 5 timed repeats after the warm-up); every
    # block is exactly `steps` sweeps between barrier + synchronize, and the first is reported too
    dt = sorted(blocks)[len(blocks) // 2]
    # the dominant kernel's average launch duration: HIP events around each launch of the same
    # sweeps, in a block of their own
    restore()
    dt_ev, kern_avg_ms = timed_block(True)
    # untimed instrumented pass: per-state work counters of the same sweeps
    restore()
    ws.set_timing(False, count=True)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    counters = ws.counters()
    ws.set_timing(False)
    exh = None
    if not args.no_extra and args.mode == 1 and world == 1:
        # SURVEY D3's exhaustive kernel (mode 2: table + plain scan + merge), same sweeps
        restore()
        exh_ms = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ws.vfi_sweep(v[cur], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], v[1 - cur],
                         idx, pk, pc, hint=None, mode=2)
            torch.cuda.synchronize()
            exh_ms.append((time.perf_counter() - t0) * 1e3)
            cur = 1 - cur
        exh = sorted(exh_ms)[1]
        restore()
    if world > 1:
        tt = torch.tensor([dt, kern_avg_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt, kern_avg_ms = float(tt[0]), float(tt[1])

    progress(f"headline: {dt / args.steps * 1e3:.4f} ms/step")
    legs = {}
    if not args.no_ks:   # BASELINE configs[4]: KS VFI sharded over the same ranks (strong)
        import bench_ks
        legs["ks_sharded"] = bench_ks.ks_leg(pkg, world, rank, dev, depth=args.ks_depth)
        if world > 1:  # the direct schedule across processes (IPC peer reads), same size
            try:  # (its failures are raised on every rank together: DirectPeers)
                legs["ks_direct"] = bench_ks.ks_direct_leg(pkg, world, rank, dev)
            except RuntimeError as e:
                legs["ks_direct"] = {"error": str(e)[:300]}
        if world == 1 and not args.no_extra:  # compute side of the N = 8 schedules, on this GPU
            legs["ks_sharded"]["direct_model"] = bench_ks.direct_model(pkg, dev)
            legs["ks_sharded"]["ghost_model"] = bench_ks.ghost_model(pkg, dev, depths=(4,))
        progress("ks_sharded done")
    if not args.no_ge:   # BASELINE configs[3]: multisection GE over the same ranks
        legs["ge_batch"] = BL.ge_batch_leg(pkg, world, rank, dev)

    if rank == 0:
        info = BL.cpu_info()
        threads = info["threads_all"]
        evals_per_sweep = N * Na * Na
        value = world * evals_per_sweep * args.steps / dt
        feas = feasible_candidates(cal["a_grid"], cal["s"], r, w)
        tests = {n: c / args.steps for n, c in zip(("exact", "superblock", "block", "candidate"),
                                                   counters)}
        kname = "bell_screen_kernel" if (args.variant >= 0 and args.variant & 8) else "bell_tree_kernel"
        # Work the kernel executes per launch (counted live, per state): every bound test and
        # candidate test is FLOPS_PER_TEST fp64 flops, every exact evaluation FLOPS_PER_CANDIDATE.
        executed = (FLOPS_PER_TEST * (tests["superblock"] + tests["block"] + tests["candidate"])
                    + FLOPS_PER_CANDIDATE * tests["exact"])
        achieved = executed / (kern_avg_ms * 1e-3) / 1e12
        # SURVEY §8(d) D3 basis: 8 flops x every candidate (i, j, a') of the exhaustive scan the
        # result is bit-identical to -- the rate an exhaustive kernel would need to match it
        effective = FLOPS_PER_CANDIDATE * evals_per_sweep / (kern_avg_ms * 1e-3) / 1e12
        # PMC / HBM-traffic passes over the same sweeps 6..25 on the current kernels
        # (tools/exp/r06_pmc.sh: tools/pmc.sh + pmc_summary / pmc_traffic, skip 5 take 20)
        pmc_d, traffic, pmc_src = _counters("tree", "vfi_tree")
        step_ms = sorted(blocks)
        out = {
            "metric": "Bellman evals/sec (Na·Na'·Nz, fp64)",
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (reference calibration: Rouwenhorst Nz=7, quadratic grid)",
            "config": {"workload": f"aiyagari_vfi_sweep Na={Na} Nz={N} rouwenhorst"
                                   + (" (BASELINE configs[1])" if (Na, N) == (20000, 7) else ""),
                       "Na": Na, "Nz": N, "sigma": cal["sigma"], "beta": cal["beta"],
                       "search": "exhaustive over a' (exact bound-tree screen)" if args.mode == 1
                                 else "exhaustive over a' (plain)",
                       "sweeps_timed": f"sweeps {args.warmup + 1}..{args.warmup + args.steps} of a "
                                       f"solve from v=0, hint = previous argmax",
                       "parallelism": (f"replicas: one GE candidate r per rank ({world})"
                                       if world > 1 and args.distinct_r else
                                       f"replicas: the same sweeps (r = 0.04) on each of {world} "
                                       f"rank(s), no data-path collective"),
                       "feasible_fraction": feas / evals_per_sweep,
                       "tests_per_sweep": tests},
            "repeats": {"n": len(blocks), "median_ms_per_step": step_ms[len(blocks) // 2]
                        / args.steps * 1e3, "min_ms_per_step": step_ms[0] / args.steps * 1e3,
                        "max_ms_per_step": step_ms[-1] / args.steps * 1e3,
                        "first_block_ms_per_step": blocks[0] / args.steps * 1e3,
                        "kernel_timing_block_ms_per_step": dt_ev / args.steps * 1e3,
                        "gpu_clock": BL.gpu_clock(local),
                        "note": "the same sweeps re-run from a snapshot; value = the median block "
                                "(SURVEY D7); "
                                "the kernel average comes from one more block of the same sweeps "
                                "with HIP events around every launch (their gaps excluded from "
                                "the contract blocks)"},
            "roofline": {"bound": "valu", "achieved": achieved, "peak": PEAK_FP64_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / PEAK_FP64_TFLOPS,
                         "traffic": traffic,
                         "kernel": kname,
                         "kernel_avg_ms": kern_avg_ms,
                         "basis": f"executed work: {FLOPS_PER_TEST} fp64 flops per bound/candidate "
                                  f"test and {FLOPS_PER_CANDIDATE} per exact evaluation, counted "
                                  f"per state in an instrumented pass of the same sweeps "
                                  f"({executed:.3g} flops/launch); peak = fp64 vector 78.6 TF/s",
                         "effective_tflops_d3": effective,
                         "effective_frac_d3": effective / PEAK_FP64_TFLOPS,
                         "effective_basis": f"SURVEY D3: {FLOPS_PER_CANDIDATE} flops x Na*Na'*Nz = "
                                            f"{evals_per_sweep} candidates per launch, the exhaustive "
                                            f"scan this kernel reproduces bit for bit",
                         "pmc": pmc_d,
                         "pmc_source": f"{pmc_src} (rocprofv3 --pmc, tools/pmc.sh + "
                                       f"tools/pmc_summary.py / pmc_traffic.py, same sweeps "
                                       f"6..25)"},
        }
        out.update(legs)
        if exh is not None:  # the plain exhaustive scan's own roofline (mode 2)
            fl = FLOPS_PER_CANDIDATE * feas / (exh * 1e-3) / 1e12
            out["exhaustive"] = {
                "workload": f"one exhaustive sweep at Na={Na} (mode 2: table + plain scan + merge; "
                            f"every feasible candidate evaluated exactly), median of 3",
                "ms_per_sweep": exh, "evals_per_s": evals_per_sweep / (exh * 1e-3),
                "roofline": {"bound": "valu", "achieved": fl, "peak": 78.6, "unit": "TFLOP/s",
                             "frac": fl / 78.6,
                             "basis": f"8 fp64 flops x {feas} feasible candidates per sweep "
                                      f"(the division counted as one flop; infeasible c <= 0 "
                                      f"candidates are NaN in the reference and skipped)"},
                "tree_speedup": exh / (dt / args.steps * 1e3)}
        if not args.no_solve:
            out["solve_to_tol"] = solve_wall(pkg, ws, cal, r, w, a_t, s_t, P_t, dev)
        if world == 1 and not args.no_extra:
            out["batch_config4_share"] = BL.batch_leg(pkg, dev)
            progress("batch_config4_share done")
            out["dist"] = BL.dist_leg(pkg, dev, cpu_threads=threads)
            progress("dist done")
            # counter passes of the kernels these legs time (tools/pmc_workloads_r05.py under
            # tools/pmc.sh, one workload per pass set: tools/exp/r06_pmc.sh)
            def attach(leg, name, kernel):
                pmc_d, tf, src = _counters(name)
                leg["roofline"].update(pmc={kernel: pmc_d}, traffic=tf, pmc_source=src)

            attach(out["batch_config4_share"], "batch", "bell_tree_kernel")
            out["labor_vfi"] = {"Na400": BL.labor_leg(pkg, dev, 400, cpu_threads=threads,
                                                      cpu=not args.no_cpu_baseline),
                                "Na20000": BL.labor_leg(pkg, dev, 20000, steps=5, reps=3,
                                                        cpu_threads=threads,
                                                        cpu=not args.no_cpu_baseline)}
            out["egm"] = {"Na20000": BL.egm_leg(pkg, dev, 20000, cpu_threads=threads),
                          "Na400": BL.egm_leg(pkg, dev, 400, cpu_threads=threads)}
            progress("labor_vfi, egm done")
            out["labor_egm"] = {"Na20000": BL.egm_leg(pkg, dev, 20000, labor=True,
                                                      cpu_threads=threads)}
            attach(out["labor_vfi"]["Na400"], "labor_na400", "bell_wide_kernel")
            attach(out["labor_vfi"]["Na20000"], "labor_na20000", "bell_tree_kernel")
            attach(out["egm"]["Na20000"], "egm_chain", "egm_chain_kernel")
            attach(out["labor_egm"]["Na20000"], "labor_egm_chain", "egm_chain_kernel")
            attach(out["dist"], "dist_push", "dist_push_kernel")
        if not args.no_panel and world == 1:   # F3/F2: KS shock panel + agent simulation
            import bench_panel
            out["ks_panel"] = bench_panel.panel_leg(pkg, dev, cpu_threads=threads)
            progress("ks_panel done")
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cal, r, w, args.cpu_sweeps, threads, info)
            progress("cpu_baseline done")
            if "ks_sharded" in out and world == 1:
                out["ks_sharded"]["cpu_baseline"] = BL.ks_cpu_baseline(pkg, threads=threads)
        if not args.no_ge and world == 1:
            out["ge_equilibrium"] = ge_wall(pkg, threads)
            if "ge_batch" in out:  # config 4's CPU baseline: the sequential C bisection
                g = out["ge_equilibrium"]
                out["ge_batch"]["cpu_baseline"] = {
                    "value": g["wall_s_cpu"], "unit": "s to equilibrium r", "cores": threads,
                    "kind": "port", "value_1core": g["wall_s_cpu_1core"],
                    "sample": "the whole sequential bisection of Aiyagari_VFI.m at its defaults "
                              "(C restatement oracle/aiy_oracle.c, OpenMP over states), the "
                              "same r trace"}
        import bench_report
        detail = None
        try:
            bench_report.write_detail(out, args.detail)
            detail = os.path.relpath(args.detail, ROOT)
        except OSError as e:
            progress(f"detail file not written: {e}")
        print(bench_report.contract_line(out, detail), flush=True)
    if world > 1:
        dist.destroy_process_group()


def dry_run_cpu(args, world, rank):
    """The multi-rank plumbing of main() on CPU (gloo): barrier + timed steps + barrier, MAX
    over ranks, rank 0 prints the contract line.  No GPU, no kernels: tests only."""
    import torch
    import torch.distributed as dist
    import bench_report
    if world > 1:
        dist.init_process_group("gloo")
    x = np.random.RandomState(rank).random_sample(1 << 15)
    for _ in range(args.warmup):
        np.sort(x)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        np.sort(x)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])
    if rank == 0:
        out = {"metric": "dry-run steps/s", "value": world * args.steps / dt, "unit": "steps/s",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "dry run (CPU, gloo): launcher and contract-line check, no GPU work",
               "config": {"workload": "dry-run", "parallelism": f"{world} gloo ranks"}}
        print(bench_report.contract_line(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def progress(msg):
    """Progress to stderr (stdout carries only the contract line)."""
    print(f"# bench: {msg}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
