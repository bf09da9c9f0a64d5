"""The measurement legs bench.py adds to its JSON line besides the headline:

  cpu_info()        host CPU model, nproc, the CPU share this job may use
  labor_leg()       D4: A3 labour VFI sweeps (Aiyagari_Endogenous_Labor_VFI.m:69-112)
  egm_leg()         D4: A4/A5 EGM steps (Aiyagari_EGM.m:74-110, ..._Labor_EGM.m:67-107)
  batch_leg()       D5: the batched multi-rate solve (config 4's per-GPU share) vs one rate
  dist_leg()        A10: histogram pushes at Na = 20,000 (HBM roofline)
  ge_batch_leg()    D5: config 4's multisection GE (64 candidates / round over the ranks)
  ks_cpu_baseline() D6: the C restatement's Krusell-Smith evals/s (bounded sample)

Every GPU leg times work whose inputs are already resident in HBM; every CPU figure is the C
restatement (oracle/liborc.so — the checker, timed as the CPU baseline, never the product).
"""
from __future__ import annotations

import os
import platform
import time

import numpy as np

PEAK_FP64_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0
FLOPS_PER_TEST = 7
FLOPS_PER_CANDIDATE = 8
FLOPS_PER_LABOR_CANDIDATE = 9  # 8 + the disutility term


def cpu_info():
    model = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    share = omp if omp > 0 else aff
    return {"model": model, "nproc": os.cpu_count(), "affinity": aff,
            "omp_num_threads": omp or None, "threads_all": share,
            "note": "all-cores figures use the CPU share of this job (OMP_NUM_THREADS when set: "
                    "the GPU box allots 16 host CPUs per GPU), 1-core figures one thread"}


def gpu_clock(dev_index=0):
    """The active core clock level of the benched GPU from sysfs (SURVEY D7 asks the clocks to
    be noted): the amdgpu driver marks the current pp_dpm_sclk level with '*'; the card is
    matched by PCI bus (torch device properties).  None when not readable."""
    import glob
    try:
        import torch
        bus = getattr(torch.cuda.get_device_properties(dev_index), "pci_bus_id", None)
    except Exception:
        bus = None
    if bus is None:  # cannot tell which card is ours
        return None
    for f in sorted(glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk")):
        try:
            pci = os.path.basename(os.path.realpath(os.path.dirname(f)))  # 0000:BB:DD.F
            if int(pci.split(":")[1], 16) != int(bus):
                continue
            cur = [ln.strip() for ln in open(f) if ln.strip().endswith("*")]
        except (OSError, ValueError, IndexError):
            continue
        if cur:
            return {"pci": pci, "sclk": cur[0]}
    return None


def _time_cpu(fn, threads):
    from oracle import corc
    corc.num_threads(threads)
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def _events(torch):
    return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)


def _median(x):
    x = sorted(x)
    return x[len(x) // 2]


# ----------------------------------------------------------------------------------- D4 labour
def labor_leg(pkg, dev, Na, steps=10, warmup=5, reps=5, cpu=True, cpu_threads=1, variant=-1):
    """A3 at the labour script's calibration (rho .6, sigma_e .2, psi 1, eta 2, Nl = 10): device
    tier sweeps from v = 0 (warm-up sweeps, then `steps` timed, median of `reps` restarts from the
    same state).  Unit: Na·Na'·Nl·Nz candidates per sweep."""
    import torch
    from oracle import corc
    from oracle import np_oracle as no
    cal = pkg.calibration.aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
    N = cal["N"]
    L = 0.01 + (1.5 - 0.01) * pkg.calibration.linspace01(10)
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t, L_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"]), t(L)
    ws = pkg.Workspace(N, Na, 10)
    if variant >= 0:
        ws.set_variant(variant)
    v = [torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(2)]
    lin = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    pk, pl, pc = (torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(3))
    cur = 0

    def sweep(first=False):
        nonlocal cur
        ws.labor_vfi_sweep(v[cur], a_t, s_t, P_t, L_t, r, w, cal["beta"], cal["sigma"], 1.0, 2.0,
                           v[1 - cur], lin, pk, pl, pc, hint=None if first else lin)
        cur = 1 - cur

    def block():  # `steps` sweeps from one C call (aiy_labor_vfi_sweeps_dev), hint = lin
        nonlocal cur
        ws.labor_vfi_sweeps(v[cur], v[1 - cur], a_t, s_t, P_t, L_t, r, w, cal["beta"],
                            cal["sigma"], 1.0, 2.0, steps, lin, pk, pl, pc, hint=lin)
        cur ^= steps & 1

    for q in range(warmup):
        sweep(first=(q == 0))
    torch.cuda.synchronize()
    snap = [x.clone() for x in (v[0], v[1], lin)]
    snap_cur = cur
    ms, kern = [], []
    for rep in range(reps + 1):  # the last block: HIP events around every kernel launch
        v[0].copy_(snap[0]); v[1].copy_(snap[1]); lin.copy_(snap[2])
        cur = snap_cur
        torch.cuda.synchronize()
        ev = rep == reps
        ws.set_timing(ev)
        e0, e1 = _events(torch)
        e0.record()
        block()
        e1.record()
        torch.cuda.synchronize()
        if ev:
            km, n, _ = ws.timing()
            kern.append(km / max(n, 1))
        else:
            ms.append(e0.elapsed_time(e1) / steps)
        ws.set_timing(False)
    # executed work of the same sweeps (instrumented pass, untimed)
    v[0].copy_(snap[0]); v[1].copy_(snap[1]); lin.copy_(snap[2])
    cur = snap_cur
    ws.set_timing(False, count=True)
    block()
    torch.cuda.synchronize()
    ex, sup, blk, cand = ws.counters()
    ws.set_timing(False)
    per_sweep = N * Na * Na * 10
    step_ms, kern_ms = _median(ms), _median(kern)
    executed = (FLOPS_PER_TEST * (sup + blk + cand) + FLOPS_PER_LABOR_CANDIDATE * ex) / steps
    out = {"workload": f"Aiyagari_Endogenous_Labor_VFI sweeps, Na={Na} Nz={N} Nl=10 (sweeps "
                       f"{warmup + 1}..{warmup + steps} from v=0, one aiy_labor_vfi_sweeps_dev "
                       f"call per timed block), device tier",
           "value": per_sweep / (step_ms * 1e-3), "unit": "evals/s",
           "ms_per_sweep": step_ms, "kernel_ms": kern_ms, "repeats": reps,
           "roofline": {"bound": "valu", "achieved": executed / (kern_ms * 1e-3) / 1e12,
                        "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                        "frac": executed / (kern_ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                        "basis": f"executed work: {FLOPS_PER_TEST} flops per bound/candidate test, "
                                 f"{FLOPS_PER_LABOR_CANDIDATE} per exact evaluation (counted), "
                                 f"{executed:.3g} flops/sweep",
                        "effective_tflops_d4": FLOPS_PER_LABOR_CANDIDATE * per_sweep
                                               / (kern_ms * 1e-3) / 1e12,
                        "effective_basis": f"SURVEY D4: 9 flops x Na*Na'*Nl*Nz = {per_sweep} "
                                           f"candidates of the exhaustive scan per sweep"}}
    if cpu:  # the C restatement's exhaustive labour sweep on the same state, 1 core and all
        V = snap[snap_cur].cpu().numpy()
        reps_cpu = max(1, int(2e8 // per_sweep))
        cpu_out = {}
        row_1core = per_sweep > 4e9   # bounded sample: one core gets one productivity row
        k = N // 2
        EV = (cal["P"][k] @ V)[None, :]   # row k's continuation, so P = [[1]] reproduces its work
        for th in sorted({1, cpu_threads}):
            if th == 1 and row_1core:
                dt = _time_cpu(lambda: corc.labor_vfi_sweep(EV, cal["a_grid"], cal["s"][k:k + 1],
                                                            np.ones((1, 1)), L, r, w, cal["beta"],
                                                            cal["sigma"], 1.0, 2.0), th)
                cpu_out[f"cores_{th}"] = {"value": per_sweep / N / dt, "seconds": dt,
                                          "sample": f"productivity row {k} of {N} (Na*Na'*Nl "
                                                    f"candidates, P = [[1]] on row {k}'s EV)"}
                continue
            dt = _time_cpu(lambda: [corc.labor_vfi_sweep(V, cal["a_grid"], cal["s"], cal["P"], L, r,
                                                         w, cal["beta"], cal["sigma"], 1.0, 2.0)
                                    for _ in range(reps_cpu)], th)
            cpu_out[f"cores_{th}"] = {"value": reps_cpu * per_sweep / dt, "seconds": dt}
        out["cpu_baseline"] = {"unit": "evals/s", "kind": "port", **cpu_out,
                               "value": cpu_out[f"cores_{cpu_threads}"]["value"],
                               "cores": cpu_threads,
                               "sample": f"{reps_cpu} exhaustive labour sweep(s) at Na={Na} "
                                         f"(oracle/aiy_oracle.c)"
                                         + ("; the 1-core figure on one productivity row"
                                            if row_1core else "")}
    return out


# ----------------------------------------------------------------------------------- D4 EGM
def egm_leg(pkg, dev, Na, labor=False, steps=50, reps=5, cpu_threads=1, variant=-1):
    """A4 (or A5) steps on device at r = 0.04 from the script's initial consumption guess
    (Aiyagari_EGM.m:64); unit = one (a, z) state per iteration; HBM roofline with the
    algorithmic bytes of SURVEY D4 (24 B: c in, c_next and policy_k out; +8 for policy_l)."""
    import torch
    from oracle import corc
    cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
    N = cal["N"]
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    a = cal["a_grid"]
    pc0 = np.tile(((1 + r) * a + w * np.mean(cal["s"]))[None, :], (N, 1))  # [N][Na]
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t = t(a), t(cal["s"]), t(cal["P"])
    ws = pkg.Workspace(N, Na)
    if variant >= 0:  # (EGM knob bit 18: the two-launch step even on small grids — A/B only)
        ws.set_variant(variant)
    c = [t(pc0), torch.zeros((N, Na), dtype=torch.float64, device=dev)]
    pk = torch.zeros_like(c[0])
    pl = torch.zeros_like(c[0]) if labor else None
    cur = 0

    def step():
        nonlocal cur
        pkg.egm_step_dev(ws, c[cur], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], cal["amin"],
                         c[1 - cur], pk, labor=labor, phi=1.0, theta=1.0, policy_l=pl)
        cur = 1 - cur

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        e0, e1 = _events(torch)
        e0.record()
        for _ in range(steps):
            step()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1) / steps)
    single_ms = _median(ms)
    # the device-tier solve loop (aiy_egm_solve_dev: speculative batches of steps; for
    # Na > 1,024 each step is ONE chained launch, interp1 of t + the RHS of t+1): `steps`
    # steps at tol = 0 from the same start, wall per step (host reads of the batches included)
    ws2 = pkg.Workspace(N, Na)
    if variant >= 0:
        ws2.set_variant(variant)
    c2 = t(pc0)
    pk2 = torch.zeros_like(c2)
    pl2 = torch.zeros_like(c2) if labor else None
    solve_dev = lambda n: pkg.egm_solve_dev(ws2, c2, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"],
                                            cal["amin"], 0.0, n, pk2, labor=labor, phi=1.0,
                                            theta=1.0, policy_l=pl2)
    solve_dev(20)
    sms = []
    for _ in range(reps):
        c2.copy_(t(pc0))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        solve_dev(200)
        torch.cuda.synchronize()
        sms.append((time.perf_counter() - t0) * 1e3 / 200)
    step_ms = _median(sms)
    # the chained launch's own duration (events recorded by its dispatch, no gaps): one more
    # pass of the same steps with timing on; Na <= 1,024 runs the fused kernel (not timed)
    ws2.set_timing(True)
    c2.copy_(t(pc0))
    solve_dev(200)
    torch.cuda.synchronize()
    km, nl, _ = ws2.timing()
    ws2.set_timing(False)
    kern_ms = km / nl if nl else None
    bps = 32 if labor else 24
    states = N * Na
    gbs_step = states * bps / (step_ms * 1e-3) / 1e9
    gbs = states * bps / ((kern_ms or step_ms) * 1e-3) / 1e9
    pcs = c[cur].cpu().numpy()
    solve = corc.labor_egm_step if labor else corc.egm_step
    args = ((1.0, 1.0, cal["amin"]) if labor else (cal["amin"],))
    reps_cpu = max(1, int(2e6 // states))
    cpu_out = {}
    for th in sorted({1, cpu_threads}):
        dt = _time_cpu(lambda: [solve(pcs, a, cal["s"], cal["P"], r, w, cal["beta"], cal["sigma"],
                                      *args) for _ in range(reps_cpu)], th)
        cpu_out[f"cores_{th}"] = {"value": reps_cpu * states / dt, "seconds": dt}
    name = "Aiyagari_Endogenous_Labor_EGM" if labor else "Aiyagari_EGM"
    # the whole solve through the host tier (the MEX path: speculative batches of steps between
    # dist reads, policy arrays copied in and out), to tol = 1e-5 from the same start
    pc_host = pc0.T.copy()  # Na x N, the script's layout
    walls, iters = [], 0
    for _ in range(3):
        t0 = time.perf_counter()
        if labor:
            R = pkg.labor_egm_solve(pc_host, a, cal["s"], cal["P"], r, w, cal["beta"], cal["sigma"],
                                    1.0, 1.0, cal["amin"], 1e-5, 1000)
        else:
            R = pkg.egm_solve(pc_host, a, cal["s"], cal["P"], r, w, cal["beta"], cal["sigma"],
                              cal["amin"], 1e-5, 1000)
        walls.append(time.perf_counter() - t0)
        iters = R["iters"]
    solve_s = _median(walls)
    if Na <= 1024 and not (variant >= 0 and variant & (1 << 18)):
        path = "1 launch per step: egm_fused_kernel, a workgroup per z-state)"
    elif Na > 1024 and not (variant >= 0 and variant & (1 << 19)):
        path = ("1 launch per step in the solve loop: egm_chain_kernel, interp1 of step t + "
                "the Euler RHS of step t+1 on the same tiles)")
    else:
        path = "2 launches per step: Euler RHS, interp1 inversion)"
    return {"workload": f"{name} steps, Na={Na} Nz={N} Rouwenhorst, device-tier solve loop "
                        f"(aiy_egm_solve_dev, 200 steps at tol = 0; " + path,
            "single_step_dev": {"us_per_step": single_ms * 1e3,
                                "path": "aiy_egm_step_dev one step at a time (the two-launch step "
                                        "for Na > 1,024, the fused launch below), Python-issued"},
            "solve": {"iters": iters, "wall_ms": solve_s * 1e3,
                      "us_per_iteration": solve_s / max(iters, 1) * 1e6,
                      "path": "host tier (aiy_egm_solve / aiy_labor_egm_solve): speculative "
                              "batches of up to 16 steps per dist read, H2D/D2H included"},
            "value": states / (step_ms * 1e-3), "unit": "state-iterations/s",
            "us_per_step": step_ms * 1e3, "repeats": reps,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS,
                         "kernel": "egm_chain_kernel" if kern_ms else "whole step (fused kernel)",
                         "kernel_avg_ms": kern_ms, "launches": nl,
                         "frac_per_step": gbs_step / HBM_PEAK_GBS,
                         "basis": f"{bps} B algorithmic per state-iteration x {states} states / "
                                  + ("the chained launch's dispatch-recorded duration (one "
                                     "launch per step)" if kern_ms else "the step time")},
            "cpu_baseline": {"unit": "state-iterations/s", "kind": "port", **cpu_out,
                             "sample": f"{reps_cpu} EGM step(s) at Na={Na} (oracle/aiy_oracle.c)"}}


# ----------------------------------------------------------------------------------- D5 batch
def batch_leg(pkg, dev, Na=20000, C=8, sweeps=25):
    """The per-GPU share of config 4 at the headline grid: C rates solved as one batch (one
    table + one tree launch per sweep over all C) against one rate alone, both running exactly
    `sweeps` sweeps from v = 0 (tol = 0: no early stop).  Unit: Na·Na'·Nz per candidate-sweep.
    Roofline: the batched tree launch's executed work (bound/candidate tests and exact
    evaluations counted by the instrumented instantiation over the same sweeps, all C
    candidates) ÷ its average launch duration (HIP events around every tree launch).  The same
    path is pinned bit for bit by tests/test_pinned_gpu.py::test_batch_config4_share_sweep25."""
    import torch
    cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
    N = cal["N"]
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    rs = list(np.linspace(-0.03, 0.035, C))
    w = [pkg.calibration.wage(r, cal["alpha"], cal["delta"]) for r in rs]
    ws = pkg.Workspace(N, Na)
    res = {}
    bufs = {}
    for n in (C, 1):
        va = torch.zeros((n, N, Na), dtype=torch.float64, device=dev)
        vb = torch.zeros_like(va)
        idx = torch.zeros((n, N, Na), dtype=torch.int32, device=dev)
        pk = torch.zeros_like(va)
        pc = torch.zeros_like(va)
        bufs[n] = (va, vb, idx, pk, pc)
        pkg.vfi.solve_batch_dev(ws, rs[:n], w[:n], va, vb, a_t, s_t, P_t, cal["beta"],
                                cal["sigma"], 0.0, 3, idx, pk, pc)  # warm-up
        ms = []
        for _ in range(3):
            va.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pkg.vfi.solve_batch_dev(ws, rs[:n], w[:n], va, vb, a_t, s_t, P_t, cal["beta"],
                                    cal["sigma"], 0.0, sweeps, idx, pk, pc)
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
        res[n] = _median(ms)
    va, vb, idx, pk, pc = bufs[C]

    def run(flags):
        ws.set_timing(**flags)
        va.zero_()
        pkg.vfi.solve_batch_dev(ws, rs, w, va, vb, a_t, s_t, P_t, cal["beta"], cal["sigma"], 0.0,
                                sweeps, idx, pk, pc)
        torch.cuda.synchronize()

    run({"on": True})
    km, nl, _ = ws.timing()
    kern_ms = km / max(nl, 1)
    run({"on": False, "count": True})
    ex, sup, blk, cand = ws.counters()
    ws.set_timing(False)
    executed = (FLOPS_PER_TEST * (sup + blk + cand) + FLOPS_PER_CANDIDATE * ex) / sweeps
    ach = executed / (kern_ms * 1e-3) / 1e12
    per = N * Na * Na * sweeps
    return {"workload": f"Aiyagari VFI at Na={Na} Nz={N} Rouwenhorst: {C} candidate rates as one "
                        f"batched solve, {sweeps} sweeps each from v=0 (config 4 per-GPU share)",
            "value": C * per / (res[C] * 1e-3), "unit": "evals/s",
            "batch_ms": res[C], "single_rate_ms": res[1],
            "single_rate_evals_per_s": per / (res[1] * 1e-3),
            "speedup_vs_sequential_rates": C * res[1] / res[C],
            "roofline": {"bound": "valu", "achieved": ach, "peak": PEAK_FP64_TFLOPS,
                         "unit": "TFLOP/s", "frac": ach / PEAK_FP64_TFLOPS,
                         "kernel": "bell_tree_kernel (batched, C candidates per launch)",
                         "kernel_avg_ms": kern_ms, "launches": nl,
                         "basis": f"executed work over all {C} candidates: {FLOPS_PER_TEST} flops "
                                  f"per bound/candidate test, {FLOPS_PER_CANDIDATE} per exact "
                                  f"evaluation (instrumented pass of the same {sweeps} sweeps): "
                                  f"{executed:.3g} flops per launch",
                         "tests_per_launch": {"exact": ex / sweeps, "superblock": sup / sweeps,
                                              "block": blk / sweeps, "candidate": cand / sweeps},
                         "effective_tflops_d3": FLOPS_PER_CANDIDATE * C * N * Na * Na
                                                / (kern_ms * 1e-3) / 1e12},
            "parity": "tests/test_pinned_gpu.py::test_batch_config4_share_sweep25_bitwise"}


# ----------------------------------------------------------------------------------- A10 dist
DIST_BYTES_PER_STATE = 20  # λ in (8), run offset (4), λ' out (8) per state and push


def dist_leg(pkg, dev, Na=20000, pushes=320, cpu_pushes=600, cpu_threads=1):
    """A10 histogram pushes (csrc/dist_kernels.hip dist_push_kernel) on the config-2 policy
    (Na = 20,000, Rouwenhorst, r = 0.04, the device VFI solve's argmax): `pushes` pushes from
    the uniform distribution through aiy_dist_stationary_dev with tol = 0 (plan once, batches of
    32 pushes per read), then the solve to max|Δλ| < 1e-13.  Unit: pushes/s over all N·Na
    states; HBM roofline on the algorithmic 20 B per state and push.  CPU: the C restatement's
    push (orc_dist_stationary, sequential), one core."""
    import torch
    from oracle import corc
    cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
    N = cal["N"]
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    vws = pkg.Workspace(N, Na)
    va = torch.zeros((N, Na), dtype=torch.float64, device=dev)
    vb = torch.zeros_like(va)
    idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    iters, _ = vws.vfi_solve(va, vb, a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], 1e-5, 1000,
                             idx)
    vws.close()
    lam0 = torch.full((N, Na), 1.0 / (N * Na), dtype=torch.float64, device=dev)
    out = torch.empty_like(lam0)
    K = torch.zeros(1, dtype=torch.float64, device=dev)
    ws = pkg.Workspace(N, Na)
    run = lambda n, tol=0.0: pkg.dist_stationary_dev(ws, lam0, a_t, P_t, out, policy_idx=idx,
                                                     tol=tol, max_iter=n, k_supply=K)
    run(64)
    torch.cuda.synchronize()
    ms = []
    for _ in range(5):
        t0 = time.perf_counter()
        run(pushes)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
    wall_ms = _median(ms)
    ws.set_timing(True)
    run(pushes)
    torch.cuda.synchronize()
    km, nl, _ = ws.timing()
    ws.set_timing(False)
    kern_ms = km / max(nl, 1)
    t0 = time.perf_counter()
    it_tol, d_tol = run(100000, 1e-13)
    torch.cuda.synchronize()
    tol_ms = (time.perf_counter() - t0) * 1e3
    states = N * Na
    gbs = DIST_BYTES_PER_STATE * states / (kern_ms * 1e-3) / 1e9
    idx_np = idx.cpu().numpy()
    lam_np = lam0.cpu().numpy()
    cpu_dt = {}
    for th in sorted({1, cpu_threads}):  # OpenMP over productivity rows (same sum order)
        cpu_dt[th] = _time_cpu(lambda: corc.dist_stationary(lam_np, cal["a_grid"], cal["P"],
                                                            idx=idx_np, tol=0.0,
                                                            max_iter=cpu_pushes), th)
    dt = cpu_dt[cpu_threads]
    return {"workload": f"A10 histogram pushes, Na={Na} Nz={N} Rouwenhorst, policy = argmax of "
                        f"the r=0.04 VFI solve ({iters} sweeps); {pushes} pushes from uniform "
                        f"lambda, device tier (aiy_dist_stationary_dev, tol=0)",
            "value": pushes / (wall_ms * 1e-3), "unit": "pushes/s",
            "states_per_s": pushes * states / (wall_ms * 1e-3),
            "us_per_push": wall_ms * 1e3 / pushes,
            "kernel_us": kern_ms * 1e3,  # events recorded by the push's own dispatch (no gaps)
            "to_tol": {"tol": 1e-13, "pushes": it_tol, "dist": d_tol, "wall_ms": tol_ms,
                       "K": float(K[0])},
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "kernel": "dist_push_kernel<false>",
                         "kernel_avg_ms": kern_ms, "launches": nl,
                         "basis": f"{DIST_BYTES_PER_STATE} B algorithmic per state and push "
                                  f"(lambda in, run offset, lambda' out) x {states} states"},
            "cpu_baseline": {"value": cpu_pushes / dt, "unit": "pushes/s", "cores": cpu_threads,
                             "kind": "port", "states_per_s": cpu_pushes * states / dt,
                             "one_core": cpu_pushes / cpu_dt[1],
                             "sample": f"{cpu_pushes} pushes of orc_dist_stationary (scatter in "
                                       f"source order, OpenMP over productivity rows, "
                                       f"oracle/aiy_oracle.c) on the same policy: {dt:.2f} s on "
                                       f"{cpu_threads} threads, {cpu_dt[1]:.2f} s on 1"}}


def ge_batch_leg(pkg, world, rank, dev, Na=400, levels=6, sequential=True):
    """Config 4: Aiyagari_VFI.m's GE (:131-206) as multisection rounds of the bisection tree
    (2^levels - 1 candidates per round, round-robin over the ranks, one batched device call per
    rank and round, one all-gather of (K_s, K_d) per round).  Wall time to the final r, max over
    ranks.  Every rank must call it."""
    import torch
    import torch.distributed as dist
    gb = pkg.ge_batch
    gb.aiyagari_vfi_multisection(Na=Na, levels=1, rank=0, world=1)  # warm-up (this rank)
    samples = []
    A = None
    for _ in range(3):
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        A = gb.aiyagari_vfi_multisection(Na=Na, levels=levels, rank=rank, world=world)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        samples.append(time.perf_counter() - t0)
    dt = _median(samples)
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt[0])
    cal = pkg.calibration.aiyagari(Na=Na)
    out = {"workload": f"Aiyagari_VFI.m GE at Na={Na} (Tauchen N=7, MC T=1e4): multisection, "
                       f"{2 ** levels - 1} candidates per round, warm start from the r0 = 0.04 "
                       f"solution, batched device evaluation",
           "value": dt, "unit": "s to equilibrium r", "higher_is_better": False,
           "n_gpus": world, "r": A.r, "steps": len(A.r_history), "rounds": A.rounds,
           "candidates": A.candidates, "candidates_per_s": A.candidates / dt,
           "parallelism": f"{world} ranks, candidates round-robin, one all-gather per round"}
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden",
                             "a11_ge_vfi_defaults.npz"))
    out["r_equals_reference_trace"] = A.r == float(g["r_final"]) and \
        A.r_history == [float(x) for x in g["r_history"]]
    if world == 1 and sequential:
        w0 = pkg.calibration.wage(0.04, cal["alpha"], cal["delta"])
        t1 = time.perf_counter()
        v0 = pkg.vfi_solve(np.zeros((cal["N"], Na)), cal["a_grid"], cal["s"], cal["P"], 0.04, w0,
                           cal["beta"], cal["sigma"])["v_old"]
        S = gb.bisection(gb.hip_vfi_evaluator(cal, v0), -0.05, 1 / cal["beta"] - 1)
        out["sequential_bisection_s"] = time.perf_counter() - t1
        out["sequential_identical_trace"] = S.r_history == A.r_history
    return out


# ----------------------------------------------------------------------------------- D6 KS CPU
def ks_cpu_baseline(pkg, nk=32768, nK=4, howard=2, threads=1):
    """The C restatement's Howard sweeps (Krusell_Smith_VFI.m:172-192) on a bounded slice of
    the scaling grid (k = nk, K = nK of the [30, 50] range): bellman_value evals/s, 1 core and
    the job's share."""
    from oracle import corc
    kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=nk, K_size=nK)
    B = np.array([0.1, 0.97, 0.08, 0.975])
    prm = pkg.ks_params()
    p = corc.ks_params(beta=prm[0], alpha=prm[1], delta=prm[2], k_min=prm[3], k_max=prm[4],
                       ug=prm[5], ub=prm[6], l_bar=prm[7], mu=prm[8], z_grid=(prm[9], prm[10]),
                       eps_grid=(prm[11], prm[12]))
    ko = np.ones_like(V0)
    nodes = nk * nK * 4
    out = {}
    for th in sorted({1, threads}):
        dt = _time_cpu(lambda: corc.ks_howard(p, kg, Kg, V0, ko, B, P, howard), th)
        out[f"cores_{th}"] = {"value": nodes * howard / dt, "seconds": dt}
    return {"unit": "evals/s", "kind": "port", **out,
            "sample": f"{howard} Howard sweeps at k={nk}, K={nK}, S=4 ({nodes} nodes; "
                      f"oracle/aiy_oracle.c, the scaling grid's first {nK} K columns)"}
