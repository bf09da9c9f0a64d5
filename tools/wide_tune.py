"""A/B of the small-grid one-launch sweep (csrc/bellman_wide_kernels.hip) against the tree
sweep, per geometry (splits S x waves NW), for A1 and the labour sweep at small grids.

    python tools/wide_tune.py [--out gpurun_out/wide_tune.jsonl] [--quick]

Per configuration: the state after `warm` sweeps from v = 0 (r = 0.04), then `n` sweeps from one
C call (aiy_vfi_sweeps_dev / aiy_labor_vfi_sweeps_dev) bracketed by HIP events, median of
`reps` restarts from the same state; and the dominant kernel's own average duration (events
recorded by its dispatch).  Every run's final value function is compared with the tree path's
(bit for bit)."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

# (splits S, waves NW, states per wave SB)
A1_GEOS = [(1, 8, 64), (4, 8, 64), (1, 8, 32), (1, 8, 16), (1, 8, 8), (1, 4, 16), (1, 4, 8),
           (1, 16, 16), (1, 16, 8), (2, 8, 16)]
LAB_GEOS = [(4, 8, 64), (1, 8, 16), (1, 8, 8), (1, 16, 16), (1, 16, 8), (2, 8, 16), (2, 8, 8),
            (4, 8, 16), (1, 4, 8)]


def run(pkg, kind, Na, geo, n=50, warm=10, reps=3, excl=False):
    dev = torch.device("cuda:0")
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    if kind == "a1":
        cal = pkg.calibration.aiyagari(Na=Na)
        Nl = 1
    else:
        cal = pkg.calibration.aiyagari(Na=Na, rho=0.6, sigma_e=0.2)
        Nl = 10
    L = t(0.01 + (1.5 - 0.01) * pkg.calibration.linspace01(10))
    N = cal["N"]
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    ws = pkg.Workspace(N, Na, Nl)
    if excl:
        ws.set_cu_exclusive(True)
    v = [torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(2)]
    idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
    pk, pl, pc = (torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(3))

    def sweeps(m, hint):
        if kind == "a1":
            ws.vfi_sweeps(v[0], v[1], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], m, idx, pk, pc,
                          hint=hint, mode=1)
        else:
            ws.labor_vfi_sweeps(v[0], v[1], a_t, s_t, P_t, L, r, w, cal["beta"], cal["sigma"], 1.0,
                                2.0, m, idx, pk, pl, pc, hint=hint)

    ws.set_wide(0)
    sweeps(warm, None)  # the state: warm sweeps from v = 0 (tree path)
    torch.cuda.synchronize()
    src = v[warm & 1].clone()
    snap = [src.clone(), src.clone(), idx.clone()]
    if geo is None:
        ws.set_wide(0)
    else:
        ws.set_wide(Na, geo[0], geo[1], geo[2])

    def restore():
        v[0].copy_(snap[0]); v[1].copy_(snap[1]); idx.copy_(snap[2])
        torch.cuda.synchronize()

    restore()
    sweeps(4, idx)  # warm-up of this path
    ms = []
    for _ in range(reps):
        restore()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sweeps(n, idx)
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1) / n)
    final = v[n & 1].cpu().numpy()
    restore()
    ws.set_timing(True)
    sweeps(n, idx)
    torch.cuda.synchronize()
    km, nl, _ = ws.timing()
    ws.set_timing(False)
    rec = {"kind": kind, "Na": Na, "geo": geo, "us_per_sweep": sorted(ms)[len(ms) // 2] * 1e3,
           "kernel_us": km / max(nl, 1) * 1e3, "launches": nl}
    if geo is not None:
        # counters (exact evaluations and candidate-level tests per sweep) and a phase trace
        # of one sweep (wave 0 of every block: cycles since entry at each phase mark)
        restore()
        ws.set_timing(False, count=True)
        sweeps(n, idx)
        torch.cuda.synchronize()
        ex, _, _, cand = ws.counters()
        rec["exact_per_sweep"] = ex / n
        rec["tests_per_sweep"] = cand / n
        restore()
        ws.set_timing(False, trace=True)
        sweeps(1, idx)
        torch.cuda.synchronize()
        tr = ws.trace_wide()
        ws.set_timing(False)
        if len(tr):
            nw = geo[1]
            bars = tr[:, 16:16 + 2 * nw:2]
            scr = tr[:, 17:17 + 2 * nw:2]
            rec["wave_bar_med"] = [int(x) for x in np.median(bars, axis=0)]
            rec["wave_screen_med"] = [int(x) for x in np.median(scr, axis=0)]
            rec["wave_screen_work_med"] = [int(x) for x in np.median(scr - bars, axis=0)]
            # per wave: bound-test rounds, entered 8-blocks, voted candidates (words 48 + w);
            # then the same for each block's slowest wave
            wk = tr[:, 48:48 + nw]
            rnd, blk, vot = wk & 0xffff, (wk >> 16) & 0xffff, wk >> 32
            work = scr - bars
            slow = np.argmax(work, axis=1)
            rows = np.arange(len(tr))
            rec["wave_work_med_max"] = {
                "cycles": [int(np.median(work)), int(work.max())],
                "rounds": [float(np.median(rnd)), int(rnd.max())],
                "blocks": [float(np.median(blk)), int(blk.max())],
                "votes": [float(np.median(vot)), int(vot.max())]}
            rec["slowest_wave_med"] = {
                "cycles": int(np.median(work[rows, slow])),
                "rounds": float(np.median(rnd[rows, slow])),
                "blocks": float(np.median(blk[rows, slow])),
                "votes": float(np.median(vot[rows, slow]))}
            ph = {}
            for q, name in enumerate(("table_issued", "table_done", "bar", "screen_wave",
                                      "screen_all", "published", "outputs"), start=3):
                col = tr[:, q]
                col = col[col >= 0]
                if len(col):
                    ph[name] = [int(np.median(col)), int(col.max())]
            rec["phase_cycles_med_max"] = ph
            rec["entry_spread_us"] = float((tr[:, 0].max() - tr[:, 0].min()) / 100.0)
            rec["span_us"] = float((tr[:, 1].max() - tr[:, 0].min()) / 100.0)
            rec["votes_med_max"] = [float(np.median(tr[:, 12])), int(tr[:, 12].max())]
            rec["blocks"] = int(len(tr))
    ws.close()
    return rec, final


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "wide_tune.jsonl"))
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--flags", type=int, default=None, help="AIY_WIDE_FLAGS (A/B)")
    ap.add_argument("--cases", default=None, help="e.g. a1:400,lab:400")
    ap.add_argument("--geos", default=None, help="e.g. 1,8,32;1,8,16 (instead of the lists)")
    ap.add_argument("--excl", action="store_true", help="CU-exclusive sweep workgroups")
    ap.add_argument("--no-tree", action="store_true", help="skip the tree reference runs")
    args = ap.parse_args()
    if args.flags is not None:
        import os
        os.environ["AIY_WIDE_FLAGS"] = str(args.flags)
    pkg = bench.load_pkg()
    cases = [("a1", 400), ("a1", 1000), ("a1", 2048), ("lab", 400), ("lab", 1000), ("lab", 2000)]
    if args.quick:
        cases = [("a1", 400), ("lab", 400)]
    if args.cases:
        cases = [(c.split(":")[0], int(c.split(":")[1])) for c in args.cases.split(",")]
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    with open(args.out, "w") as f:
        for kind, Na in cases:
            ref, vref = run(pkg, kind, Na, None)
            ref["same"] = True
            if not args.no_tree:
                print(json.dumps(ref), flush=True)
                f.write(json.dumps(ref) + "\n")
            geos = A1_GEOS if kind == "a1" else LAB_GEOS
            if args.geos:
                geos = [tuple(int(x) for x in g.split(",")) for g in args.geos.split(";")]
            for geo in geos:
                rec, vv = run(pkg, kind, Na, geo, excl=args.excl)
                rec["excl"] = args.excl
                rec["same"] = bool(np.array_equal(vv, vref))
                rec["speedup_vs_tree"] = ref["us_per_sweep"] / rec["us_per_sweep"]
                print(json.dumps(rec), flush=True)
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
