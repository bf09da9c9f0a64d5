"""Per-launch SQ/GRBM counter summary of one kernel from tools/pmc.sh passes.

    python tools/pmc_summary.py gpurun_out/pmc [kernel-prefix] [out.json] [skip] [take]

skip/take: per pass, drop the first `skip` launches of the kernel (warm-up sweeps) and keep the
next `take` (default: all) — bench.py's timed window is launches warmup+1 .. warmup+steps.

Derived figures (gfx950; SQ_* cycle counters are in quad-cycles, GRBM_GUI_ACTIVE in cycles
summed over the 8 XCDs — MI355X_MICROARCH.md "Per-instruction cycle constants"):
  waves_per_simd   = SQ_WAVE_CYCLES / (kernel cycles × 1024 SIMDs / 4)   (mean resident waves)
  valu_busy        = SQ_ACTIVE_INST_VALU × 4 / (kernel cycles × 1024)   (fraction of SIMD cycles
                     issuing a VALU instruction, summed over waves)
  wait_frac        = SQ_WAIT_ANY / SQ_WAVE_CYCLES      (wave parked on s_waitcnt / barrier)
  wait_inst_frac   = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stalls: dependency / pipe busy)
  active_frac      = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  valu_per_wave    = SQ_INSTS_VALU / SQ_WAVES, etc.
kernel cycles = GRBM_GUI_ACTIVE / 8 (per XCD).
"""
import collections
import csv
import json
import sys
from pathlib import Path

SIMDS = 1024


def per_launch(root: Path, prefix: str, skip: int = 0, take: int = 0):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in root.rglob("*counter_collection.csv"):
        pas = f.relative_to(root).parts[0]
        for r in csv.DictReader(open(f)):
            if prefix in r["Kernel_Name"]:
                vals[(pas, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    keep = {}
    for pas in {p for p, _ in vals}:
        ids = sorted((int(d) for p, d in vals if p == pas))
        ids = ids[skip:skip + take] if take else ids[skip:]
        keep.update({(pas, str(d)): vals[(pas, str(d))] for d in ids})
    agg = collections.defaultdict(list)
    for (_, _), cs in keep.items():
        for k, v in cs.items():
            agg[k].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    src = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
    prefix = sys.argv[2] if len(sys.argv) > 2 else "bell_tree_kernel"
    out = Path(sys.argv[3]) if len(sys.argv) > 3 else None
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    take = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    c, n = per_launch(src, prefix, skip, take)
    d = {}
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc:
        d["kernel_cycles"] = cyc
        if "SQ_WAVE_CYCLES" in c:
            d["waves_per_simd"] = c["SQ_WAVE_CYCLES"] * 4 / (cyc * SIMDS)
        if "SQ_ACTIVE_INST_VALU" in c:
            d["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * SIMDS)
    wc = c.get("SQ_WAVE_CYCLES")
    if wc:
        for k, name in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_frac"),
                        ("SQ_ACTIVE_INST_ANY", "active_frac"),
                        ("SQ_ACTIVE_INST_VALU", "active_valu_frac")):
            if k in c:
                d[name] = c[k] / wc
    w = c.get("SQ_WAVES")
    if w:
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS",
                  "SQ_INSTS_VMEM_RD", "SQ_INSTS_BRANCH", "SQ_INSTS_VALU_FMA_F64",
                  "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64"):
            if k in c:
                d[k.lower().replace("sq_insts_", "") + "_per_wave"] = c[k] / w
    rec = {"kernel": prefix, "launches": n, "skip": skip, "take": take, "counters_per_launch": c, "derived": d,
           "method": "rocprofv3 --pmc, one pass per counter group (tools/pmc.sh); averages "
                     "over launches; SQ cycle counters x4 (quad-cycles), GRBM_GUI_ACTIVE / 8 XCDs"}
    s = json.dumps(rec, indent=1)
    if out:
        out.write_text(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
