"""Per-dispatch durations of one kernel from a `rocprofv3 --kernel-trace` CSV, in launch order.

    python tools/sweep_times.py <trace-dir> [kernel-prefix] [first] [last]

Prints the count, sum and percentiles of the durations and the first few dispatches, so the
cold sweeps of a solve (the largest) are visible next to the warm ones.  first/last select a
window of the kernel's dispatches (0-based, in order).
"""
import csv
import sys
from pathlib import Path

import numpy as np


def durations(root: Path, prefix: str):
    rows = []
    for f in root.rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith(prefix) or prefix in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    return np.array([d for _, d in rows], dtype=np.float64) / 1e3  # us


def main():
    root = Path(sys.argv[1])
    prefix = sys.argv[2] if len(sys.argv) > 2 else "bell_tree_kernel"
    d = durations(root, prefix)
    if len(sys.argv) > 3:
        lo = int(sys.argv[3])
        hi = int(sys.argv[4]) if len(sys.argv) > 4 else len(d)
        d = d[lo:hi]
    if not len(d):
        raise SystemExit(f"no dispatches of {prefix!r}")
    p = np.percentile(d, [50, 90, 99])
    print(f"{prefix}: n={len(d)} sum={d.sum() / 1e3:.3f} ms mean={d.mean():.1f} us "
          f"p50={p[0]:.1f} p90={p[1]:.1f} p99={p[2]:.1f} max={d.max():.1f} us")
    print("first:", " ".join(f"{x:.0f}" for x in d[:12]))


if __name__ == "__main__":
    main()
