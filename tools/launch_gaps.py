"""Launch-floor attribution from a rocprofv3 kernel trace: for every
kernel whose name contains one of the given substrings, the median in-kernel duration
(End - Start) and the median gap from the previous dispatch on the same queue to its start
(the dependent kernel boundary).  The boundary of a back-to-back dependent chain is what the
guide's `boundary` row prices (1.45 us between trivial kernels); everything else is inside the
kernel.
    python tools/launch_gaps.py <run_kernel_trace.csv> <substring> [<substring> ...]"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def main():
    path, names = sys.argv[1], sys.argv[2:]
    rows = list(csv.DictReader(open(path)))
    by_q = defaultdict(list)
    for r in rows:
        by_q[(r["Agent_Id"], r["Queue_Id"])].append(r)
    stats = defaultdict(lambda: {"dur": [], "gap": [], "prev": defaultdict(int)})
    for q, rs in by_q.items():
        rs.sort(key=lambda r: int(r["Start_Timestamp"]))
        for a, b in zip(rs, rs[1:]):
            nm = b["Kernel_Name"]
            key = next((n for n in names if n in nm), None)
            if key is None:
                continue
            s = stats[key]
            s["dur"].append((int(b["End_Timestamp"]) - int(b["Start_Timestamp"])) * 1e-3)
            s["gap"].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) * 1e-3)
            s["prev"][a["Kernel_Name"][:60]] += 1
    out = {}
    for k, s in stats.items():
        gaps = [g for g in s["gap"] if g < 50.0]  # drop host-side pauses (syncs, reads)
        out[k] = {"n": len(s["dur"]), "median_us": statistics.median(s["dur"]),
                  "min_us": min(s["dur"]),
                  "median_gap_us": statistics.median(gaps) if gaps else None,
                  "gap_n": len(gaps), "prev": dict(s["prev"])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
