"""Per-phase kernel statistics from a rocprofv3 kernel trace (tools/launch_probe.py): the trace
is split into phases at host pauses of more than 10 ms; within a phase, for every kernel name,
the count, the median in-kernel duration (End - Start) and the median gap from the previous
dispatch on the same queue (the dependent kernel boundary; gaps over 50 us — host reads and
syncs — are counted apart), and the phase's wall span.
    python tools/phase_stats.py <run_kernel_trace.csv> [out.json]"""
import csv
import json
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("aiy::", "")
    return name.split("(")[0][:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    phases, cur, last_end = [], [], None
    for r in rows:
        s = int(r["Start_Timestamp"])
        if last_end is not None and s - last_end > 10_000_000:
            phases.append(cur)
            cur = []
        cur.append(r)
        last_end = max(last_end or 0, int(r["End_Timestamp"]))
    if cur:
        phases.append(cur)
    out = []
    for ph in phases:
        st = defaultdict(lambda: {"dur": [], "gap": [], "long_gaps": 0})
        prev_end = None
        for r in ph:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            d = st[short(r["Kernel_Name"])]
            d["dur"].append((e - s) * 1e-3)
            if prev_end is not None:
                g = (s - prev_end) * 1e-3
                if g < 50.0:
                    d["gap"].append(g)
                else:
                    d["long_gaps"] += 1
            prev_end = e
        span = (int(ph[-1]["End_Timestamp"]) - int(ph[0]["Start_Timestamp"])) * 1e-3
        out.append({"span_us": round(span, 1), "kernels": {
            k: {"n": len(v["dur"]), "median_us": round(statistics.median(v["dur"]), 2),
                "min_us": round(min(v["dur"]), 2),
                "median_gap_us": round(statistics.median(v["gap"]), 2) if v["gap"] else None,
                "long_gaps": v["long_gaps"]} for k, v in st.items()}})
    txt = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
