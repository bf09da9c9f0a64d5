"""Kernel statistics from a rocprofv3 --kernel-trace database (rocpd SQLite, the default
output format on this image): per kernel name, calls, total/avg/min/max duration in us.

    python tools/prof_db_stats.py gpurun_out/.../run_results.db [name-substring ...] [--csv out.csv]
"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        d = (e - s) / 1e3
        a = agg.setdefault(n, [0, 0.0, float("inf"), 0.0])
        a[0] += 1
        a[1] += d
        a[2] = min(a[2], d)
        a[3] = max(a[3], d)
    return sorted(((n, a[0], a[1], a[1] / a[0], a[2], a[3]) for n, a in agg.items()),
                  key=lambda x: -x[2])


def main():
    args = sys.argv[1:]
    out = None
    if "--csv" in args:
        k = args.index("--csv")
        out = args[k + 1]
        del args[k:k + 2]
    db, keys = args[0], args[1:]
    rows = [r for r in stats(db) if not keys or any(k in r[0] for k in keys)]
    for n, calls, tot, avg, mn, mx in rows:
        print(f"{calls:7d} {tot:12.1f} {avg:10.3f} {mn:10.3f} {mx:10.3f}  {n[:120]}")
    if out:
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "MinUs", "MaxUs"])
            w.writerows(rows)


if __name__ == "__main__":
    main()
