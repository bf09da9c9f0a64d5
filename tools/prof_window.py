"""Average duration of the dominant kernel over bench.py's timed window, from a rocprofv3
kernel trace: bench.py launches it warmup + steps (+3 instrumented) times in that order, and
times launches warmup+1 .. warmup+steps with HIP events.  Usage:
    python tools/prof_window.py <run_kernel_trace.csv> <kernel substring> <warmup> <steps>"""
import csv
import json
import sys


def main():
    path, name, warmup, steps = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]
    win = dur[warmup:warmup + steps]
    print(json.dumps({"kernel": name, "launches": len(dur), "window": [warmup + 1, warmup + steps],
                      "avg_ms_window": sum(win) / len(win), "min_ms": min(win), "max_ms": max(win),
                      "avg_ms_all": sum(dur) / len(dur)}))


if __name__ == "__main__":
    main()
