"""Reads the kernel + HIP-API traces of tools/ge_concurrency.py (tools/exp/r06_g08.sh) for 1, 2
and 4 concurrent warm solves: per stream, the sweep kernels' durations, the gaps between
consecutive kernels of one stream, how many other kernels were running when each started, the
queues used, and the host-side launch calls' durations per thread.  VERDICT r5 item 7."""
import csv
import json
import sys
from collections import defaultdict

import numpy as np


def load(tag, root="gpurun_out/r06_g08"):
    K = list(csv.DictReader(open(f"{root}/t{tag}/run_kernel_trace.csv")))
    H = list(csv.DictReader(open(f"{root}/t{tag}/run_hip_api_trace.csv")))
    return K, H


def analyse(tag):
    K, H = load(tag)
    sw = [k for k in K if "bell_wide" in k["Kernel_Name"] or "bell_tree" in k["Kernel_Name"]
          or "bell_table" in k["Kernel_Name"]]
    # the timed reps: the last 5 x (solves) of the run — keep kernels after the warm-up solve
    # (the first solve's kernels run alone before the slots are created)
    sw.sort(key=lambda k: int(k["Start_Timestamp"]))
    t_all = np.array([[int(k["Start_Timestamp"]), int(k["End_Timestamp"])] for k in sw])
    # drop the warm start solve (first 1/ (5n+1) of the sweeps, approximately: before the
    # first time two streams are active... simpler: skip kernels of the first stream seen)
    first_stream = sw[0]["Stream_Id"]
    body = [k for k in sw if k["Stream_Id"] != first_stream] or sw
    by = defaultdict(list)
    for k in body:
        by[k["Stream_Id"]].append(k)
    out = {"kernels": len(body), "streams": len(by),
           "queues": sorted({k["Queue_Id"] for k in body})}
    durs, gaps, conc = [], [], []
    ivals = np.array([[int(k["Start_Timestamp"]), int(k["End_Timestamp"])] for k in body])
    for s, ks in by.items():
        st = np.array([int(k["Start_Timestamp"]) for k in ks])
        en = np.array([int(k["End_Timestamp"]) for k in ks])
        durs += list((en - st) / 1e3)
        g = (st[1:] - en[:-1]) / 1e3
        gaps += list(g[g < 200])  # within a solve (not between reps)
    for a, b in ivals:
        conc.append(int(((ivals[:, 0] < a) & (ivals[:, 1] > a)).sum()))
    q = lambda x: {"p10": float(np.percentile(x, 10)), "p50": float(np.median(x)),
                   "p90": float(np.percentile(x, 90)), "mean": float(np.mean(x))}
    out["kernel_us"] = q(durs)
    out["gap_us"] = q(gaps)
    out["running_at_start"] = q(conc)
    out["queue_of_stream"] = {s: sorted({k["Queue_Id"] for k in ks}) for s, ks in by.items()}
    # host side: launch API durations per thread
    L = [h for h in H if "Launch" in h["Function"]]
    ld = defaultdict(list)
    for h in L:
        ld[h["Thread_Id"]].append((int(h["End_Timestamp"]) - int(h["Start_Timestamp"])) / 1e3)
    allL = [x for v in ld.values() for x in v]
    out["launch_api_us"] = q(allL) if allL else None
    other = defaultdict(list)
    for h in H:
        if h["Function"] in ("hipMemcpyAsync", "hipEventQuery", "hipEventRecord",
                             "hipStreamSynchronize", "hipMemcpyWithStream"):
            other[h["Function"]].append((int(h["End_Timestamp"]) - int(h["Start_Timestamp"])) / 1e3)
    out["api_us"] = {f: q(v) | {"n": len(v)} for f, v in other.items()}
    return out


if __name__ == "__main__":
    res = {t: analyse(t) for t in sys.argv[1:] or ["1", "2", "4"]}
    print(json.dumps(res, indent=1))
