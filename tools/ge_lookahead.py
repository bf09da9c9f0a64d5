"""Wall time of the GE bisection at Aiyagari_VFI.m's defaults (configs[0]) with the speculative
driver at lookahead 1, 2, 3 (ge.aiyagari_vfi_overlapped), median of 5, and the sequential
driver; every trace must equal the sequential one."""
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

import torch  # noqa: E402

torch.cuda.set_device(0)  # torch's context first (as bench.py), then the library's calls
pkg = bench.load_pkg()
pkg.ge.aiyagari_vfi(max_iter=5)
seq = pkg.ge.aiyagari_vfi()
t0 = time.perf_counter()
seq = pkg.ge.aiyagari_vfi()
out = {"sequential_s": time.perf_counter() - t0}
for la in (1, 2, 3, 4):
    pkg.ge.aiyagari_vfi_overlapped(max_iter=5, lookahead=la)
    ws = []
    same = True
    for _ in range(5):
        t0 = time.perf_counter()
        o = pkg.ge.aiyagari_vfi_overlapped(lookahead=la)
        ws.append(time.perf_counter() - t0)
        same = same and o["r_history"] == seq["r_history"] and o["iters"] == seq["iters"]
        if not same:
            print("DIFF", la, o["r_history"], seq["r_history"], o["iters"], seq["iters"], flush=True)
    out[f"lookahead_{la}"] = {"median_s": sorted(ws)[2], "min_s": min(ws), "same_trace": same,
                              "solve_slots": o["solves"]}
print(json.dumps(out), flush=True)
for la in (2,):
    o = pkg.ge.aiyagari_vfi_overlapped(lookahead=la)
    print(f"timeline lookahead {la}: wall {o['wall_s'] * 1e3:.1f} ms")
    for k, r, j, a, b, it in o["timeline"]:
        print(f"  {k:5s} j={j:2d} r={r if r is None else round(r, 6)} {a * 1e3:7.2f} -> {b * 1e3:7.2f} ms"
              f" ({(b - a) * 1e3:5.2f}) it={it}")
