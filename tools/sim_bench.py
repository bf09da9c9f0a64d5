"""A9 Monte-Carlo chain alone (tuning aid): device-tier K supply at the scripts' size (Na = 400,
N = 7, T = 10^4, the r = 0.04 VFI policy) and at Na = 20,000, HIP events over 20 calls.
    python tools/sim_bench.py"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

pkg = bench.load_pkg()
dev = torch.device("cuda:0")
t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
import os
modes = [int(x) for x in os.environ.get("SIM_MODES", "-1,0").split(",")]
for Na, mode in [(n, m) for n in (400, 900, 1900, 20000) for m in modes]:
    cal = pkg.calibration.aiyagari(Na=Na)
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    R = pkg.vfi_solve(np.zeros((cal["N"], Na)), cal["a_grid"], cal["s"], cal["P"], r, w,
                      cal["beta"], cal["sigma"], 1e-5, 1000)
    ws = pkg.Workspace(cal["N"], Na)
    ws.set_sim(mode)
    U = t(np.random.default_rng(0).random(9999))
    pol, a_t, P_t = t(R["policy_k"]), t(cal["a_grid"]), t(cal["P"])
    ks = torch.zeros(1, dtype=torch.float64, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    for _ in range(3):
        pkg.sim_capital_dev(ws, pol, a_t, P_t, 3, float(cal["a_grid"][Na // 3]), U, ks, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        pkg.sim_capital_dev(ws, pol, a_t, P_t, 3, float(cal["a_grid"][Na // 3]), U, ks, st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(json.dumps({"Na": Na, "sim_mode": mode, "T": 10000, "ms_per_chain": ms, "ns_per_step": ms * 1e6 / 1e4,
                      "K_s": float(ks[0]), "status": int(st[0])}))
    ws.close()
