"""Workloads for the launch-floor attribution (run under rocprofv3 --kernel-trace, then
tools/phase_stats.py): each phase is a back-to-back chain on one stream with no host
synchronisation inside it, and phases are separated by 20 ms of host sleep so that the trace
splits into them.  Phases (in order):
  0 trivial one-wave kernels (torch add_), dependent through one scalar
  1 EGM steps, Na = 400 (egm_fused_kernel)      2 EGM steps, Na = 20,000 (two launches)
  3 EGM steps, Na = 20,000 one-pass (variant bit 12)
  4 EGM host-tier solve, Na = 20,000 (speculative batches: reads, copies)
  5-7 histogram pushes, Na = 400 / 4,000 / 20,000 on a synthetic monotone policy
  8 headline sweeps, Na = 20,000 (table + tree)
  9-10 KS Howard sweeps of emulated rank 0 of 8 (k = 32,768, K = 64), depth 4: fused
       Howard+slopes launches, then slopes + Howard launches (bench_ks.ghost_model's schedule)"""
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

pkg = bench.load_pkg()
dev = torch.device("cuda:0")
t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)


def phase_end():
    torch.cuda.synchronize()
    time.sleep(0.02)


x = torch.zeros(1, dtype=torch.float64, device=dev)
for _ in range(300):
    x.add_(1.0)
phase_end()

for Na, variant in ((400, -1), (20000, -1), (20000, 4096)):
    cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
    N, r = cal["N"], 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    a = cal["a_grid"]
    ws = pkg.Workspace(N, Na)
    ws.set_variant(variant)
    c = [t(np.tile(((1 + r) * a + w * np.mean(cal["s"]))[None, :], (N, 1))),
         torch.zeros((N, Na), dtype=torch.float64, device=dev)]
    pk = torch.zeros_like(c[0])
    a_t, s_t, P_t = t(a), t(cal["s"]), t(cal["P"])
    for q in range(200):
        pkg.egm_step_dev(ws, c[q & 1], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"],
                         cal["amin"], c[1 - (q & 1)], pk)
    phase_end()

cal = pkg.calibration.aiyagari(Na=20000, shocks="rouwenhorst")
r = 0.04
w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
a = cal["a_grid"]
pc0 = np.tile(((1 + r) * a + w * np.mean(cal["s"]))[:, None], (1, cal["N"]))
for _ in range(2):
    R = pkg.egm_solve(pc0.copy(), a, cal["s"], cal["P"], r, w, cal["beta"], cal["sigma"],
                      cal["amin"], 1e-5, 1000)
phase_end()

for Na in (400, 4000, 20000):
    cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
    N = cal["N"]
    j = np.arange(Na)
    idx = np.stack([np.clip((j * (0.9 + 0.02 * i)).astype(np.int32), 0, Na - 1)
                    for i in range(N)]).astype(np.int32)
    ws = pkg.Workspace(N, Na)
    lam0 = torch.full((N, Na), 1.0 / (N * Na), dtype=torch.float64, device=dev)
    out = torch.empty_like(lam0)
    pkg.dist_stationary_dev(ws, lam0, t(cal["a_grid"]), t(cal["P"]), out, policy_idx=t(idx),
                            tol=0.0, max_iter=200)
    phase_end()

cal = pkg.calibration.aiyagari(Na=20000, shocks="rouwenhorst")
N = cal["N"]
ws = pkg.Workspace(N, 20000)
va = torch.zeros((N, 20000), dtype=torch.float64, device=dev)
vb = torch.zeros_like(va)
idx = torch.zeros((N, 20000), dtype=torch.int32, device=dev)
ws.vfi_solve(va, vb, t(cal["a_grid"]), t(cal["s"]), t(cal["P"]), r, w, cal["beta"],
             cal["sigma"], 1e-5, 60, idx)
phase_end()

kd = pkg.ks_dist
kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=32768, K_size=64)
B = np.array([0.1, 0.97, 0.08, 0.975])
V = t(V0.transpose(2, 1, 0))
V2 = V.clone()
dV, dV2 = torch.empty_like(V), torch.empty_like(V)
ko = torch.ones_like(V)
K0, K1, s0, s1 = kd.shard_slices(64, 0, 8)
sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), K0, K1, s0, s1)
sh.improve(V, ko)
rects = kd.ghost_rects(sh.kp_idx, 64, K0, K1, s0, s1, 4)
shards = [sh] + [sh.ghost(*rr) for rr in rects[1:4]]
shards[-1].hints(ko)
phase_end()
for fused in (True, False):
    for blk in range(6):
        if fused:
            shards[3].slopes(V, dV)
        for i in range(1, 5):
            if fused:
                shards[4 - i].howard_fused(V, dV, ko, V2, dV2)
                dV, dV2 = dV2, dV
            else:  # ks_dev_howard: its own slopes launch, then the sweep
                shards[4 - i].howard(V, ko, V2)
            V, V2 = V2, V
    phase_end()
print("probe done")
