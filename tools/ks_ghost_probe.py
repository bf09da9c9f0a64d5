"""GPU-side timing of the 8-rank KS Howard schedule on one GPU (bench_ks.ghost_model's blocks,
no exchanges), for rocprofv3 --kernel-trace + tools/phase_stats.py: one phase per emulated rank
(k = 32,768, K = 64, depth 4, 24 fused sweeps after one warm block), 20 ms apart, so the trace
gives each rank's kernel time per sweep without the Python issue gaps of a wall-clock timer."""
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
kd = pkg.ks_dist
depth = int(sys.argv[1]) if len(sys.argv) > 1 else 4
kg, Kg, P, V0 = pkg.calibration.krusell_smith(k_size=32768, K_size=64)
B = np.array([0.1, 0.97, 0.08, 0.975])
V = torch.as_tensor(np.ascontiguousarray(V0.transpose(2, 1, 0)), device=dev)
V2 = V.clone()
dV, dV2 = torch.empty_like(V), torch.empty_like(V)
ko = torch.ones_like(V)
for rank in range(8):
    K0, K1, s0, s1 = kd.shard_slices(64, rank, 8)
    sh = kd.HipShard(kg, Kg, B, P, pkg.ks_params(), K0, K1, s0, s1)
    sh.improve(V, ko)
    rects = kd.ghost_rects(sh.kp_idx, 64, K0, K1, s0, s1, depth)
    shards = [sh] + [sh.ghost(*r) for r in rects[1:depth]]
    shards[-1].hints(ko)
    torch.cuda.synchronize()
    time.sleep(0.02)
    for blk in range(7):  # one warm block, then 6 blocks = 24 sweeps
        shards[depth - 1].slopes(V, dV)
        for i in range(1, depth + 1):
            shards[depth - i].howard_fused(V, dV, ko, V2, dV2)
            V, V2 = V2, V
            dV, dV2 = dV2, dV
    torch.cuda.synchronize()
    time.sleep(0.02)
    for g in shards[1:]:
        g.close()
    sh._ghosts.clear()
    sh.close()
print("ks ghost probe done")
