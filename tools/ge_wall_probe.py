"""The GE wall of Aiyagari_VFI.m's defaults (the overlapped driver, median of 5 runs after two
warm-ups) under the hardware-queue count this process inherits (GPU_MAX_HW_QUEUES, read by the
HIP runtime at start).  bench.py raises the count to 16 for its own process and starts this
script with the inherited value, so the contract line shows both.  Prints one JSON
line."""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import bench
    pkg = bench.load_pkg()
    import torch
    torch.cuda.set_device(0)
    kw = {"lookahead": int(sys.argv[1])} if len(sys.argv) > 1 else {}  # (A/B: default otherwise)
    pkg.ge.aiyagari_vfi_overlapped(max_iter=5, **kw)
    pkg.ge.aiyagari_vfi_overlapped(max_iter=5, **kw)
    walls, out = [], None
    for _ in range(5):
        t0 = time.perf_counter()
        out = pkg.ge.aiyagari_vfi_overlapped(**kw)
        walls.append(time.perf_counter() - t0)
    print(json.dumps({"hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "runtime default"),
                      "wall_s_gpu": sorted(walls)[2], "wall_s_gpu_runs": walls,
                      "lookahead": out["lookahead"], "r": out["r"]}), flush=True)


if __name__ == "__main__":
    main()
