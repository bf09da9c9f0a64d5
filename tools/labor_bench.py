"""Labour-VFI legs of bench.py alone (tuning aid): python tools/labor_bench.py [Na ...]."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import bench_legs as BL  # noqa: E402


def main():
    import torch
    pkg = bench.load_pkg()
    dev = torch.device("cuda", 0)
    for Na in [int(x) for x in sys.argv[1:]] or [400, 20000]:
        out = BL.labor_leg(pkg, dev, Na, steps=10 if Na <= 4000 else 5, reps=3, cpu=False)
        print(json.dumps({"Na": Na, "ms_per_sweep": out["ms_per_sweep"],
                          "kernel_ms": out["kernel_ms"], "frac": out["roofline"]["frac"]}))


if __name__ == "__main__":
    main()
