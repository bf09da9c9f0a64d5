"""Labour-VFI legs of bench.py alone (tuning aid):
    python tools/labor_bench.py [Na ...] [--variants v1,v2,...]"""
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
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    variants = [-1]
    for x in sys.argv[1:]:
        if x.startswith("--variants="):
            variants = [int(v) for v in x.split("=", 1)[1].split(",")]
    for Na in [int(x) for x in args] or [400, 20000]:
        for var in variants:
            out = BL.labor_leg(pkg, dev, Na, steps=10 if Na <= 4000 else 5, reps=3, cpu=False,
                               variant=var)
            print(json.dumps({"Na": Na, "variant": var, "ms_per_sweep": out["ms_per_sweep"],
                              "kernel_ms": out["kernel_ms"], "frac": out["roofline"]["frac"]}))


if __name__ == "__main__":
    main()
