"""A/B of the EGM step: one launch per step on small grids (egm_fused_kernel, the default for
Na <= 1024) vs the two-launch step (variant bit 11).  Per-step time of bench_legs.egm_leg."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import bench  # noqa: E402
import bench_legs as BL  # noqa: E402


def main():
    import torch
    pkg = bench.load_pkg()
    dev = torch.device("cuda", 0)
    out = {}
    for Na in (400, 1024, 20000):
        for labor in (False, True):
            for var in (-1, 2048, -1):
                r = BL.egm_leg(pkg, dev, Na, labor=labor, variant=var)
                key = f"Na{Na}_{'labor' if labor else 'egm'}_{'default' if var < 0 else 'two_launch'}"
                out.setdefault(key, []).append(round(r["us_per_step"], 2))
                print(key, out[key], "solve_ms", round(r["solve"]["wall_ms"], 3), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
