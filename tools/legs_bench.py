"""EGM / labour-EGM / push legs of bench.py alone (A/B aid): one JSON line each.
    python tools/legs_bench.py"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import bench_legs as BL  # noqa: E402

import torch  # noqa: E402

pkg = bench.load_pkg()
dev = torch.device("cuda", 0)
for name, fn in (("egm", lambda: BL.egm_leg(pkg, dev, 20000)),
                 ("labor_egm", lambda: BL.egm_leg(pkg, dev, 20000, labor=True)),
                 ("dist", lambda: BL.dist_leg(pkg, dev, cpu_pushes=1))):
    out = fn()
    keep = {k: out[k] for k in ("us_per_step", "us_per_push") if k in out}
    rf = out.get("roofline", {})
    keep["kernel_avg_ms"] = rf.get("kernel_avg_ms")
    print(json.dumps({"leg": name, **keep}))
