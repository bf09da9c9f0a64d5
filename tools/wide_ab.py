"""A/B of two builds of the library on the small-grid sweep (tools/wide_tune.run, default geometry
per size): run as `python tools/wide_ab.py TAG` with AIY_HIP_LIB selecting the build; prints one
JSON line per (kind, Na)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import bench  # noqa: E402
import wide_tune  # noqa: E402

pkg = bench.load_pkg()
tag = sys.argv[1] if len(sys.argv) > 1 else "?"
for kind, Na, geo in (("lab", 400, (1, 8, 16)), ("lab", 1000, (1, 8, 32)), ("a1", 400, (1, 8, 32))):
    rec, _ = wide_tune.run(pkg, kind, Na, geo, n=50, warm=10, reps=5)
    print(json.dumps({"tag": tag, "kind": kind, "Na": Na, "us_per_sweep": round(rec["us_per_sweep"], 3),
                      "kernel_us": round(rec["kernel_us"], 3),
                      "slowest_wave": rec.get("slowest_wave_med")}), flush=True)
