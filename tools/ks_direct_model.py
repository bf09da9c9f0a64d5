"""Print bench_ks.direct_model (the direct schedule's compute side on one GPU, with the staged
hand-off of the slowest shard) as JSON.    python tools/ks_direct_model.py [out.json]"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import bench_ks  # noqa: E402

torch.cuda.set_device(0)
pkg = bench.load_pkg()
out = bench_ks.direct_model(pkg, torch.device("cuda:0"))
s = json.dumps(out, indent=1)
print(s)
if len(sys.argv) > 1:
    Path(sys.argv[1]).write_text(s)
