"""A/B of the overlapped GE driver (round-4 rework vs the HEAD copy in _ge_base.py): wall time
and identical traces, alternating, 4 rounds.  (Record of profiles/r04_g25_ge_driver_ab.txt: the
rework was reverted, and _ge_base.py was a temporary copy of the package's ge.py at HEAD placed
next to it for the run.)"""
import importlib
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
import bench  # noqa: E402

pkg = bench.load_pkg()
base = importlib.import_module(pkg.__name__ + "._ge_base")
pkg.ge.aiyagari_vfi_overlapped(max_iter=5)
base.aiyagari_vfi_overlapped(max_iter=5)
for rnd in range(4):
    for name, mod in (("base", base), ("new", pkg.ge)):
        out = mod.aiyagari_vfi_overlapped()
        print(json.dumps({"impl": name, "round": rnd, "wall_s": out["wall_s"], "r": out["r"],
                          "iters": out["iters"][:3]}))
        sys.stdout.flush()
