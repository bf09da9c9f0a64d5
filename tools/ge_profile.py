"""Wall-time breakdown of the GE leg (Aiyagari_VFI.m defaults): calibration, each VFI solve and
each Monte-Carlo supply, timed around the host-tier calls the driver makes.  Usage (GPU box):
    python tools/ge_profile.py [repeats]"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from tests.conftest import load_pkg
    pkg = load_pkg()
    ge = pkg.ge
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ge.aiyagari_vfi(max_iter=5)
    acc = {}
    orig = {k: getattr(ge, k) for k in ("vfi_solve", "sim_capital")}
    orig_cal = ge.cb.aiyagari

    def wrap(name, fn):
        def f(*a, **k):
            t0 = time.perf_counter()
            r = fn(*a, **k)
            acc.setdefault(name, []).append(time.perf_counter() - t0)
            return r
        return f

    for k, fn in orig.items():
        setattr(ge, k, wrap(k, fn))
    ge.cb.aiyagari = wrap("calibration", orig_cal)
    walls = []
    for _ in range(reps):
        acc.clear()
        t0 = time.perf_counter()
        out = ge.aiyagari_vfi()
        walls.append(time.perf_counter() - t0)
    print(json.dumps({"wall_s": walls, "sweeps": int(sum(out["iters"])), "iters": out["iters"],
                      "last_breakdown_s": {k: [round(x, 5) for x in v] for k, v in acc.items()},
                      "totals_s": {k: round(sum(v), 5) for k, v in acc.items()}}))


if __name__ == "__main__":
    main()
