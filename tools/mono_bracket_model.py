"""Work model of the monotonicity bracket for the headline tree screen.

The tree kernel's wave handles 64 consecutive states (lanes) of one productivity row and runs
the 8-block screen for the UNION over its lanes of the 8-blocks whose bound passes: a block
is entered by the whole wave when any lane's bound (Dmax8 − B)·max(c_{k0}, 0)^n ≥ 1 − 2^-48
holds.  The bracket would certify lanes 0 and 63 with the full screen and let the
interior lanes screen only blocks meeting [k*(lane 0), k*(lane 63)].  This counts, per tile,
the blocks the wave enters both ways, with each lane's bar at its exact optimum (the best case
for any screen), on the state the headline bench times (sweep 16 of the Na = 20,000 solve from
v = 0, inside its window of sweeps 6..25) and on the converged solution.

    python tools/mono_bracket_model.py [--tiles 256] [--out gpurun_out/mono_bracket.json]

The value function comes from the HIP solve (aiy_vfi_solve), so this runs on the GPU box; the
bound arithmetic is the kernel's own (bell_dev.hpp: table_D, screen_B, kThr), in numpy fp64."""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

TAU = 2.0 ** -46
THR = 0.99999999999999644729  # 1 - 2^-48


def tile_counts(V, a, s, P, r, w, beta, sigma, tiles, rng):
    N, Na = V.shape
    npw = int(round(sigma)) - 1
    EV = (beta * P) @ V                      # EV(i, k) (summation order is immaterial here)
    ne = npw * EV
    D = (ne + 1.0) + TAU * (np.abs(ne) + 1.0)
    nb8 = (Na + 7) // 8
    Dpad = np.full((N, nb8 * 8), -np.inf)
    Dpad[:, :Na] = D
    Dm8 = Dpad.reshape(N, nb8, 8).max(axis=2)
    a0 = a[np.minimum(np.arange(nb8) * 8, Na - 1)]  # each 8-block's first candidate
    ntile = (Na + 63) // 64
    picks = rng.choice(N * ntile, size=min(tiles, N * ntile), replace=False)
    res = {"union": [], "bracket": [], "lane": [], "span": []}
    for p in picks:
        i, t = divmod(int(p), ntile)
        j = np.arange(t * 64, min(t * 64 + 64, Na))
        coh = (1 + r) * a[j] + w * s[i]
        # each lane's exact optimum over the feasible prefix (c > 0)
        c = coh[:, None] - a[None, :]
        with np.errstate(divide="ignore", invalid="ignore"):
            u = (np.where(c > 0, c, np.nan) ** (1 - sigma) - 1) / (1 - sigma)
        val = u + EV[i][None, :]
        val = np.where(np.isnan(val), -np.inf, val)
        kstar = np.argmax(val, axis=1)
        best = val[np.arange(len(j)), kstar]
        B = npw * best - TAU * npw * np.abs(best)
        cb = np.maximum(coh[:, None] - a0[None, :], 0.0)
        tb = (Dm8[i][None, :] - B[:, None]) * cb ** npw
        passing = tb >= THR                  # [lanes, blocks]
        union = passing.any(axis=0)
        lo, hi = kstar[0] // 8, kstar[-1] // 8
        inb = np.zeros(nb8, bool)
        inb[lo:hi + 1] = True
        brk = passing[0] | passing[-1] | (passing[1:-1] & inb[None, :]).any(axis=0)
        res["union"].append(int(union.sum()))
        res["bracket"].append(int(brk.sum()))
        res["lane"].append(float(passing.sum(axis=1).mean()))
        res["span"].append(int(kstar[-1] - kstar[0]))
    return {k: float(np.mean(v)) for k, v in res.items()} | {"tiles": len(picks)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=256)
    ap.add_argument("--na", type=int, default=20000)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "mono_bracket.json"))
    args = ap.parse_args()
    import bench
    pkg = bench.load_pkg()
    cal = pkg.calibration.aiyagari(Na=args.na, shocks="rouwenhorst")
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    beta, sigma = cal["beta"], cal["sigma"]
    out = {"na": args.na, "rule": "blocks a 64-state wave enters: union over lanes (today) vs "
           "lanes 0 and 63 full + interior lanes inside [k*(0), k*(63)] (bracket); bars at "
           "each lane's exact optimum"}
    rng = np.random.default_rng(7)
    N = len(s)
    for name, iters in (("sweep16", 15), ("converged", 1000)):
        R = pkg.vfi_solve(np.zeros((N, args.na)), a, s, P, r, w, beta, sigma, 1e-5, iters)
        V = np.ascontiguousarray(R["v_new"])  # the next sweep's v_old
        out[name] = tile_counts(V, a, s, P, r, w, beta, sigma, args.tiles, rng)
        out[name]["after_sweeps"] = R["iters"]
        print(name, json.dumps(out[name]), flush=True)
    Path(args.out).parent.mkdir(parents=True, exist_ok=True)
    Path(args.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
