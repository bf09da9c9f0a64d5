"""Coalescence of the A9 capital chain (Aiyagari_VFI.m:104-129) on CPU: two chains driven by the
same shocks from different starting capital become bit-identical after a few steps and stay so.
This is what the speculative-segment chain (sim_chain_par_kernel) relies on for speed — not for
correctness, its repair passes are exact whatever the starts.  For the VFI policy at r = 0.04 (the
reference defaults) it reports, over starts on a stride of the grid, the steps until the path from
that start equals the path from the reference's own k1 bit for bit, for several shock offsets.

    python tools/sim_coalesce.py [--r 0.04] [--stride 10] [--steps 1000]
Uses the C restatement (oracle/corc), so it is a tool, never imported by the product path."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import corc  # noqa: E402
from oracle import np_oracle as no  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--r", type=float, default=0.04)
    ap.add_argument("--stride", type=int, default=10)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--offsets", type=int, default=4)
    args = ap.parse_args()
    cal = no.calib_aiyagari(Na=400)
    a, s, P = cal["a_grid"], cal["s"], cal["P"]
    alpha, delta, beta, sigma = 0.36, 0.08, 0.96, 5.0
    w = (1 - alpha) * ((args.r + delta) / alpha) ** (alpha / (alpha - 1))
    R = corc.vfi_solve(np.zeros((7, a.size)), a, s, P, args.r, w, beta, sigma)
    pol = R["policy_k"]
    U_all = no.matlab_rand_stream(2 + args.offsets * args.steps)[2:]
    worst = 0
    for o in range(args.offsets):
        U = U_all[o * args.steps:(o + 1) * args.steps - 1]
        z1 = 3
        _, ref = corc.sim_capital(pol, a, P, z1, float(a[a.size // 2]), U, return_path=True)
        steps = []
        for i in range(0, a.size, args.stride):
            _, p = corc.sim_capital(pol, a, P, z1, float(a[i]), U, return_path=True)
            diff = np.nonzero(p != ref)[0]
            steps.append(0 if diff.size == 0 else int(diff[-1]) + 1)
        worst = max(worst, max(steps))
        print(f"offset {o}: steps to coalesce over {len(steps)} starts: min {min(steps)} "
              f"median {int(np.median(steps))} max {max(steps)}")
    print(f"worst {worst} of {args.steps - 1} steps")


if __name__ == "__main__":
    main()
