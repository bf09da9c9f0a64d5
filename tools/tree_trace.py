"""Instrumented look at one tree sweep (Na = 20,000, Nz = 7): per-work-item durations, where
the time goes (tests vs candidates), and how the XCDs are loaded.  Tuning aid only."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    import torch
    pkg = bench.load_pkg()
    Na = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    variants = [int(v) for v in sys.argv[2:]] or [2]
    cal = pkg.calibration.aiyagari(Na=Na, shocks="rouwenhorst")
    N = cal["N"]
    r = 0.04
    w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
    dev = torch.device("cuda", 0)
    t = lambda x: torch.as_tensor(np.ascontiguousarray(x), device=dev)
    a_t, s_t, P_t = t(cal["a_grid"]), t(cal["s"]), t(cal["P"])
    for var in variants:
        v = [torch.zeros((N, Na), dtype=torch.float64, device=dev) for _ in range(2)]
        idx = torch.zeros((N, Na), dtype=torch.int32, device=dev)
        ws = pkg.Workspace(N, Na)
        ws.set_variant(var)
        cur = 0
        for q in range(101):
            if q in (10, 25, 100):
                ws.set_timing(True, trace=True)
            ws.vfi_sweep(v[cur], a_t, s_t, P_t, r, w, cal["beta"], cal["sigma"], v[1 - cur], idx,
                         hint=None if q == 0 else idx, mode=1)
            cur = 1 - cur
            if q in (10, 25, 100):
                torch.cuda.synchronize()
                ms, _, _ = ws.timing()
                ws.set_timing(False)
                T = ws.trace()
                if len(sys.argv) > 1 and "AIY_TRACE_DUMP" in __import__("os").environ:
                    np.save(f"{__import__('os').environ['AIY_TRACE_DUMP']}_v{var}_s{q}.npy", T)
                hw = (T[:, 2] >> 32) & 0xffffffff  # HW_REG_HW_ID of the item's wave
                T[:, 2] &= 0xffffffff             # XCC id
                dur = (T[:, 1] - T[:, 0]) / 100.0  # µs (100 MHz)
                t0 = T[:, 0].min()
                st = (T[:, 0] - t0) / 100.0
                en = (T[:, 1] - t0) / 100.0
                print(f"variant {var} sweep {q}: kernel {ms*1e3:.1f} us, items {len(T)}, "
                      f"span {en.max():.1f} us, start spread {st.max():.1f} us")
                print("  item duration us p50/p90/p99/max:",
                      np.percentile(dur, [50, 90, 99, 100]).round(1))
                for name, col in (("sup", 3), ("blk", 4), ("cand", 5), ("exact", 6)):
                    x = T[:, col].astype(float)
                    c = np.corrcoef(x, dur)[0, 1] if x.std() > 0 else 0
                    print(f"  {name}: mean {x.mean():.1f} max {x.max():.0f} corr(dur) {c:.2f}")
                boot = (T[:, 0] - T[:, 12]) / 100.0
                print("  entry->start us p50/p90/max: %s; start-up cycles mean %.0f; output cycles "
                      "mean %.0f; entry spread %.1f us" % (np.percentile(boot, [50, 90, 100]).round(1),
                      T[:, 13].mean(), T[:, 14].mean(), (T[:, 12].max() - T[:, 12].min()) / 100.0))
                pairs = T[:, 15].astype(float)
                nsubpass = T[:, 5].astype(float) / 8.0  # candidate tests / 8 per passing sub-block
                print("  (state, sub-block) pairs passing per wave: mean %.1f; passing sub-blocks "
                      "x 64 lanes: mean %.1f (ratio %.3f)" % (pairs.mean(), (nsubpass * 64).mean(),
                      pairs.sum() / max((nsubpass * 64).sum(), 1)))
                cy = T[:, 8:12].astype(float)
                print("  wave-0 cycles mean: top/sup-tests %.0f  block-tests %.0f  fine %.0f  exact %.0f"
                      % tuple(cy.mean(0)))
                slow = np.argsort(dur)[-5:]
                print("  slowest items (row, tile, dur, sup, blk, cand, exact):")
                ntile = (Na + 63) // 64
                for k in slow:
                    print("   ", k // ntile, k % ntile, round(dur[k], 1), *T[k, 3:7])
                for x in range(8):
                    m = T[:, 2] == x
                    if m.any():
                        print(f"  xcd {x}: items {m.sum()} busy-sum {dur[m].sum():.0f} us "
                              f"last end {en[m].max():.1f}")
                rows = np.arange(len(T)) // ntile
                print("  per-row mean dur:", [round(dur[rows == i].mean(), 1) for i in range(N)])
                # co-residency: items whose wave ran on the same SIMD (XCC, SE, SH, CU, SIMD)
                # during the item's own lifetime (entry to exit)
                simd = (T[:, 2] << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 7) | \
                    (((hw >> 8) & 15) << 2) | ((hw >> 4) & 3)
                ent = (T[:, 12] - t0) / 100.0
                co = np.zeros(len(T), int)
                for k in range(len(T)):
                    m = (simd == simd[k]) & (ent < en[k]) & (en > ent[k])
                    co[k] = int(m.sum())  # including itself
                print("  SIMDs used %d; items per SIMD max %d" % (len(np.unique(simd)),
                      np.bincount(np.unique(simd, return_inverse=True)[1]).max()))
                for c in sorted(set(co)):
                    m = co == c
                    print(f"    co-resident {c}: items {m.sum()} dur mean {dur[m].mean():.1f} "
                          f"p90 {np.percentile(dur[m], 90):.1f} max {dur[m].max():.1f} "
                          f"end max {en[m].max():.1f}")
                late = np.argsort(en)[-10:]
                print("  last to finish (row, tile, entry, dur, end, co, sup, blk, cand):")
                for k in late:
                    print("   ", k // ntile, k % ntile, round(ent[k], 1), round(dur[k], 1),
                          round(en[k], 1), co[k], *T[k, 3:6])


if __name__ == "__main__":
    main()
