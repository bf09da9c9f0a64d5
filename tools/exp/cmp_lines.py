"""Print the legs of several contract lines side by side (scalar fields only).
    python tools/exp/cmp_lines.py gpurun_out/r05_g49/bench.out gpurun_out/r05_g50/bench.out"""
import json
import sys

rows = {}
for f in sys.argv[1:]:
    line = [l for l in open(f) if l.startswith("{")][-1]
    d = json.loads(line)
    rows.setdefault("headline", []).append(f"{d['value']:.4g} ({d['ms_per_step'] * 1e3:.2f} us)")
    for k, v in d["legs"].items():
        if isinstance(v, dict):
            keys = [kk for kk in ("us_per_step", "us_per_push", "ms_per_sweep", "wall_ms", "wall_s_gpu",
                                  "vfi_iteration_ms", "value") if kk in v]
            if keys:
                rows.setdefault(k, []).append(f"{keys[0]}={v[keys[0]]:.4g}")
for k, v in rows.items():
    print(f"{k:22s}", "  ".join(v))
