#!/bin/bash
# Tree-kernel geometry sweep at the headline size: one short bench per variant (results are
# identical across variants, only the time differs).  VARIANTS / NA / BENCH_EXTRA override.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-variants}
mkdir -p "$OUT"
for v in ${VARIANTS:-0 2 4 6 16 18 20}; do
  timeout -k 10 120 python -u bench.py --na ${NA:-20000} --no-cpu-baseline --no-ge --no-ks --no-panel \
      --steps 20 --warmup 5 --variant $v ${BENCH_EXTRA} > "$OUT/v$v.log" 2>&1 || exit $?
  python3 - "$OUT/v$v.log" $v <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        s = d.get("solve_to_tol", {})
        print(f"variant {sys.argv[2]}: step {d['ms_per_step']*1e3:.1f} us kernel "
              f"{d['roofline']['kernel_avg_ms']*1e3:.1f} us value {d['value']:.3e} "
              f"solve {s.get('wall_ms', 0):.2f} ms iters {s.get('iters')}")
EOF
done
