#!/bin/bash
# headline geometry re-check on the current kernel: R (states per lane) and W (waves per tile)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02b_s9; mkdir -p $OUT
Q="--no-cpu-baseline --no-ge --no-ks --no-panel --no-extra --no-solve"
for v in 16 17 18 19 0 1; do
  timeout -k 10 120 python -u bench.py $Q --variant $v > $OUT/b_$v.json 2>&1 || { echo "fail $v"; tail -3 $OUT/b_$v.json; exit 1; }
  python3 -c "
import json
for l in open('$OUT/b_$v.json'):
    if l.startswith('{'): d=json.loads(l); print('variant $v', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(d['roofline']['kernel_avg_ms']*1e3,2))"
done
exit 0
