#!/bin/bash
# Small-grid sweep A/B: batch thresholds (flags 1, 4) and the 8-pair labour round (flag 8).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g47
mkdir -p $O
for fl in 0 1 4 8 12; do
timeout -k 10 200 python -u tools/wide_tune.py --no-tree --flags $fl --cases a1:400,lab:400 --geos "1,8,32;1,8,16" --out $O/tune_f$fl.jsonl > $O/tune_f$fl.log 2>&1 || { tail -5 $O/tune_f$fl.log; exit 1; }
done
python - <<'PY'
import json
for fl in (0,1,4,8,12):
  for l in open(f"gpurun_out/r05_g47/tune_f{fl}.jsonl"):
    r=json.loads(l)
    print(fl, r['kind'], r['geo'], round(r['us_per_sweep'],2), round(r['kernel_us'],2), r.get('same'), r.get('wave_work_med_max'), r.get('slowest_wave_med'))
PY
