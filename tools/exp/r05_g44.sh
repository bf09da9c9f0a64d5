#!/bin/bash
# Small-grid sweep: per-wave screen work (rounds, entered blocks, votes) of the slowest waves.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g46
mkdir -p $O
timeout -k 10 200 python -u tools/wide_tune.py --no-tree --cases a1:400,lab:400 --geos "1,8,32;1,8,16" --out $O/tune.jsonl > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/${TAG:-r05_g46}/tune.jsonl"):
    r=json.loads(l)
    print(r['kind'], r['geo'], round(r['us_per_sweep'],2), round(r['kernel_us'],2), r.get('same'), r.get('wave_work_med_max'), r.get('slowest_wave_med'))
PY
