#!/bin/bash
# Small-grid sweep geometries re-tuned at HEAD (batch2 default, batched prologue/screen loads).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g51
mkdir -p $O
timeout -k 10 400 python -u tools/wide_tune.py --no-tree --cases a1:400,lab:400,a1:1000,lab:1000 --geos "1,8,32;1,8,16;1,4,16;1,4,32;1,16,32;1,16,16;2,8,32;1,8,64" --out $O/tune.jsonl > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05_g51/tune.jsonl"):
    r=json.loads(l)
    print(r['kind'], r['Na'], r['geo'], round(r['us_per_sweep'],2), round(r['kernel_us'],2), r.get('same'), r.get('slowest_wave_med'))
PY
