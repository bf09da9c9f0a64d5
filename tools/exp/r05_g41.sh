#!/bin/bash
# Small-grid sweep: labour levels loaded with the prologue; shared vs CU-exclusive workgroups.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05_g41}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u tools/wide_tune.py --cases a1:400,lab:400 --geos "1,8,32;1,8,16;1,16,16" --out $O/tune.jsonl > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
timeout -k 10 200 python -u tools/wide_tune.py --cases a1:400,lab:400 --geos "1,8,32;1,8,16;1,16,16" --excl --no-tree --out $O/tune_excl.jsonl > $O/tune_excl.log 2>&1 || { tail -5 $O/tune_excl.log; exit 1; }
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/${TAG:-r05_g41}/tune*.jsonl".replace("${TAG:-r05_g41}","r05_g41"))):
    for l in open(f):
        r=json.loads(l)
        print(f.split('/')[-1], r['kind'], r['geo'], round(r['us_per_sweep'],2), round(r['kernel_us'],2), r.get('same'), r.get('phase_cycles_med_max'))
PY
