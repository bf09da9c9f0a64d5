#!/bin/bash
# Small-grid sweep: the output phase's arguments in the prologue batch too.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g60
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_labor_gpu.py tests/test_ge_gpu.py tests/test_vfi_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/wide_tune.py --no-tree --cases a1:400,lab:400,lab:1000 --geos "1,8,32;1,8,16;1,4,16" --out $O/tune.jsonl > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r05_g60/tune.jsonl"):
    r=json.loads(l)
    print(r['kind'], r['Na'], r['geo'], round(r['us_per_sweep'],2), round(r['kernel_us'],2), r.get('same'), r.get('phase_cycles_med_max'))
PY
