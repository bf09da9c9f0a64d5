#!/bin/bash
# Labour small-grid screen: the 64-block pre-screen (kWideCoarse = 16) — bit-exactness with the
# flag forced on, then the A/B against the default (4).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g52
mkdir -p $O
AIY_WIDE_FLAGS=20 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wide_gpu.py tests/test_labor_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for fl in 4 20; do
timeout -k 10 300 python -u tools/wide_tune.py --no-tree --flags $fl --cases lab:400,lab:1000,lab:2000 --geos "1,8,16;1,8,32;1,16,16" --out $O/tune_f$fl.jsonl > $O/tune_f$fl.log 2>&1 || { tail -5 $O/tune_f$fl.log; exit 1; }
done
python - <<'PY'
import json
for fl in (4,20):
  for l in open(f"gpurun_out/r05_g52/tune_f{fl}.jsonl"):
    r=json.loads(l)
    print(fl, r['kind'], r['Na'], r['geo'], round(r['us_per_sweep'],2), round(r['kernel_us'],2), r.get('same'), r.get('wave_work_med_max'), r.get('slowest_wave_med'))
PY
