#!/bin/bash
# exhaustive scan with direct outputs: parity tests + small-grid tree vs exhaustive timings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02b_s8; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_labor_gpu.py tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py tests/test_mex_gpu.py tests/test_ge_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/labor_bench.py 100 400 1000 2000 --variants=2,1024 > $OUT/labor.txt 2>&1; echo "labor rc=$?"; grep '^{' $OUT/labor.txt
Q="--no-cpu-baseline --no-ge --no-ks --no-panel --no-extra --no-solve --steps 50"
for na in 400 1000 2000 4000; do
  for v in 2 1024; do
    timeout -k 10 120 python -u bench.py $Q --na $na --variant $v > $OUT/b_${na}_$v.json 2>&1 || { echo "bench fail $na $v"; tail -3 $OUT/b_${na}_$v.json; exit 1; }
    python3 -c "
import json
for l in open('$OUT/b_${na}_$v.json'):
    if l.startswith('{'): d=json.loads(l); print('A1 Na=$na variant=$v', round(d['ms_per_step']*1e3,2), 'us/step')"
  done
done
exit 0
