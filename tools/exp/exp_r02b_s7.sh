#!/bin/bash
# labour cooperating waves: labour parity tests + Na 400/2000/20000 variant timings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02b_s7; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_labor_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/labor_bench.py 400 2000 --variants=16,2,4,6 > $OUT/labor.txt 2>&1; echo "labor rc=$?"; grep '^{' $OUT/labor.txt
timeout -k 10 200 python -u tools/labor_bench.py 20000 --variants=16,18,20 > $OUT/labor20k.txt 2>&1; echo "labor20k rc=$?"; grep '^{' $OUT/labor20k.txt
exit 0
