#!/bin/bash
# dealt 8-block tests (variant bit 12 now also splits the 8-block bound tests, LDS union): parity, labour and A1 small-grid times, trace
# labour and A1 sweep times at small Na with and without it, labour trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02c_s8; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_labor_gpu.py tests/test_vfi_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/labor_bench.py 400 1000 2000 --variants=2,4100,4102,4098 > $OUT/labor_bench.txt 2>&1; rc=$?
grep -v amdgpu.ids $OUT/labor_bench.txt; [ $rc -ne 0 ] && exit $rc
Q="--no-cpu-baseline --no-ge --no-ks --no-panel --no-extra --no-solve"
for v in 2 4098; do
  timeout -k 10 120 python -u bench.py $Q --na 400 --variant $v > $OUT/bench_na400_v$v.json 2>&1 || exit 1
  python -c "import json,sys; d=[json.loads(l) for l in open('$OUT/bench_na400_v$v.json') if l.startswith('{')][0]; print('A1 Na400 variant $v', d['ms_per_step'], d['repeats']['median_ms_per_step'])"
done
timeout -k 10 300 python -u tools/labor_trace.py 400 4100 > $OUT/labor_trace.txt 2>&1; rc=$?
grep -E "^variant|tree phase|wave-0" $OUT/labor_trace.txt
exit $rc
