#!/bin/bash
# sub-block split at Na = 20,000: labour and A1 with 2/4 cooperating waves vs the 1-wave default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02c_s7; mkdir -p $OUT
timeout -k 10 300 python -u tools/labor_bench.py 20000 --variants=16,18,4114,20,4116 > $OUT/labor_bench.txt 2>&1; rc=$?
grep -v amdgpu.ids $OUT/labor_bench.txt; [ $rc -ne 0 ] && exit $rc
Q="--no-cpu-baseline --no-ge --no-ks --no-panel --no-extra --no-solve"
for v in 16 4114 4116; do
  timeout -k 10 120 python -u bench.py $Q --variant $v > $OUT/bench_v$v.json 2>&1 || exit 1
  python -c "import json,sys; d=[json.loads(l) for l in open('$OUT/bench_v$v.json') if l.startswith('{')][0]; print('A1 Na20000 variant $v', d['ms_per_step'], d['repeats']['median_ms_per_step'], d['roofline']['kernel_avg_ms'])"
done
