#!/bin/bash
# descending-j tile order (variant bit 13) for the headline tree kernel: parity, bench A/B, trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02c_s11; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_vfi_gpu.py -x -q --timeout 300 --timeout-method thread -k "noisy or hint" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
Q="--no-cpu-baseline --no-ge --no-ks --no-panel --no-extra --no-solve"
for v in 16 8192 16 8192; do
  timeout -k 10 120 python -u bench.py $Q --variant $v > $OUT/bench_v$v.json 2>&1 || exit 1
  python -c "import json,sys; d=[json.loads(l) for l in open('$OUT/bench_v$v.json') if l.startswith('{')][0]; print('A1 Na20000 variant $v', d['ms_per_step'], d['repeats']['median_ms_per_step'], d['roofline']['kernel_avg_ms'])"
done
timeout -k 10 200 python -u tools/tree_trace.py 20000 16 8192 > $OUT/trace.txt 2>&1; echo "trace rc=$?"
grep -E "^variant|entry->start|item duration" $OUT/trace.txt
