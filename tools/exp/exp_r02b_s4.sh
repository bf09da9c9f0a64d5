#!/bin/bash
# momentum start: VFI-family GPU parity tests, headline bench with/without momentum, tree trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02b_s4; mkdir -p $OUT
Q="--no-cpu-baseline --no-ge --no-ks --no-panel --no-extra --no-solve"
timeout -k 10 120 python -u bench.py $Q > $OUT/bench_mom.json 2>&1; rc=$?; echo "bench mom rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/bench_mom.json; exit $rc; }
timeout -k 10 120 python -u bench.py $Q --variant 528 > $OUT/bench_nomom.json 2>&1; rc=$?; echo "bench nomom rc=$rc"; [ $rc -ne 0 ] && exit $rc
python - <<'PY'
import json
for f in ("bench_mom", "bench_nomom"):
    for line in open(f"gpurun_out/r02b_s4/{f}.json"):
        if line.startswith("{"):
            d = json.loads(line); print(f, d["ms_per_step"], d["repeats"]["median_ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"])
PY
timeout -k 10 600 python -u -m pytest tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py tests/test_batch_gpu.py tests/test_labor_gpu.py tests/test_ge_gpu.py tests/test_ge_batch_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u tools/tree_trace.py 20000 16 528 > $OUT/trace.txt 2>&1; echo "trace rc=$?"
grep -E "^variant|entry->start|wave-0" $OUT/trace.txt
exit 0
