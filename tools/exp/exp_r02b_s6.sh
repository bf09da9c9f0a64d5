#!/bin/bash
# exhaustive kernel rewrite: VFI-family parity tests + bench with the exhaustive leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02b_s6; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py tests/test_labor_gpu.py tests/test_ge_gpu.py tests/test_mex_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ge --no-ks --no-panel --no-solve > $OUT/bench.json 2>&1; rc=$?; echo "bench rc=$rc"
python3 - <<'PY'
import json
for line in open("gpurun_out/r02b_s6/bench.json"):
    if line.startswith("{"):
        d = json.loads(line)
        print(d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["roofline"]["frac"])
        print(json.dumps(d.get("exhaustive")))
PY
exit 0
