#!/bin/bash
# KS column-shaped kernels: KS GPU parity tests, KS leg + ghost model, rocprof of the KS leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02b_s5; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_ks_gpu.py tests/test_ks_dist_gpu.py tests/test_mex_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -u bench_ks.py > $OUT/ks.json 2>&1; rc=$?; echo "ks rc=$rc"; grep '^{' $OUT/ks.json | cut -c1-600
[ $rc -ne 0 ] && exit $rc
timeout -k 10 150 python -u bench_ks.py --ghost-model > $OUT/ghost.json 2>&1; echo "ghost rc=$?"; grep '^{' $OUT/ghost.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$OUT/prof -o run -- python3 $PWD/bench_ks.py > $OUT/prof.log 2>&1; echo "prof rc=$?"
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r02b_s5/prof/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/r02b_s5/prof/run_kernel_stats.csv")
for r in csv.DictReader(open(f[0])):
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
exit 0
