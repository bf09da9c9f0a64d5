#!/bin/bash
# descending-j tile order for the labour tree at Na = 20,000 (default 16 vs 8192), labour parity
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02c_s12; mkdir -p $OUT
timeout -k 10 300 python -u tools/labor_bench.py 20000 --variants=16,8192,16,8192 > $OUT/labor_bench.txt 2>&1; rc=$?
grep -v amdgpu.ids $OUT/labor_bench.txt
exit $rc
