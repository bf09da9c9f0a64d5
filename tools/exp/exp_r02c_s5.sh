#!/bin/bash
# labour tree at the script's Na = 400: where a sweep's ~52 us go (trace), W = 1/2/4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02c_s5; mkdir -p $OUT
timeout -k 10 300 python -u tools/labor_trace.py 400 0 2 4 > $OUT/labor_trace.txt 2>&1; rc=$?
grep -v amdgpu.ids $OUT/labor_trace.txt
exit $rc
