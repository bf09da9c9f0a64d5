#!/bin/bash
# Round 4: tree dispatch order A/B (variant 16 = XCD ranges in row-major order; 80 = the same
# ranges dealt heaviest first, bit 6) + raw per-item traces of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g7
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VARS="16 80 2064 8208 8272" ROUNDS=3 O=$O/ab bash tools/ab_variant.sh || exit 1
AIY_TRACE_DUMP=$O/trace timeout -k 10 200 python3 tools/tree_trace.py 20000 8208 > $O/tree_trace.txt 2>&1 || { tail -20 $O/tree_trace.txt; exit 1; }
grep -E "variant|co-resident|span" $O/tree_trace.txt
