#!/bin/bash
# Round 4: the start-up climb with eight probes per round (variant bit 21) — parity, then the
# headline A/B against the default (67600 = 16 | 2048 | 1 << 16) and a trace of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g15
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vfi_gpu.py tests/test_spec_solve_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VARS="67600 2164752" ROUNDS=3 O=$O/ab bash tools/ab_variant.sh || exit 1
timeout -k 10 200 python3 tools/tree_trace.py 20000 67600 2164752 > $O/tree_trace.txt 2>&1 || { tail -20 $O/tree_trace.txt; exit 1; }
grep -E "variant|co-resident|entry->start" $O/tree_trace.txt
