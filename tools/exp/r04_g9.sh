#!/bin/bash
# Round 4: packed workgroups (variant bits 16-17: 2/4/8 one-wave tiles per workgroup) — parity,
# then the headline A/B against the new default (2064), and a trace of the 4-wave packing.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g9
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vfi_gpu.py tests/test_spec_solve_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VARS="2064 67600 133136 198672 131152" ROUNDS=3 O=$O/ab bash tools/ab_variant.sh || exit 1
timeout -k 10 200 python3 tools/tree_trace.py 20000 133136 > $O/tree_trace.txt 2>&1 || { tail -20 $O/tree_trace.txt; exit 1; }
grep -E "variant|co-resident|span" $O/tree_trace.txt
