#!/bin/bash
# Round 4: per-item tree trace with SIMD co-residency (sweeps 10, 25, 100) + the MEX GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g4
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_mex_gpu.py tests/test_dist_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/tree_trace.py 20000 16 > $O/tree_trace.txt 2>&1 || { tail -20 $O/tree_trace.txt; exit 1; }
cat $O/tree_trace.txt
