#!/bin/bash
# Round 4: labour tree (A3) dispatch orders at Na = 20,000 — the per-XCD permutations (bit 11
# cheapest last, bit 6 heaviest first) against the default XCD ranges (16); parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g13
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_labor_gpu.py tests/test_pinned_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 200 python3 tools/labor_bench.py 20000 --variants=16,2064,80 >> $O/ab.txt 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done
cat $O/ab.txt
