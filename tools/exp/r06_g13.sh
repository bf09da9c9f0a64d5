#!/bin/bash
# Labour small-grid sweep: per-level cash / bar once, the lane's blocks' operands read once, five
# levels' pairs per bound-test round (A) vs HEAD~ (B: libaiyagari_hip_B.so); wide tests with A.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g13
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_wide_gpu.py tests/test_labor_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 200 python -u tools/wide_ab.py A >> $O/ab.jsonl 2> $O/errA.log || { tail -5 $O/errA.log; exit 1; }
  AIY_HIP_LIB=$PWD/aiyagari-replication_amd/libaiyagari_hip_B.so timeout -k 10 200 python -u tools/wide_ab.py B >> $O/ab.jsonl 2> $O/errB.log || { tail -5 $O/errB.log; exit 1; }
done
cut -c1-200 $O/ab.jsonl
