#!/bin/bash
# Speculative-segment chain vs serial vs the C restatement (forced modes, never-coalescing drift
# policy, find-empty at segment edges, shape fallback).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g17
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_sim_par_gpu.py tests/test_sim_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
