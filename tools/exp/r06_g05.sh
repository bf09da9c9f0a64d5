#!/bin/bash
# EGM whole-solve launch: phase split, workgroups spread (SP=1) vs packed on one XCD (SP=8)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g05
mkdir -p $O
timeout -k 10 200 python -u tools/egm_grid_probe.py > $O/sp1.json 2> $O/sp1.err || { tail -5 $O/sp1.err; exit 1; }
cat $O/sp1.json
AIY_EGM_SP=8 timeout -k 10 200 python -u tools/egm_grid_probe.py > $O/sp8.json 2> $O/sp8.err || { tail -5 $O/sp8.err; exit 1; }
cat $O/sp8.json
AIY_EGM_SP=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_egm_gpu.py -k "workgroup or speculative" > $O/tests8.log 2>&1 || { tail -30 $O/tests8.log; exit 1; }
tail -1 $O/tests8.log
