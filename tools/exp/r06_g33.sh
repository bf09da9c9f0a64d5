#!/bin/bash
# Staged KS sweep: boundary rows dispatched after a fraction of the interior rows (AIY_KS_BND_AT)
# instead of after all of them.  KS staged/dist suites at 0.5, then the one-GPU probe per value.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g33
mkdir -p $O
AIY_KS_BND_AT=0.5 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ks_staged_gpu.py tests/test_ks_dist_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for at in 1.0 0.75 0.5 0.25; do
    AIY_KS_BND_AT=$at timeout -k 10 200 python3 tools/ks_staged_probe.py > $O/p_${at}_$rep.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    echo "at=$at rep=$rep $(tail -1 $O/p_${at}_$rep.json | cut -c1-220)"
  done
done
