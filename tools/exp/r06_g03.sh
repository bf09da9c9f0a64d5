#!/bin/bash
# Staged KS sweep after the fixes (one host-page poller + a device go word; halo stored and read
# sc1, no fences): tests, then the probe with boundary rows last (default) and first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g03
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ks_staged_gpu.py tests/test_ks_dist_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/ks_staged_probe.py > $O/probe0.json 2> $O/probe0.err || { tail -5 $O/probe0.err; exit 1; }
cat $O/probe0.json
AIY_KS_BND_FIRST=1 timeout -k 10 300 python -u tools/ks_staged_probe.py > $O/probe1.json 2> $O/probe1.err || { tail -5 $O/probe1.err; exit 1; }
cat $O/probe1.json
