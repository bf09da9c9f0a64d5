#!/bin/bash
# XCD-dealt KS sweep as the default + the KS panel prologue applied: KS suites; then the
# concurrency traces (r06_g08.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g09
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ks_gpu.py tests/test_ks_dist_gpu.py tests/test_ks_staged_gpu.py tests/test_ks_panel_gpu.py tests/test_mex_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/exp/r06_g08.sh
