#!/bin/bash
# Round 4: the KS direct schedule across processes (IPC-mapped column buffers + host-page
# sweep counters) on one card, and the packed-workgroup default through the VFI suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g10
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ks_dist_gpu.py -x -v --timeout 120 --timeout-method thread -k "direct" > $O/direct.log 2>&1
rc=$?; tail -15 $O/direct.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py tests/test_ks_dist_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
