#!/bin/bash
# Round 4: start-window knobs on top of the default — bit 22 (extrapolated window ±2), bit 23
# (hint window reduced to the hint when the extrapolated one is used), both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g33
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vfi_gpu.py tests/test_pinned_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
VARS="2164752 6359056 10553360 14747664" ROUNDS=3 O=$O/ab bash tools/ab_variant.sh
