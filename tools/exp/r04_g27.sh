#!/bin/bash
# Round 4: the start-up's drift extrapolated linearly from the last two shifts (variant bit 21;
# mom packs both shifts) — parity, then the headline A/B against the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g27
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py tests/test_batch_gpu.py tests/test_labor_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="build_ab/libaiyagari_hip_base.so aiyagari-replication_amd/libaiyagari_hip.so" ROUNDS=2 O=$O/libs bash tools/ab_headline.sh || exit 1
VARS="67600 2164752" ROUNDS=3 O=$O/ab bash tools/ab_variant.sh
