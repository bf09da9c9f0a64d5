#!/bin/bash
# Round 4: the start-up climb with paired loads (same evaluations, fewer dependent rounds) —
# parity, then headline and labour A/B against the previous build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g32
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py tests/test_labor_gpu.py tests/test_batch_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="build_ab/libaiyagari_hip_base.so aiyagari-replication_amd/libaiyagari_hip.so" ROUNDS=4 O=$O/ab bash tools/ab_headline.sh || exit 1
for r in 1 2; do
  AIY_HIP_LIB=$PWD/build_ab/libaiyagari_hip_base.so timeout -k 10 200 python3 tools/labor_bench.py 20000 | sed 's/^/base /'
  timeout -k 10 200 python3 tools/labor_bench.py 20000 | sed 's/^/new  /'
done
