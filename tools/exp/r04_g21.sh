#!/bin/bash
# Round 4: the tree path's table with 2 / 4 candidates per thread (bell_table_tree_kernel<KPT>)
# — parity on the in-tree build (KPT = 2), then the headline A/B of base / kpt2 / kpt4.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g21
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py tests/test_labor_gpu.py tests/test_ev_mfma_gpu.py tests/test_vfi_large_gpu.py tests/test_ge_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="build_ab/libaiyagari_hip_base.so build_ab/libaiyagari_hip_kpt2.so build_ab/libaiyagari_hip_kpt4.so" ROUNDS=3 O=$O/ab bash tools/ab_headline.sh
