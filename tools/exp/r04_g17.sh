#!/bin/bash
# Round 4: the MC chain (A9) with a register window + prefetched policy values — parity (sim,
# GE, batch, MEX), then chain timing against the previous build (build_ab/libaiyagari_hip_base.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g17
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sim_gpu.py tests/test_ge_gpu.py tests/test_batch_gpu.py tests/test_pinned_gpu.py tests/test_mex_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  AIY_HIP_LIB=$PWD/build_ab/libaiyagari_hip_base.so timeout -k 10 120 python3 tools/sim_bench.py > $O/base_$r.txt 2>&1 || { tail -5 $O/base_$r.txt; exit 1; }
  timeout -k 10 120 python3 tools/sim_bench.py > $O/new_$r.txt 2>&1 || { tail -5 $O/new_$r.txt; exit 1; }
done
grep -h '"Na"' $O/base_*.txt | sed 's/^/base /'; grep -h '"Na"' $O/new_*.txt | sed 's/^/new  /'
