#!/bin/bash
# Round 4: per-wave diff slots in the EGM chain and push kernels (no end-of-kernel workgroup
# barrier) — parity, then the legs against the previous build, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g18
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_egm_gpu.py tests/test_dist_gpu.py tests/test_pinned_gpu.py tests/test_ks_dist_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  AIY_HIP_LIB=$PWD/build_ab/libaiyagari_hip_base.so timeout -k 10 200 python3 tools/legs_bench.py > $O/base_$r.txt 2>&1 || { tail -5 $O/base_$r.txt; exit 1; }
  timeout -k 10 200 python3 tools/legs_bench.py > $O/new_$r.txt 2>&1 || { tail -5 $O/new_$r.txt; exit 1; }
done
grep -h '"leg"' $O/base_*.txt | sed 's/^/base /'; grep -h '"leg"' $O/new_*.txt | sed 's/^/new  /'
