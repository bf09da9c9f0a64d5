#!/bin/bash
# fused small-grid EGM step: EGM/GE/MEX GPU parity tests, then one launch vs two per step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02c_s4; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_egm_gpu.py tests/test_ge_gpu.py tests/test_mex_gpu.py tests/test_vfi_gpu.py tests/test_spec_solve_gpu.py tests/test_batch_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/exp/egm_ab.py > $OUT/egm_ab.txt 2>&1; rc=$?; echo "egm_ab rc=$rc"
grep -v amdgpu.ids $OUT/egm_ab.txt | tail -20
exit $rc
