export TMPDIR=/tmp
mkdir -p gpurun_out/r02_s8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_s8/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r02_s8/pytest.log; grep -E "FAIL|Error" gpurun_out/r02_s8/pytest.log | head
[ $rc -ge 124 ] && exit $rc
NA=400 TAG=r02_s8v400 VARIANTS="0 2 16 18" bash tools/variant_sweep.sh || exit 1
