export TMPDIR=/tmp
mkdir -p gpurun_out/r02_s7
timeout -k 10 300 python -u -m pytest tests/test_vfi_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_s7/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r02_s7/pytest.log
[ $rc -ge 124 ] && exit $rc
TAG=r02_s7v VARIANTS="0 16" bash tools/variant_sweep.sh || exit 1
timeout -k 10 200 python -u tools/tree_trace.py 20000 0 > gpurun_out/r02_s7/trace_v0.txt 2>&1; grep -v xcd gpurun_out/r02_s7/trace_v0.txt | tail -30
