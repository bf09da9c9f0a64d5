export TMPDIR=/tmp
mkdir -p gpurun_out/r02_s5
timeout -k 10 300 python -u -m pytest tests/test_vfi_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_s5/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r02_s5/pytest.log
[ $rc -ge 124 ] && exit $rc
TAG=r02_s5v VARIANTS="0 64 80" bash tools/variant_sweep.sh || exit 1
timeout -k 10 200 python -u tools/tree_trace.py 20000 64 > gpurun_out/r02_s5/trace_v64.txt 2>&1; grep -v xcd gpurun_out/r02_s5/trace_v64.txt | tail -30
