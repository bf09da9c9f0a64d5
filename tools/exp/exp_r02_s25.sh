set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_s25
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vfi_gpu.py tests/test_pinned_gpu.py > gpurun_out/r02_s25/pytest.log 2>&1 || { tail -30 gpurun_out/r02_s25/pytest.log; exit 1; }
tail -2 gpurun_out/r02_s25/pytest.log
TAG=r02_s25v VARIANTS="16 18 2" BENCH_EXTRA="--no-extra --no-ge --no-ks --no-panel --repeats 3" timeout -k 10 400 bash tools/variant_sweep.sh
timeout -k 10 120 python -u tools/tree_trace.py 20000 18 > gpurun_out/r02_s25/trace.txt 2>&1
