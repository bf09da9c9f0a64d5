set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_s16
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_vfi_gpu.py tests/test_labor_gpu.py tests/test_pinned_gpu.py tests/test_spec_solve_gpu.py tests/test_batch_gpu.py > gpurun_out/r02_s16/pytest.log 2>&1 || { tail -30 gpurun_out/r02_s16/pytest.log; exit 1; }
tail -3 gpurun_out/r02_s16/pytest.log
TAG=r02_s16v VARIANTS="16 0 2 18" BENCH_EXTRA="--no-extra --repeats 3" timeout -k 10 300 bash tools/variant_sweep.sh
timeout -k 10 120 python -u tools/tree_trace.py 20000 16 > gpurun_out/r02_s16/trace.txt 2>&1
