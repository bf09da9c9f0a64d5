set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_s31
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_spec_solve_gpu.py > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -3 $O/pytest1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_vfi_gpu.py tests/test_ge_gpu.py tests/test_ge_batch_gpu.py tests/test_mex_gpu.py tests/test_pinned_gpu.py > $O/pytest2.log 2>&1 || { tail -40 $O/pytest2.log; exit 1; }
tail -2 $O/pytest2.log
