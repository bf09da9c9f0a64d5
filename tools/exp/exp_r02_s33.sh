set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_s33
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_spec_solve_gpu.py > $O/pytest1.log 2>&1 || { tail -40 $O/pytest1.log; exit 1; }
tail -2 $O/pytest1.log
timeout -k 10 300 python -u tools/ge_timing.py
