set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_s26
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_egm_gpu.py tests/test_mex_gpu.py > gpurun_out/r02_s26/pytest.log 2>&1 || { tail -30 gpurun_out/r02_s26/pytest.log; exit 1; }
tail -2 gpurun_out/r02_s26/pytest.log
timeout -k 10 900 python -u bench.py > gpurun_out/r02_s26/bench.json 2> gpurun_out/r02_s26/bench.err
tail -c 300 gpurun_out/r02_s26/bench.json
