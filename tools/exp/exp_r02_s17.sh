set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_s17
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r02_s17/pytest.log 2>&1 || { tail -30 gpurun_out/r02_s17/pytest.log; exit 1; }
tail -3 gpurun_out/r02_s17/pytest.log
TAG=r02_s17v VARIANTS="16 0 17" BENCH_EXTRA="--no-extra --repeats 3" timeout -k 10 300 bash tools/variant_sweep.sh
timeout -k 10 120 python -u tools/tree_trace.py 20000 16 > gpurun_out/r02_s17/trace.txt 2>&1
