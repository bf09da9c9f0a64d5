#!/bin/bash
# HEAD sanity after the reverted experiments: smoke, the KS / sim / GE GPU suites, a headline-only bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g35
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ks_gpu.py tests/test_ks_staged_gpu.py tests/test_sim_par_gpu.py tests/test_ge_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-ks --no-ge --no-panel --no-extra > $O/bench.out 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -1 $O/bench.out | cut -c1-300
