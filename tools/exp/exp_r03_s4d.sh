#!/bin/bash
# Round 3 session 3: pipelined speculative VFI solve — the VFI/solve/GE GPU tests, then the
# solve-to-tol and GE legs through bench.py (no extras).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03_s4d}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "spec or pinned or ge or vfi or batch or labor or mex" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ks --no-panel --no-extra > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('step', d['ms_per_step'], 'solve', d['solve_to_tol'], 'ge', d['ge_equilibrium']['wall_s_gpu'], d['ge_equilibrium']['wall_s_gpu_sequential'], 'ge_batch', d['ge_batch']['value'])"
