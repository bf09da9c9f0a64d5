#!/bin/bash
# Round 4: GPU suite + smoke + default bench with bits 23-24 in the A1 default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g37
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python -u bench.py --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.out').read().strip().splitlines()[-1]); l=d['legs']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], l['batch_config4_share']['value'], l['labor_vfi.Na20000']['ms_per_sweep'], l['solve_to_tol']['wall_ms'])"
