#!/bin/bash
# Round 4: GPU suite + smoke + default bench with bit 23 in the A1 default; labour A/B of bit 23.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g35
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python -u bench.py --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.out').read().strip().splitlines()[-1]); l=d['legs']; print(d['value'], d['ms_per_step'], d['roofline']['frac'], l['batch_config4_share']['value'], l['labor_vfi.Na20000']['ms_per_sweep'], l['solve_to_tol']['wall_ms'])"
for r in 1 2; do
  timeout -k 10 300 python3 tools/labor_bench.py 20000 --variants=2097168,10485776 >> $O/labor.txt 2>> $O/labor.err || { tail -5 $O/labor.err; exit 1; }
done
cat $O/labor.txt
