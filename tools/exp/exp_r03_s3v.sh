#!/bin/bash
# Round 3 session 3: chained EGM solve (one launch per step for Na > 1024) — EGM GPU tests and
# the egm legs (chained vs two-launch, variant bit 13).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03_s3v}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "egm or mex" > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u - > $O/egm_ab.json 2> $O/egm_ab.err <<'PY'
import json, torch, bench, bench_legs
pkg = bench.load_pkg(); dev = torch.device("cuda:0")
out = {}
for Na in (20000,):
    for var in (-1, 8192, 16384):
        for lab in (False, True):
            r = bench_legs.egm_leg(pkg, dev, Na, labor=lab, variant=var)
            out[f"{Na}_{var}_{'labor' if lab else 'egm'}"] = {"solve_dev_us_per_step": r["us_per_step"], "single_step_us": r["single_step_dev"]["us_per_step"], "host_solve": r["solve"]["us_per_iteration"]}
print(json.dumps(out, indent=1))
PY
rc=$?; cat $O/egm_ab.json; tail -3 $O/egm_ab.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/egm_trace.py $O/egm_trace.txt > /dev/null 2>&1 && cat $O/egm_trace.txt
