#!/bin/bash
# Closing re-run after the late KS changes: the GPU suite, the default bench (contract line +
# detail), and the KS sweep's counter passes refreshed (tools/exp/r06_pmc.sh's ks workload).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g32
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 300 $O/bench.out
P="sq sq2 grbm fetch write"
OUT=$O/pmc_ks PASSES="$P" PMC_CMD=$PWD/tools/pmc_workloads_r05.py BENCH_ARGS="ks" timeout -k 10 400 bash tools/pmc.sh > $O/pmc_ks.log 2>&1 || { tail -5 $O/pmc_ks.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_ks ks_howard_slopes_xcd_kernel $O/pmc_ks_howard_slopes.json 0 0 > /dev/null && python3 tools/pmc_traffic.py $O/pmc_ks ks_howard_slopes_xcd_kernel $O/traffic_ks_howard_slopes.json 0 0 > /dev/null
python3 -c "import json; d=json.load(open('$O/pmc_ks_howard_slopes.json'))['derived']; print({k: round(v, 3) for k, v in d.items()})"
