#!/bin/bash
# Round 4: GPU suite after the pruning + EGM chain rework, the bench, and the EGM chain's
# kernel-trace stats and HBM traffic (tools/pmc_workloads_r04.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04_g3}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run -- python3 tools/pmc_workloads_r04.py > $O/prof.log 2>&1 || exit 1
OUT=$O/pmc PASSES="fetch write" PMC_CMD=$PWD/tools/pmc_workloads_r04.py BENCH_ARGS="" bash tools/pmc.sh > $O/pmc.log 2>&1 || exit 1
python3 tools/pmc_traffic.py $O/pmc egm_chain_kernel $O/traffic_egm_chain.json 0 200
python3 tools/pmc_traffic.py $O/pmc egm_chain_kernel $O/traffic_labor_egm_chain.json 200 200
