#!/bin/bash
# Round 4: PMC + HBM traffic of the kernels the bench legs time (egm_chain_kernel, labour EGM
# chain, ks_howard_slopes_kernel, dist_push_kernel), then a kernel-trace --stats profile of the
# default bench run (the roofline kernels' average durations) and the bench itself.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04_g2}
mkdir -p $O
timeout -k 10 120 python3 tools/pmc_workloads_r04.py > $O/workloads.log 2>&1 || { tail -20 $O/workloads.log; exit 1; }
OUT=$O/pmc PMC_CMD=$PWD/tools/pmc_workloads_r04.py BENCH_ARGS="" bash tools/pmc.sh || exit $?
E="egm_chain_kernel"
python3 tools/pmc_summary.py $O/pmc "$E" $O/pmc_egm_chain.json 0 200 > /dev/null
python3 tools/pmc_traffic.py $O/pmc "$E" $O/traffic_egm_chain.json 0 200 > /dev/null
python3 tools/pmc_summary.py $O/pmc "$E" $O/pmc_labor_egm_chain.json 200 200 > /dev/null
python3 tools/pmc_traffic.py $O/pmc "$E" $O/traffic_labor_egm_chain.json 200 200 > /dev/null
python3 tools/pmc_summary.py $O/pmc "ks_howard_slopes_kernel" $O/pmc_ks_howard_slopes.json > /dev/null
python3 tools/pmc_traffic.py $O/pmc "ks_howard_slopes_kernel" $O/traffic_ks_howard_slopes.json > /dev/null
python3 tools/pmc_summary.py $O/pmc "dist_push_kernel" $O/pmc_dist_push.json > /dev/null
python3 tools/pmc_traffic.py $O/pmc "dist_push_kernel" $O/traffic_dist_push.json > /dev/null
for f in $O/pmc_*.json $O/traffic_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', json.dumps(d.get('derived', d))[:400])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof_bench.out 2> $O/prof_bench.err || exit $?
tail -c 400 $O/prof_bench.out
