#!/bin/bash
# Round 3 session 3: PMC + HBM traffic of the headline tree kernel on the current code, over
# bench.py's timed sweeps 6..25 (skip the 5 warm-up launches, take 20).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03_s3s}
mkdir -p $O
OUT=$O/pmc BENCH_ARGS="--no-cpu-baseline --no-ge --no-solve --no-ks --no-panel --no-extra --steps 20 --warmup 5 --repeats 1" bash tools/pmc.sh || exit $?
K="bell_tree_kernel<4, false, 1, 1, 1, false>"
python3 tools/pmc_summary.py $O/pmc "$K" $O/pmc_tree.json 5 20 > /dev/null
python3 tools/pmc_traffic.py $O/pmc "$K" $O/traffic_vfi_tree.json 5 20 > /dev/null
python3 tools/pmc_summary.py $O/pmc "bell_table_kernel" $O/pmc_table.json 5 20 > /dev/null
python3 tools/pmc_traffic.py $O/pmc "bell_table_kernel" $O/traffic_table.json 5 20 > /dev/null
for f in $O/pmc_tree.json $O/traffic_vfi_tree.json $O/pmc_table.json $O/traffic_table.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', json.dumps(d.get('derived', d))[:500])"; done
