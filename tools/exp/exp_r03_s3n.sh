#!/bin/bash
# Round 3 session 3: PMC of the secondary kernels (VERDICT r2 items 3 and missing 7): the
# config-4 batched tree launch, labour tree (Na 400 W=4, Na 20,000 W=1), EGM RHS/interp, push.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03_s3n}
mkdir -p $O
OUT=$O/pmc PMC_CMD=$PWD/tools/pmc_workloads.py BENCH_ARGS=" " bash tools/pmc.sh || exit $?
S=tools/pmc_summary.py; T=tools/pmc_traffic.py
python3 $S $O/pmc "bell_tree_kernel<4, false, 1, 1, 1, false>" $O/pmc_batch.json 0 25 > /dev/null
python3 $T $O/pmc "bell_tree_kernel<4, false, 1, 1, 1, false>" $O/traffic_batch.json 0 25 > /dev/null
python3 $S $O/pmc "bell_tree_kernel<4, true, 1, 5, 4, false>" $O/pmc_labor_na400.json > /dev/null
python3 $S $O/pmc "bell_tree_kernel<4, true, 1, 5, 1, false>" $O/pmc_labor_na20000.json > /dev/null
python3 $S $O/pmc "egm_rhs_kernel" $O/pmc_egm_rhs.json > /dev/null
python3 $S $O/pmc "egm_interp_kernel" $O/pmc_egm_interp.json > /dev/null
python3 $T $O/pmc "egm_rhs_kernel" $O/traffic_egm_rhs.json > /dev/null
python3 $T $O/pmc "egm_interp_kernel" $O/traffic_egm_interp.json > /dev/null
python3 $S $O/pmc "dist_push_kernel<false>" $O/pmc_dist_push.json > /dev/null
python3 $T $O/pmc "dist_push_kernel<false>" $O/traffic_dist_push.json > /dev/null
for f in $O/pmc_*.json $O/traffic_*.json; do echo "== $f"; python3 -c "import json,sys; d=json.load(open('$f')); print(json.dumps(d.get('derived', d))[:400])"; done
