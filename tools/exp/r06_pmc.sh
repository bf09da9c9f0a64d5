#!/bin/bash
# Round 6: PMC + HBM-traffic passes of every kernel a bench leg times, at HEAD (the round-5
# set re-run, plus the speculative-segment chain): the headline tree over bench sweeps 6..25,
# then one workload per process from tools/pmc_workloads_r05.py (batch, labour 400 / 20k,
# A1 400, KS — now ks_howard_slopes_xcd_kernel — EGM, dist, sim).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06_pmc}
mkdir -p $O
P="sq sq2 grbm fetch write"
OUT=$O/pmc_tree PASSES="$P" BENCH_ARGS="--no-cpu-baseline --no-ge --no-solve --no-ks --no-panel --no-extra --steps 20 --warmup 5 --repeats 1" bash tools/pmc.sh > $O/pmc_tree.log 2>&1 || { tail -5 $O/pmc_tree.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_tree bell_tree_kernel $O/pmc_tree.json 5 20 > /dev/null
python3 tools/pmc_traffic.py $O/pmc_tree bell_tree_kernel $O/traffic_vfi_tree.json 5 20 > /dev/null
# workload | kernel prefix | skip | take | output names (pmc_X / traffic_X) ...
run() {
  local wl=$1
  OUT=$O/pmc_$wl PASSES="$P" PMC_CMD=$PWD/tools/pmc_workloads_r05.py BENCH_ARGS="$wl" bash tools/pmc.sh > $O/pmc_$wl.log 2>&1 || { tail -5 $O/pmc_$wl.log; exit 1; }
}
summ() {  # workload kernel skip take name
  python3 tools/pmc_summary.py $O/pmc_$1 $2 $O/pmc_$5.json $3 $4 > /dev/null || exit 1
  python3 tools/pmc_traffic.py $O/pmc_$1 $2 $O/traffic_$5.json $3 $4 > /dev/null || exit 1
}
run batch;    summ batch bell_tree_kernel 0 25 batch
run labor400; summ labor400 bell_wide_kernel 5 10 labor_na400
run labor20k; summ labor20k bell_tree_kernel 5 5 labor_na20000
run a1_400;   summ a1_400 bell_wide_kernel 0 0 a1_na400
run ks;       summ ks ks_howard_slopes_xcd_kernel 0 0 ks_howard_slopes
run egm;      summ egm egm_chain_kernel 0 200 egm_chain; summ egm egm_chain_kernel 200 200 labor_egm_chain
run dist;     summ dist dist_push_kernel 0 0 dist_push
run sim;      summ sim "sim_par_seg_kernel<512, false>" 0 0 sim_par_seg
for f in $O/pmc_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['launches'], json.dumps({k: round(v, 3) for k, v in d['derived'].items() if k in ('valu_busy','waves_per_simd','wait_frac','kernel_cycles')}))"; done
for f in $O/traffic_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d.get('bytes_per_launch'))"; done
echo "r06 pmc done"
