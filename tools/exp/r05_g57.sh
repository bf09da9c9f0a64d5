#!/bin/bash
# Closing counters for the kernels changed late in round 5 (small-grid sweep: A1 / labour at
# Na = 400; the push), plus the default bench's kernel-trace stats at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g57
mkdir -p $O
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 bench.py --no-cpu-baseline --detail $O/prof_bench_detail.json > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
P="sq sq2 grbm fetch write"
run() {
  local wl=$1
  OUT=$O/pmc_$wl PASSES="$P" PMC_CMD=$PWD/tools/pmc_workloads_r05.py BENCH_ARGS="$wl" timeout -k 10 300 bash tools/pmc.sh > $O/pmc_$wl.log 2>&1 || { tail -5 $O/pmc_$wl.log; exit 1; }
}
summ() {  # workload kernel skip take name
  python3 tools/pmc_summary.py $O/pmc_$1 $2 $O/pmc_$5.json $3 $4 > /dev/null || exit 1
  python3 tools/pmc_traffic.py $O/pmc_$1 $2 $O/traffic_$5.json $3 $4 > /dev/null || exit 1
}
run labor400; summ labor400 bell_wide_kernel 5 10 labor_na400
run a1_400;   summ a1_400 bell_wide_kernel 0 0 a1_na400
run dist;     summ dist dist_push_kernel 0 0 dist_push
for f in $O/pmc_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['launches'], json.dumps({k: round(v, 3) for k, v in d['derived'].items() if k in ('valu_busy','waves_per_simd','wait_frac','kernel_cycles')}))"; done
for f in $O/traffic_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d.get('bytes_per_launch'))"; done
echo "g57 done"
