#!/bin/bash
# Final profiles: the default bench's kernel-trace stats, and the A9 chain's counter passes on
# its default (spread) segment kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g40
mkdir -p $O
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 bench.py --no-cpu-baseline --detail $O/prof_bench_detail.json > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
head -12 $O/prof/run_kernel_stats.csv | cut -c1-150
P="sq sq2 grbm fetch write"
OUT=$O/pmc_sim PASSES="$P" PMC_CMD=$PWD/tools/pmc_workloads_r05.py BENCH_ARGS="sim" timeout -k 10 300 bash tools/pmc.sh > $O/pmc_sim.log 2>&1 || { tail -5 $O/pmc_sim.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_sim "sim_par_seg_kernel<512, false>" $O/pmc_sim_par_seg.json 0 0 > /dev/null && python3 tools/pmc_traffic.py $O/pmc_sim "sim_par_seg_kernel<512, false>" $O/traffic_sim_par_seg.json 0 0 > /dev/null
python3 -c "import json; d=json.load(open('$O/pmc_sim_par_seg.json')); print(d['launches'], {k: round(v, 3) for k, v in d['derived'].items()})"
