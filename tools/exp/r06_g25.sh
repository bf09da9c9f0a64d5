#!/bin/bash
# Kernel-trace stats of the spread speculative chain (tools/sim_bench.py, mode -1 only)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT SIM_MODES=-1
O=gpurun_out/r06_g25
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 tools/sim_bench.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -i "sim_par\|sim_chain" $O/prof/run_kernel_stats.csv | cut -c1-220
