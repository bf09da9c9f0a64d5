#!/bin/bash
# Spread chain with four-wave table staging: tests, chain timings, kernel-trace stats, GE walls.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g26
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sim_par_gpu.py tests/test_sim_gpu.py tests/test_ge_gpu.py tests/test_ge_batch_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SIM_MODES=-1,1 timeout -k 10 200 python -u tools/sim_bench.py > $O/sim.log 2>&1 || { tail -5 $O/sim.log; exit 1; }
grep '"Na": 400\|"Na": 900' $O/sim.log
SIM_MODES=-1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 tools/sim_bench.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -i "sim_par" $O/prof/run_kernel_stats.csv | cut -c1-160
for rep in 1 2; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python3 tools/ge_wall_probe.py > $O/ge_$rep.json 2> $O/ge.err || { tail -5 $O/ge.err; exit 1; }
  cut -c1-120 $O/ge_$rep.json
done
