#!/bin/bash
# Speculative-segment A9 chain (sim_chain_par_kernel): sim / GE / MEX tests, then chain timings
# (by size vs the serial kernels) and the GE wall.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g16
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sim_gpu.py tests/test_ge_gpu.py tests/test_ge_batch_gpu.py tests/test_mex_gpu.py tests/test_pinned_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/sim_bench.py > $O/sim.log 2>&1 || { tail -5 $O/sim.log; exit 1; }
cat $O/sim.log | grep Na
for rep in 1 2; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python3 tools/ge_wall_probe.py > $O/ge_$rep.json 2> $O/ge.err || { tail -5 $O/ge.err; exit 1; }
  cut -c1-200 $O/ge_$rep.json
done
