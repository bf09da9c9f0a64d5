#!/bin/bash
# GE wall (overlapped driver, median of 5, 16 queues as in bench.py) vs the chains' host poll
# interval, alternating; and the probe at the inherited 4 queues (bench.py no longer overrides
# on import).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g15
mkdir -p $O
for rep in 1 2 3; do
  for nap in 2e-4 2e-5 0; do
    AIY_GE_CHAIN_NAP=$nap GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python3 tools/ge_wall_probe.py > $O/n${nap}_$rep.json 2> $O/n.err || { tail -5 $O/n.err; exit 1; }
    echo "nap=$nap rep=$rep $(cut -c1-100 $O/n${nap}_$rep.json)"
  done
  GPU_MAX_HW_QUEUES=4 timeout -k 10 120 python3 tools/ge_wall_probe.py > $O/q4_$rep.json 2> $O/n.err || { tail -5 $O/n.err; exit 1; }
  echo "queues=4 rep=$rep $(cut -c1-100 $O/q4_$rep.json)"
done
