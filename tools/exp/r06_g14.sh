#!/bin/bash
# GE wall (tools/ge_wall_probe.py: overlapped driver, median of 5) at 4 vs 16 hardware queues,
# alternating; plus the concurrency case 6 solves, no chains (is it the stream count?).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g14
mkdir -p $O
for rep in 1 2 3; do
  for q in 4 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python3 tools/ge_wall_probe.py > $O/q${q}_$rep.json 2> $O/q$q.err || { tail -5 $O/q$q.err; exit 1; }
    echo "q=$q rep=$rep $(cut -c1-150 $O/q${q}_$rep.json)"
  done
done
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python3 tools/ge_concurrency.py --queues $q --cases 4:0,6:0,8:0,2:2,4:2 --specs 16 --out $O/conc_q$q.json > $O/conc_q$q.log 2>&1 || { tail -5 $O/conc_q$q.log; exit 1; }
  echo "== queues $q"; grep spec $O/conc_q$q.log | cut -c1-170
done
