#!/bin/bash
# Polled event waits (C spec loop + driver) vs the concurrency slowdown; GE lookahead walls.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05_g28}
mkdir -p $O
for q in 4 16; do
  echo "=== queues $q"
  timeout -k 10 120 python tools/ge_concurrency.py --cases 1:0,1:1,2:2,4:2,4:0,6:0,8:0 --specs 16 --queues $q --out $O/conc_q${q}.json 2>&1 | grep spec || exit 1
done
timeout -k 10 200 python tools/ge_lookahead.py > $O/ge_la.log 2>&1 || { tail -5 $O/ge_la.log; exit 1; }
head -2 $O/ge_la.log | cut -c1-800
