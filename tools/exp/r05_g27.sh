#!/bin/bash
# Solve / chain interference vs hardware queues and stream priority (tools/ge_concurrency.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05_g27}
mkdir -p $O
for q in 4 8 16; do
  for pr in "" "--prio"; do
    echo "=== queues $q $pr"
    timeout -k 10 120 python tools/ge_concurrency.py --cases 1:1,2:2,4:2,4:0,6:0 --specs 16 --queues $q $pr --out $O/conc_q${q}${pr}.json 2>&1 | grep spec || exit 1
  done
done
