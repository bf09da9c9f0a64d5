#!/bin/bash
# Concurrent solves: default geometry vs (1,8,64), shared vs CU-exclusive workgroups.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05_g29}
mkdir -p $O
for opt in "" "--excl" "--geo 1,8,64" "--geo 1,8,64 --excl" "--geo 1,16,64 --excl"; do
  echo "=== $opt"
  timeout -k 10 120 python tools/ge_concurrency.py --cases 1:0,2:2,4:0,4:2,6:0,8:0 --specs 16 $opt --out $O/conc.json 2>&1 | grep spec || exit 1
done
