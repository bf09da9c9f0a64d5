#!/bin/bash
# what slows solves beside Monte-Carlo chains (no profiler): chains CU-
# exclusive (GE driver default) vs shared, and the chains' host poll interval.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g11
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 120 python3 tools/ge_concurrency.py --cases 1:0,2:0,0:1,1:1,2:1,2:2,4:2 --specs 16 --out $O/$tag.json "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "== $tag $*"; grep spec $O/$tag.log | cut -c1-170
}
run excl
run shared --chain-shared
run busypoll --chain-nap 0
run excl2
