#!/bin/bash
# VERDICT r5 item 7 follow-up: the kernel trace (r06_g08) shows each solve's stream idle ~2/3 of
# its span, with ~60 us stalls of hipLaunchKernel hitting every host thread at once.  Runtime
# settings that could cause periodic runtime-wide stalls, one process each (no profiler).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g10
mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 120 python3 tools/ge_concurrency.py --cases 1:0,2:0,4:0,2:2 --specs 16 --out $O/$tag.json > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "== $tag $*"; grep spec $O/$tag.log | cut -c1-160
}
run base X=1
run sigpool ROC_SIGNAL_POOL_SIZE=4096
run aql ROC_AQL_QUEUE_SIZE=16384
run batch DEBUG_CLR_MAX_BATCH_SIZE=4096
run cpusync DEBUG_CLR_BATCH_CPU_SYNC_SIZE=4096
run activewait ROC_ACTIVE_WAIT_TIMEOUT=0
run base2 X=1
