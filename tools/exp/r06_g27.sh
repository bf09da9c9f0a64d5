#!/bin/bash
# GE wall: the driver's chains spread (-1) vs one workgroup (1), three alternating rounds, 16 queues
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g27
mkdir -p $O
for rep in 1 2 3; do
  for m in -1 1; do
    AIY_GE_SIM_MODE=$m GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python3 tools/ge_wall_probe.py > $O/m${m}_$rep.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    echo "mode=$m rep=$rep $(cut -c1-200 $O/m${m}_$rep.json)"
  done
done
