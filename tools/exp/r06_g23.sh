#!/bin/bash
# Speculative chain phase split by timing probes (results wrong by design): P1 no in-order sum,
# P2 no repair passes, P3 neither and no segment phase (z scan + tables only); default = all.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g23
mkdir -p $O
for L in "" _P1 _P2 _P3; do
  AIY_HIP_LIB=$PWD/aiyagari-replication_amd/libaiyagari_hip$L.so SIM_MODES=-1 timeout -k 10 200 python -u tools/sim_bench.py > $O/b$L.log 2>&1 || { tail -5 $O/b$L.log; exit 1; }
  grep '"Na": 400' $O/b$L.log | sed "s/^/lib$L /"
done
