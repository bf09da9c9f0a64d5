#!/bin/bash
# GE driver lookahead 1 vs 2 with the speculative-segment chains: three alternating rounds at
# 16 hardware queues, one at the inherited count.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g20
mkdir -p $O
for rep in 1 2 3; do
  for la in 1 2; do
    GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python3 tools/ge_wall_probe.py $la > $O/q16_la${la}_$rep.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
    echo "q16 la=$la rep=$rep $(cut -c1-160 $O/q16_la${la}_$rep.json)"
  done
done
for la in 1 2; do
  timeout -k 10 120 python3 tools/ge_wall_probe.py $la > $O/qinh_la${la}.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "inherited la=$la $(cut -c1-160 $O/qinh_la${la}.json)"
done
