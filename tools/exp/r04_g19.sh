#!/bin/bash
# Round 4: labour tree (A3) at Na = 20,000 with cooperating waves per tile (variant bits 1-2,
# bit 12 = round-robin deal of the first superblock's passing 8-blocks) against the default 16.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g19
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 tools/labor_bench.py 20000 --variants=16,18,20,4114,4116 >> $O/ab.txt 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done
cat $O/ab.txt
