#!/bin/bash
# Round 4: the linear drift extrapolation (bit 21) at the other sizes' defaults: A1 Na = 400
# (variant 2), labour Na = 20,000 (16) and Na = 400 (4 | 4096).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g28
mkdir -p $O
VARS="2 2097154" ROUNDS=3 O=$O/a400 ARGS="--no-cpu-baseline --no-ks --no-ge --no-panel --no-extra --na 400" bash tools/ab_variant.sh || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 tools/labor_bench.py 20000 --variants=16,2097168 >> $O/labor.txt 2>> $O/labor.err || { tail -5 $O/labor.err; exit 1; }
  timeout -k 10 300 python3 tools/labor_bench.py 400 --variants=4100,2101252 >> $O/labor.txt 2>> $O/labor.err || { tail -5 $O/labor.err; exit 1; }
done
cat $O/labor.txt
