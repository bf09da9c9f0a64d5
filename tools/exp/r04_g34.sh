#!/bin/bash
# Round 4: bit 23 (hint window = the hint when the extrapolated window is used) — labour at
# Na = 20,000 and A1 (simplified code), A/B against the current defaults.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g34
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 tools/labor_bench.py 20000 --variants=2097168,10485776 >> $O/labor.txt 2>> $O/labor.err || { tail -5 $O/labor.err; exit 1; }
done
cat $O/labor.txt
VARS="2164752 10553360" ROUNDS=3 O=$O/ab bash tools/ab_variant.sh
