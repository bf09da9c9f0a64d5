#!/bin/bash
# Round 3 session 3: re-tune tree geometries after the launch-bounds / LEAN staging change.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03_s3o}
mkdir -p $O
timeout -k 10 300 python -u tools/labor_bench.py 400 --variants=-1,2,4,4098,4100 > $O/labor400.txt 2>&1 || exit $?
cat $O/labor400.txt | grep Na
timeout -k 10 300 python -u tools/labor_bench.py 20000 --variants=16,18,20,4114 > $O/labor20000.txt 2>&1 || exit $?
cat $O/labor20000.txt | grep Na
TAG=r03_s3o/a1_400 NA=400 VARIANTS="0 2 4 16 18" bash tools/variant_sweep.sh || exit $?
TAG=r03_s3o/a1_20000 NA=20000 VARIANTS="16 18" bash tools/variant_sweep.sh || exit $?
