#!/bin/bash
# kernel + HIP-runtime trace of tools/ge_concurrency.py with 2 and with 4
# concurrent warm Na = 400 solves (no chains), to see whether the solves' kernels serialise on
# queues or overlap and each run slower.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g08
mkdir -p $O
for c in 1:0 2:0 4:0; do
  tag=${c%%:*}
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $PWD/$O/t$tag -o run -- python3 tools/ge_concurrency.py --cases $c --specs 16 --out $O/conc$tag.json > $O/conc$tag.log 2>&1 || { tail -5 $O/conc$tag.log; exit 1; }
  tail -1 $O/conc$tag.log
done
ls $O/t2/ | head
