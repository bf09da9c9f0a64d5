#!/bin/bash
# Kernel trace of one warm solve alone and beside one MC chain (tools/ge_concurrency.py): are
# the sweep kernels slower, or are the gaps between them longer?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05_g26}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/prof -o run -- python3 tools/ge_concurrency.py --cases 1:0,1:1 --specs 16 --out $O/conc.json > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
cat $O/prof.log | grep spec
