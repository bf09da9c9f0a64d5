#!/bin/bash
# Staged KS sweep: where the one-GPU model's hand-off time goes (tools/ks_staged_probe.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g02
mkdir -p $O
timeout -k 10 300 python -u tools/ks_staged_probe.py > $O/probe.json 2> $O/probe.err || { tail -5 $O/probe.err; exit 1; }
cat $O/probe.json
