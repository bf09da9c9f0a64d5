#!/bin/bash
# Monotonicity-bracket work model on the headline state.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g59
mkdir -p $O
timeout -k 10 400 python -u tools/mono_bracket_model.py --tiles 256 --out $O/mono_bracket.json > $O/mono.log 2>&1 || { tail -5 $O/mono.log; exit 1; }
cat $O/mono.log
