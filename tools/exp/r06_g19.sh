#!/bin/bash
# Hybrid tree launch with no cooperative tile (its own cost) vs the default and H = 8; then the
# GE driver's lookahead 1-4 at 16 hardware queues with the speculative-segment chains.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g19
mkdir -p $O
O=$O/ab VARS="27330576 1033963536 94439440" ROUNDS=2 bash tools/ab_variant.sh
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u tools/ge_lookahead.py > gpurun_out/r06_g19/lookahead.json 2> gpurun_out/r06_g19/lookahead.err || { tail -5 gpurun_out/r06_g19/lookahead.err; exit 1; }
cat gpurun_out/r06_g19/lookahead.json
