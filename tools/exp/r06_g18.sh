#!/bin/bash
# Hybrid tree launch (variant bit 26: heavy tiles on two waves): bit-exact tests, then the
# headline A/B against the default (H = 8, 32, 128 cooperative tiles per XCD range).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g18
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vfi_gpu.py -k "dispatch_orders or packed_workgroups" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
O=$O/ab VARS="27330576 94439440 362874896 631310352" ROUNDS=2 bash tools/ab_variant.sh
