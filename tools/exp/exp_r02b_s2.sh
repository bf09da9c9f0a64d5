#!/bin/bash
# KS ghost-sweep session: GPU tests of ks_dist, the RCCL same-GPU probe, the ghost compute model
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/r02b_s2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_ks_dist_gpu.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest_ks.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/pytest_ks.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 150 python -u bench_ks.py --ghost-model > $OUT/ghost_model.json 2> $OUT/ghost_model.err; rc=$?
echo "ghost rc=$rc"; cat $OUT/ghost_model.json; tail -3 $OUT/ghost_model.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 100 python -u tools/exp/probe_rccl_same_gpu.py > $OUT/rccl_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -12 $OUT/rccl_probe.log
exit 0
