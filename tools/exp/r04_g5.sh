#!/bin/bash
# Round 4: KS direct (peer-read) schedule — parity tests and the one-GPU 8-shard model; the tree
# trace with SIMD co-residency; the MEX/dist GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ks_gpu.py tests/test_mex_gpu.py tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench_ks.py --direct-model > $O/direct_model.json 2> $O/direct_model.err || { tail -20 $O/direct_model.err; exit 1; }
cat $O/direct_model.json
timeout -k 10 200 python3 tools/tree_trace.py 20000 16 > $O/tree_trace.txt 2>&1 || { tail -20 $O/tree_trace.txt; exit 1; }
cat $O/tree_trace.txt
