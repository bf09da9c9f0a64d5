#!/bin/bash
# Round 3 session 3: staged-push load batching, P/V prefetch, tree launch bounds (no spills),
# LEAN staging two loads at a time — full GPU suite, the push trace, the whole bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03_s3j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u tools/dist_trace.py $O/dist_trace.txt > /dev/null 2> $O/dist_trace.err || { tail -5 $O/dist_trace.err; exit 1; }
head -12 $O/dist_trace.txt
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench ok
