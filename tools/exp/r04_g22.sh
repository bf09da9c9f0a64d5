#!/bin/bash
# Round 4 (experimental): the direct schedule's sweep hand-off through command-processor
# packets (hipStreamWaitValue64 / hipStreamWriteValue64 on the mapped page) — cost in the
# one-GPU model, then the 3-rank on-card test in that mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r04_g22
mkdir -p $O
timeout -k 10 120 python3 bench_ks.py --direct-model > $O/direct_model.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/direct_model.json').read().strip().splitlines()[-1]); print(json.dumps(d['handoff']))"
timeout -k 10 200 python -u -m pytest tests/test_ks_dist_gpu.py -x -v --timeout 90 --timeout-method thread -k "direct_ipc" > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; exit $rc
