#!/bin/bash
# Round 3 session 3: LDS-staged histogram push — dist GPU tests, the bench dist leg, the probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_s3e}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "dist" > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "
import json, torch, bench, bench_legs
pkg = bench.load_pkg()
print(json.dumps(bench_legs.dist_leg(pkg, torch.device('cuda:0'))))" > $O/dist_leg.json 2> $O/dist_leg.err || { tail -5 $O/dist_leg.err; exit 1; }
cat $O/dist_leg.json
