#!/bin/bash
# Round 3 session 3: histogram push with the long runs' chunks in one parallel pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_s3f}
mkdir -p $O
export PYTHONPATH=$PWD
cat > $O/dl.py <<'PY'
import json, torch, bench, bench_legs
pkg = bench.load_pkg()
print(json.dumps(bench_legs.dist_leg(pkg, torch.device('cuda:0'))))
PY
timeout -k 10 300 python -u $O/dl.py > $O/dist_leg.json 2> $O/dist_leg.err || { tail -5 $O/dist_leg.err; exit 1; }
cut -c1-700 $O/dist_leg.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 $O/dl.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -i "dist_push\|Name" $O/prof/run_kernel_stats.csv | cut -c1-200
