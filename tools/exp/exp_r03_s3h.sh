#!/bin/bash
# Round 3 session 3: prefetched P/V/c rows (table, EGM, push kernels) — full GPU suite, the
# phase probe, the push trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03_s3h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -8 $O/pytest_gpu.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python -u tools/dist_trace.py $O/dist_trace.txt > /dev/null 2> $O/dist_trace.err || { tail -5 $O/dist_trace.err; exit 1; }
cat $O/dist_trace.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/probe -o run -- python3 tools/launch_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
python3 tools/phase_stats.py $O/probe/run_kernel_trace.csv $O/phase_stats.json > /dev/null && echo phases ok
