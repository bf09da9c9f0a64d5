#!/bin/bash
# Round 3 session 2: GPU tests (KS (K,Z)-sliced ghost blocks, fused Howard+slopes, A10 plan +
# speculation, one-pass EGM scatter step), the launch-floor probe under rocprofv3, the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_s2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/probe -o run -- python3 tools/launch_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
python3 tools/launch_gaps.py $O/probe/run_kernel_trace.csv add_ egm_rhs egm_interp egm_fused egm_scatter > $O/launch_gaps.json && cat $O/launch_gaps.json
timeout -k 10 700 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench ok"
