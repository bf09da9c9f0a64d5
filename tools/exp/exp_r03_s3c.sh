#!/bin/bash
# Round 3 session 3: launch/phase attribution (tools/launch_probe.py under rocprofv3), then the
# GPU suite on the EGM default flip and the NaN-aware KS slope test.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_s3c}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/probe -o run -- python3 tools/launch_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
python3 tools/phase_stats.py $O/probe/run_kernel_trace.csv $O/phase_stats.json > /dev/null && echo phases ok
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "egm or ks_gpu or mfma" > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; exit $rc
