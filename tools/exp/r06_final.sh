#!/bin/bash
# Round 6 closing runs.  Part A: the GPU suite and the default bench (contract line + detail).
# Part B (PART=b): the bench's kernel-trace stats and the PMC / traffic passes of every timed kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06_final}
mkdir -p $O
if [ "${PART:-a}" = a ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 420 python -u bench.py --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  tail -c 400 $O/bench.out
else
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 bench.py --no-cpu-baseline --detail $O/prof_bench_detail.json > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
  TAG=$(basename $O)_pmc timeout -k 10 700 bash tools/exp/r06_pmc.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
  tail -12 $O/pmc.log
fi
