#!/bin/bash
# Round-2 (third session) closing artifacts: full GPU tests, smoke, bench, rocprof stats + window
# of the headline kernel, PMC passes (VALU/wait/occupancy and HBM traffic) over the timed sweeps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02c_final5}
mkdir -p $O
K='bell_tree_kernel<4, false, 1, 1, 1, false>'
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep -v amdgpu.ids $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench ok"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
python3 tools/prof_window.py $O/prof/run_kernel_trace.csv "$K" 5 20 > $O/prof_window.json && cat $O/prof_window.json
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv
PM="--no-cpu-baseline --no-extra --no-solve --no-ge --no-ks --no-panel --repeats 1 --steps 20 --warmup 5"
OUT=$O/pmc PASSES="sq sq2 grbm fetch write" BENCH_ARGS="$PM" timeout -k 10 600 bash tools/pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc "$K" $O/pmc_tree_final.json 5 20 > /dev/null && python3 tools/pmc_traffic.py $O/pmc "$K" $O/traffic_vfi_tree.json 5 20
echo "final done"
