#!/bin/bash
# Round 4: the GPU suite at the packed-workgroup default (2 one-wave tiles per workgroup), the default bench, its
# kernel-trace stats, and the PMC/traffic passes of the timed kernels on the final code
# (headline tree over bench sweeps 6..25; EGM chain / KS Howard / dist push over
# tools/pmc_workloads_r04.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04_g16}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --detail $O/bench_detail.json > $O/bench.out 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
tail -c 600 $O/bench.out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 bench.py --no-cpu-baseline --detail $O/prof_bench_detail.json > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
OUT=$O/pmc_tree PASSES="sq sq2 fetch write" BENCH_ARGS="--no-cpu-baseline --no-ge --no-solve --no-ks --no-panel --no-extra --steps 20 --warmup 5 --repeats 1" bash tools/pmc.sh > $O/pmc_tree.log 2>&1 || { tail -5 $O/pmc_tree.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_tree bell_tree_kernel $O/pmc_tree.json 5 20 > /dev/null
python3 tools/pmc_traffic.py $O/pmc_tree bell_tree_kernel $O/traffic_vfi_tree.json 5 20 > /dev/null
OUT=$O/pmc_w PASSES="sq sq2 fetch write" PMC_CMD=$PWD/tools/pmc_workloads_r04.py BENCH_ARGS="" bash tools/pmc.sh > $O/pmc_w.log 2>&1 || { tail -5 $O/pmc_w.log; exit 1; }
python3 tools/pmc_summary.py $O/pmc_w egm_chain_kernel $O/pmc_egm_chain.json 0 200 > /dev/null
python3 tools/pmc_traffic.py $O/pmc_w egm_chain_kernel $O/traffic_egm_chain.json 0 200 > /dev/null
python3 tools/pmc_summary.py $O/pmc_w egm_chain_kernel $O/pmc_labor_egm_chain.json 200 200 > /dev/null
python3 tools/pmc_traffic.py $O/pmc_w egm_chain_kernel $O/traffic_labor_egm_chain.json 200 200 > /dev/null
for f in $O/pmc_tree.json $O/traffic_vfi_tree.json $O/traffic_egm_chain.json $O/traffic_labor_egm_chain.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', json.dumps(d.get('derived', d))[:400])"; done
