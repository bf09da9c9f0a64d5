set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02_s28
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_vfi_gpu.py tests/test_spec_solve_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
K='bell_tree_kernel<4, false, 1, 1, 1, false>'
timeout -k 10 300 rocprofv3 --kernel-trace -d $PWD/$O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra --no-ge --no-ks --no-panel > $O/bench.json 2> $O/bench.err || exit 1
python3 tools/prof_window.py $O/prof/run_kernel_trace.csv "$K" 5 20
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['roofline']['kernel_avg_ms'], d['ms_per_step'])"
