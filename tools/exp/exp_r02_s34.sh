set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_s34
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_batch_gpu.py tests/test_spec_solve_gpu.py tests/test_labor_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --no-ge --no-ks --no-panel > $O/bench.json 2>&1
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['repeats']['median_ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['solve_to_tol']['wall_ms'])"
timeout -k 10 300 python -u tools/ge_timing.py
