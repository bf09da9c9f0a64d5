set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_s23
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_labor_gpu.py tests/test_batch_gpu.py > gpurun_out/r02_s23/pytest.log 2>&1 || { tail -30 gpurun_out/r02_s23/pytest.log; exit 1; }
tail -2 gpurun_out/r02_s23/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ge --no-ks --no-panel --no-extra > gpurun_out/r02_s23/bench.log 2>&1
python3 - <<'PY'
import json
for l in open('gpurun_out/r02_s23/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('value %.4g step %.2f us kernel %.2f us frac %.4f solve %.2f ms' % (d['value'], d['ms_per_step']*1e3, d['roofline']['kernel_avg_ms']*1e3, d['roofline']['frac'], d['solve_to_tol']['wall_ms']))
PY
timeout -k 10 120 python -u tools/tree_trace.py 20000 16 > gpurun_out/r02_s23/trace.txt 2>&1
