set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_s27
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_labor_gpu.py tests/test_pinned_gpu.py > gpurun_out/r02_s27/pytest.log 2>&1 || { tail -30 gpurun_out/r02_s27/pytest.log; exit 1; }
tail -2 gpurun_out/r02_s27/pytest.log
timeout -k 10 300 python -u tools/labor_bench.py 400 20000
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ge --no-ks --no-panel --no-extra > gpurun_out/r02_s27/bench.log 2>&1
python3 - <<'PY'
import json
for l in open('gpurun_out/r02_s27/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print('value %.4g step %.2f us (median %.2f) kernel %.2f us frac %.4f solve %.2f ms' % (d['value'], d['ms_per_step']*1e3, d['repeats']['median_ms_per_step']*1e3, d['roofline']['kernel_avg_ms']*1e3, d['roofline']['frac'], d['solve_to_tol']['wall_ms']))
PY
