set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_s22
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ge --no-ks --no-panel --no-extra > gpurun_out/r02_s22/bench.log 2>&1
python3 - <<'PY'
import json
for l in open('gpurun_out/r02_s22/bench.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'], d['repeats'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d.get('solve_to_tol'))
PY
