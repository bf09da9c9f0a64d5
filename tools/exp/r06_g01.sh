#!/bin/bash
# Round 6, first GPU call: the one-launch staged KS sweep (three buffers, waits and publish in the
# launch), ADVICE r5 fixes (GE pool invalidate, wide split fences, opt-in chain exclusivity):
# the affected tests, then the one-GPU direct-schedule model (hand-off cost per sweep).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g01
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ks_staged_gpu.py tests/test_egm_gpu.py tests/test_ks_dist_gpu.py tests/test_ge_gpu.py tests/test_wide_gpu.py tests/test_sim_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u bench_ks.py --direct-model > $O/direct_model.json 2> $O/direct_model.err || { tail -5 $O/direct_model.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open("gpurun_out/r06_g01/direct_model.json").read().strip().splitlines()[-1])
h=d["handoff"]
print("slowest sweep ms", d["gpu_ms_per_sweep_slowest"], "improve", d["improve_ms_slowest"], "proj", d["projected_vfi_iteration_ms"])
print("handoff", {k: h[k] for k in ("shard","gpu_ms_per_sweep_with_handoff","handoff_us_per_sweep","timeouts","projected_vfi_iteration_ms","remote_columns","interior_columns","boundary_columns")})
PY
# EGM legs at Na = 400 / 20,000 (the one-workgroup solve at 400)
timeout -k 10 300 python -u - > $O/egm.json 2> $O/egm.err <<'PY' || { tail -5 $O/egm.err; exit 1; }
import json, sys, torch
sys.path.insert(0, ".")
import bench, bench_legs
pkg = bench.load_pkg()
dev = torch.device("cuda", 0)
out = {}
for lab in (False, True):
    for Na in (400, 1000):
        L = bench_legs.egm_leg(pkg, dev, Na, labor=lab, cpu_threads=1)
        out[f"{'labor_' if lab else ''}egm_Na{Na}"] = {k: L[k] for k in ("us_per_step", "single_step_dev", "solve")}
print(json.dumps(out))
PY
python -c "
import json; d=json.loads(open('gpurun_out/r06_g01/egm.json').read().strip().splitlines()[-1])
for k,v in d.items(): print(k, 'us/step', round(v['us_per_step'],3), 'single', round(v['single_step_dev']['us_per_step'],2), 'solve_ms', round(v['solve']['wall_ms'],3), v['solve']['iters'])"
