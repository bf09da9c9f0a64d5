#!/bin/bash
# Staged KS sweep with its interior rows dealt tile-major by XCD: KS staged / dist / KS suites
# bit-exact, the one-GPU probe (worst shard), and the bench_ks direct model (hand-off).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g34
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ks_staged_gpu.py tests/test_ks_dist_gpu.py tests/test_ks_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 200 python3 tools/ks_staged_probe.py > $O/p_$rep.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  echo "rep=$rep $(tail -1 $O/p_$rep.json | cut -c1-220)"
done
timeout -k 10 300 python3 bench_ks.py > $O/ks.json 2> $O/ks.err || { tail -5 $O/ks.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/ks.json').read().strip().splitlines()[-1]); m=d['direct_model']
print('howard_ms', round(d['howard_ms_per_sweep'],4), 'vfi_ms', round(d['vfi_iteration_ms'],3), 'proj', round(m['projected_vfi_iteration_ms'],3), 'handoff', {k: m['handoff'][k] for k in ('handoff_us_per_sweep','gpu_ms_per_sweep_with_handoff','projected_vfi_iteration_ms')})"
