#!/bin/bash
# (not applied: the patch tools/exp/r05_g63_ks_panel_prologue.patch; no GPU box could be prepared before the session ended)
# KS panel step: grid and first-agent loads in flight together (one round trip instead of three).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g63
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ks_panel_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-ge --no-ks --no-extra --no-solve --detail $O/b.json > $O/b.out 2>&1 || { tail -5 $O/b.out; exit 1; }
python - <<'PY'
import json
d=json.loads([l for l in open("gpurun_out/r05_g63/b.out") if l.startswith("{")][-1])
print(json.dumps(d["legs"].get("ks_panel"))[:400])
PY
