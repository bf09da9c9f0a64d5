#!/bin/bash
# Round 3 session 3: full GPU suite (no -x) after the MFMA tolerance fix and the one-pass EGM
# end-segment rework; EGM step A/B (one-pass vs two-launch) at Na = 20,000 and 4,099.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_s3b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -25 $O/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u - > $O/egm_ab.json 2> $O/egm_ab.err <<'PY'
import json, torch, bench, bench_legs
pkg = bench.load_pkg(); dev = torch.device("cuda:0")
out = {}
for Na in (20000, 4099):
    for var in (-1, 4096):
        r = bench_legs.egm_leg(pkg, dev, Na, variant=var)
        out[f"{Na}_{var}"] = {"us_per_step": r["us_per_step"], "solve": r["solve"]}
        rl = bench_legs.egm_leg(pkg, dev, Na, labor=True, variant=var)
        out[f"{Na}_{var}_labor"] = {"us_per_step": rl["us_per_step"], "solve": rl["solve"]}
print(json.dumps(out, indent=1))
PY
rc=$?; cat $O/egm_ab.json; tail -5 $O/egm_ab.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u - > $O/dist_runs.json 2> $O/dist_runs.err <<'PY'
import json, numpy as np, torch, bench
pkg = bench.load_pkg()
cal = pkg.calibration.aiyagari(Na=20000, shocks="rouwenhorst")
r = 0.04; w = pkg.calibration.wage(r, cal["alpha"], cal["delta"])
R = pkg.vfi_solve(np.zeros((cal["N"], 20000)), cal["a_grid"], cal["s"], cal["P"], r, w, cal["beta"], cal["sigma"], 1e-5, 1000)
idx = R["idx"] - 1
out = {}
for i in range(idx.shape[0]):
    L = np.bincount(idx[i], minlength=20000)
    out[i] = {"max": int(L.max()), "argmax": int(L.argmax()), "n_gt32": int((L > 32).sum()), "top": sorted(L.tolist())[-5:]}
print(json.dumps(out))
PY
rc=$?; cat $O/dist_runs.json; tail -5 $O/dist_runs.err; exit $rc
