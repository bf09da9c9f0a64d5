#!/bin/bash
# Experiment: KS fused Howard sweep dealt tile-major by XCD (AIY_KS_XCD) — bit-exactness of the
# KS suites with it on, then kernel times of the N = 1 ks leg off / on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g07
mkdir -p $O
AIY_KS_XCD=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ks_gpu.py tests/test_ks_dist_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for q in 0 1 0 1; do
  if [ $q = 1 ]; then export AIY_KS_XCD=1; else unset AIY_KS_XCD; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof$q -o run -- python3 bench_ks.py > $O/ks$q.json 2> $O/ks$q.err || { tail -5 $O/ks$q.err; exit 1; }
  python - $q <<'PY'
import csv, glob, json, sys
q = sys.argv[1]
d = json.loads(open(f"gpurun_out/r06_g07/ks{q}.json").read().strip().splitlines()[-1])
f = glob.glob(f"gpurun_out/r06_g07/prof{q}/**/run_kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "ks_" in r["Name"]]
print("XCD", q, "howard_ms_per_sweep", round(d["howard_ms_per_sweep"], 4), "improve_ms", round(d.get("improve_ms", 0), 3))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:3]:
    print("   ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
# KS panel prologue patch (tools/exp/r05_g63_ks_panel_prologue.patch) A/B: libaiyagari_hip_panelB.so
unset AIY_KS_XCD
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ks_panel_gpu.py > $O/panel_tests_base.log 2>&1 || { tail -20 $O/panel_tests_base.log; exit 1; }
AIY_HIP_LIB=$PWD/aiyagari-replication_amd/libaiyagari_hip_panelB.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ks_panel_gpu.py > $O/panel_tests_B.log 2>&1 || { tail -20 $O/panel_tests_B.log; exit 1; }
tail -1 $O/panel_tests_B.log
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench_panel.py --no-cpu > $O/panel_A$rep.json 2>&1 || exit 1
  AIY_HIP_LIB=$PWD/aiyagari-replication_amd/libaiyagari_hip_panelB.so timeout -k 10 200 python -u bench_panel.py --no-cpu > $O/panel_B$rep.json 2>&1 || exit 1
done
python - <<'PY'
import json
for tag in ("A", "B"):
    for rep in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/r06_g07/panel_{tag}{rep}.json").read().strip().splitlines()[-1])
        print(tag, rep, {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.items() if k in ("us_per_period", "value", "sim_us_per_period", "big_us_per_period")})
PY
