#!/bin/bash
# KS Howard: the budget term log(max(c, 1e-10)) cached by the improvement (validated by the k_opt
# bits) vs HEAD (_B): KS suites bit-exact, then the N = 1 ks leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g36
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ks_gpu.py tests/test_ks_dist_gpu.py tests/test_ks_staged_gpu.py tests/test_mex_gpu.py tests/test_ks_panel_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old new old; do
  if [ $v = old ]; then export AIY_HIP_LIB=$PWD/aiyagari-replication_amd/libaiyagari_hip_B.so; else unset AIY_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof_$v -o run -- python3 bench_ks.py > $O/ks_$v.json 2> $O/ks_$v.err || { tail -5 $O/ks_$v.err; exit 1; }
  python - $v <<'PY'
import csv, glob, json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/r06_g36/ks_{v}.json").read().strip().splitlines()[-1])
f = glob.glob(f"gpurun_out/r06_g36/prof_{v}/**/run_kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "ks_" in r["Name"]]
print(v, "howard_ms_per_sweep", round(d["howard_ms_per_sweep"], 4), "improve_ms", round(d.get("improve_ms", 0), 3), "vfi_iteration_ms", round(d.get("vfi_iteration_ms", 0), 3))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:3]:
    print("   ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
done
