#!/bin/bash
# Experiment: KS Howard with precomputed pwch coefficients (AIY_KS_QTEST: a separate coefficient
# pass before each fused sweep, Horner-only queries) — kernel times from a kernel trace of the
# N = 1 ks leg with and without; plus bit-exactness of the sharded solve with the knob on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g06
mkdir -p $O
# (the shared static Q buffer of the experiment races between concurrent shards: timing only)

for q in 0 1; do
  if [ $q = 1 ]; then export AIY_KS_QTEST=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof$q -o run -- python3 bench_ks.py > $O/ks$q.json 2> $O/ks$q.err || { tail -5 $O/ks$q.err; exit 1; }
done
python - <<'PY'
import csv, glob, json
for q in (0, 1):
    d = json.loads(open(f"gpurun_out/r06_g06/ks{q}.json").read().strip().splitlines()[-1])
    f = glob.glob(f"gpurun_out/r06_g06/prof{q}/**/run_kernel_stats.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "ks_" in r["Name"]]
    print("QTEST", q, "howard_ms_per_sweep", round(d["howard_ms_per_sweep"], 4), "improve_ms", round(d.get("improve_ms", 0), 3))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:5]:
        print("   ", r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
