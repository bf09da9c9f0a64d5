#!/bin/bash
# Tree kernel: every kernel argument it reads in the start-up batch (best0, idx0, tw, ntile, the grid size,
# the output pointers): tree/VFI tests, then the headline + solve legs twice and kernel-trace stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r05_g61
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vfi_gpu.py tests/test_pinned_gpu.py tests/test_vfi_large_gpu.py tests/test_ev_mfma_gpu.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
FL="--no-cpu-baseline --no-ge --no-ks --no-panel --no-extra"
for rep in 1 2; do
timeout -k 10 200 python -u bench.py $FL --detail $O/h_$rep.json > $O/h_$rep.out 2>&1 || { tail -5 $O/h_$rep.out; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof -o run -- python3 bench.py $FL --detail $O/prof_detail.json > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python - <<'PY'
import csv,glob,json
for tag in ("h_1","h_2"):
    d=json.loads([l for l in open(f"gpurun_out/r05_g61/{tag}.out") if l.startswith("{")][-1])
    print(tag, "step_us", round(d["ms_per_step"]*1e3,2), "solve_ms", d["legs"].get("solve_to_tol",{}).get("wall_ms"))
f=glob.glob("gpurun_out/r05_g61/prof/**/run_kernel_stats.csv",recursive=True)
rows=list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:5]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,2))
PY
