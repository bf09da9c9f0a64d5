#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.  Each GPU step has its
# own time limit; a fault/abort/timeout (exit >= 124 or a signal) ends the session at once.
# Test FAILURES (pytest exit 1) do not stop later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ] || [ "$rc" -gt 128 ]; }
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
echo "host: $(nproc) cpus, OMP_NUM_THREADS=$OMP_NUM_THREADS"; rocm-smi --showproductname 2>/dev/null | grep -i -m2 "card\|gfx" || true
for s in ${STEPS:-tests smoke bench prof}; do
  case $s in
    tests) if [ -n "$PYTEST_K" ]; then step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$PYTEST_K";
           else step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread; fi ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python -u bench.py ${BENCH_ARGS} ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o run -- python3 "$PWD/bench.py" --no-cpu-baseline --no-ge --no-solve ${BENCH_ARGS} ;;
    pmc)   PMC_ARGS="--no-cpu-baseline --no-ge --no-solve --no-ks --steps 20 --warmup 5"
           step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/$OUT/pmc/fetch" -o run -- python3 "$PWD/bench.py" $PMC_ARGS
           step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/$OUT/pmc/write" -o run -- python3 "$PWD/bench.py" $PMC_ARGS
           python3 tools/pmc_traffic.py "$OUT/pmc" bell_tree_kernel "$OUT/traffic_vfi_tree.json" ;;
    custom) step custom 600 bash -c "$CUSTOM" ;;
  esac
done
echo "=== done"
