#!/bin/bash
# PMC passes over a short bench run, one counter group per pass (gfx950 slot limits:
# <= 8 SQ, <= 4 TCC (FETCH_SIZE uses 3, WRITE_SIZE 2), <= 2 GRBM).  Each pass is KILL-bounded.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
ARGS=${BENCH_ARGS:---no-cpu-baseline --no-ge --steps 3 --warmup 2}
CMD=${PMC_CMD:-$PWD/bench.py}  # the program each pass profiles (bench.py $ARGS by default)
mkdir -p "$OUT"
pass() {  # name, counters...
  local name=$1; shift
  echo "=== pmc $name: $*"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$PWD/$OUT/$name" -o run -- python3 $CMD $ARGS > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
}
for ps in ${PASSES:-sq sq2 grbm fetch write}; do
  case $ps in
    sq)    pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU ;;
    sq2)   pass sq2 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA ;;
    grbm)  pass grbm GRBM_GUI_ACTIVE GRBM_COUNT ;;
    fetch) pass fetch FETCH_SIZE ;;
    write) pass write WRITE_SIZE ;;
  esac
done
echo "=== pmc done"
