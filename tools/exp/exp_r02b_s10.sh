#!/bin/bash
# PMC of the KS Howard and slopes kernels (bench_ks.py at the scaling size, N = 1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r02b_s10; mkdir -p $O
pass() { local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$PWD/$O/pmc/$name" -o run -- python3 "$PWD/bench_ks.py" --howard 10 > "$O/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$O/$name.log"; exit $rc; }; }
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass sq2 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
pass fetch FETCH_SIZE
pass write WRITE_SIZE
for k in ks_howard_kernel ks_slopes_cols_kernel; do
  python3 tools/pmc_summary.py $O/pmc "aiy::$k" $O/pmc_$k.json 3 0 > /dev/null && python3 -c "
import json; d=json.load(open('$O/pmc_$k.json')); print('$k', json.dumps(d['derived']))"
  python3 tools/pmc_traffic.py $O/pmc "aiy::$k" $O/traffic_$k.json 3 0 && true
done
exit 0
