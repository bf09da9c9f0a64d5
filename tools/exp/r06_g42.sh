#!/bin/bash
# Speculative chain: the in-order sum reads 16 values ahead into distinct registers (no readlane
# between dependent adds), vs HEAD (_B): sim suites, kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT SIM_MODES=-1,1
O=gpurun_out/r06_g42
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sim_par_gpu.py tests/test_sim_gpu.py tests/test_ge_gpu.py tests/test_ge_batch_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old; do
  if [ $v = old ]; then export AIY_HIP_LIB=$PWD/aiyagari-replication_amd/libaiyagari_hip_B.so; else unset AIY_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/prof_$v -o run -- python3 tools/sim_bench.py > $O/sim_$v.log 2>&1 || { tail -5 $O/sim_$v.log; exit 1; }
  grep '"Na": 400' $O/sim_$v.log | sed "s/^/$v /"
  grep -i "sim_par\|sim_chain_par" $O/prof_$v/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/$v /"
done
