#!/bin/bash
# Speculative chain: the repair passes read the stored path in 64-value chunks (no dependent
# global load per step).  Tests, then A/B against the previous build (AIY_HIP_LIB, _B).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r06_g22
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sim_par_gpu.py tests/test_sim_gpu.py tests/test_ge_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  SIM_MODES=-1 timeout -k 10 200 python -u tools/sim_bench.py > $O/new_$rep.log 2>&1 || { tail -5 $O/new_$rep.log; exit 1; }
  grep '"Na": 400\|"Na": 900' $O/new_$rep.log | sed 's/^/new /'
  SIM_MODES=-1 AIY_HIP_LIB=$PWD/aiyagari-replication_amd/libaiyagari_hip_B.so timeout -k 10 200 python -u tools/sim_bench.py > $O/old_$rep.log 2>&1 || { tail -5 $O/old_$rep.log; exit 1; }
  grep '"Na": 400\|"Na": 900' $O/old_$rep.log | sed 's/^/old /'
done
