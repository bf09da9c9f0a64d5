#!/bin/bash
# A/B of the headline sweep between two builds of the library on one box (AIY_HIP_LIB): runs
# the headline-only bench alternately, ROUNDS times each, and prints one line per run.
#   LIBS="build_ab/libaiyagari_hip_base.so aiyagari-replication_amd/libaiyagari_hip.so" bash tools/ab_headline.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
O=${O:-gpurun_out/ab}
mkdir -p $O
ARGS=${ARGS:---no-cpu-baseline --no-ks --no-ge --no-panel --no-extra}
for rnd in $(seq 1 ${ROUNDS:-2}); do
  for L in $LIBS; do
    tag=$(basename $L .so)_$rnd
    AIY_HIP_LIB=$PWD/$L timeout -k 10 300 python3 bench.py $ARGS --detail $O/$tag.json > $O/$tag.out 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/$tag.out').read().strip().splitlines()[-1]); l=d.get('legs',{})
print('$tag', 'step_ms %.5f'%d['ms_per_step'], 'kern_ms %.5f'%d['roofline']['kernel_avg_ms'], 'frac %.4f'%d['roofline']['frac'], 'min %.5f max %.5f'%(d['repeats']['min_ms_per_step'], d['repeats']['max_ms_per_step']), 'solve_ms', l.get('solve_to_tol',{}).get('wall_ms'))"
  done
done
