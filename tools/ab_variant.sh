#!/bin/bash
# A/B of the headline sweep between tree variants on one box: headline-only bench per variant,
# alternated ROUNDS times; one line per run.   VARS="16 80" ROUNDS=3 bash tools/ab_variant.sh
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
export TMPDIR=/tmp
O=${O:-gpurun_out/abv}
mkdir -p $O
ARGS=${ARGS:---no-cpu-baseline --no-ks --no-ge --no-panel --no-extra}
for rnd in $(seq 1 ${ROUNDS:-2}); do
  for V in $VARS; do
    tag=v${V}_$rnd
    timeout -k 10 300 python3 bench.py $ARGS --variant $V --detail $O/$tag.json > $O/$tag.out 2> $O/$tag.err || { tail -5 $O/$tag.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/$tag.out').read().strip().splitlines()[-1]); l=d.get('legs',{})
print('$tag', 'step_ms %.5f'%d['ms_per_step'], 'kern_ms %.5f'%d['roofline']['kernel_avg_ms'], 'frac %.4f'%d['roofline']['frac'], 'min %.5f max %.5f'%(d['repeats']['min_ms_per_step'], d['repeats']['max_ms_per_step']), 'solve_ms', l.get('solve_to_tol',{}).get('wall_ms'))"
  done
done
