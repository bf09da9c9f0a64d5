#!/bin/bash
# screen-kernel chunk sweep: one short bench per k_chunk (results identical, only time differs)
for ck in ${CKS:-512 1024 2048 4096 8192}; do
  for v in ${VARIANTS:-0}; do
    timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-ge --steps 50 --k-chunk $ck --variant $v || exit $?
  done
done
