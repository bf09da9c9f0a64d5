#!/bin/bash
# GPU-call runner: tools/run_steps.sh OUTDIR "name|seconds|command" ...
# Each step runs under its own `timeout -k 10`, output to OUTDIR/name.log; the call stops at the
# first step that does not exit 0 (a failing test, a fault, an abort or a time limit alike), so
# nothing more runs on the GPU after trouble.
out=$1; shift
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; to=${rest%%|*}; cmd=${rest#*|}
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "$out/$name.log"
  if [ $rc -ne 0 ]; then echo "=== stop after $name (rc $rc)"; exit $rc; fi
done
