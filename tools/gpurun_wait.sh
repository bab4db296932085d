#!/bin/bash
# Host side: submit one gpurun call, re-submitting only while the pool reports no free box / back-off (nothing ran,
# nothing charged); any other outcome (success or a real failure) ends it.  Usage: tools/gpurun_wait.sh OUT TIMEOUT CMD
out=$1; lim=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  rc=$?
  if grep -qE "no free box right now|backing off|are busy|retry in a few minutes" "$out"; then sleep 150; continue; fi
  exit $rc
done
exit 3
