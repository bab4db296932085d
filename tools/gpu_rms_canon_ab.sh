#!/bin/bash
# GPU box: the standalone row norm in the canonical summation order (default) against the round-4 kernels
# (ACE_MI_RMSNORM_LEGACY=1), whole bench lines at 60 s and 240 s, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-lines --no-bf16-line --no-profile"
rm -f gpurun_out/rms_ab.log
for r in 1 2; do
  for sec in 60 240; do
    echo "sec=$sec canon" >> gpurun_out/rms_ab.log
    timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 >> gpurun_out/rms_ab.log || exit 1
    echo "sec=$sec legacy" >> gpurun_out/rms_ab.log
    ACE_MI_RMSNORM_LEGACY=1 timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 >> gpurun_out/rms_ab.log || exit 1
  done
done
