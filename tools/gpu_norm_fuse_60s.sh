#!/bin/bash
# GPU box: the fused row norm at the short-sequence shape (60 s, configs[1]) on / off, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-lines --no-bf16-line --no-profile --seconds 60"
rm -f gpurun_out/nf60.log
for r in 1 2; do
  echo "on" >> gpurun_out/nf60.log
  ACE_MI_NORM_FUSE=1 timeout -k 10 240 $B 2>/dev/null | tail -1 >> gpurun_out/nf60.log || exit 1
  echo "off" >> gpurun_out/nf60.log
  timeout -k 10 240 $B 2>/dev/null | tail -1 >> gpurun_out/nf60.log || exit 1
done
