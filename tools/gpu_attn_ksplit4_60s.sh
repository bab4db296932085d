#!/bin/bash
# GPU box: the short-range key split (ACE_MI_ATTN_KSPLIT=4, merge launches) against the default at 60 s, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-lines --no-bf16-line --no-profile --seconds 60"
rm -f gpurun_out/ks4_60.log
for r in 1 2; do
  echo "ksplit4" >> gpurun_out/ks4_60.log
  ACE_MI_ATTN_KSPLIT=4 timeout -k 10 240 $B 2>/dev/null | tail -1 >> gpurun_out/ks4_60.log || exit 1
  echo "default" >> gpurun_out/ks4_60.log
  timeout -k 10 240 $B 2>/dev/null | tail -1 >> gpurun_out/ks4_60.log || exit 1
done
