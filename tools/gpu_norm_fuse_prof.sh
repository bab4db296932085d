#!/bin/bash
# GPU box: where the fused row norm's time goes -- bench lines of the 240 s loop with their per-kernel breakdown
# (HIP events of the profiled call), fusion on / off, and different waits before a tile hands its rows over
# (ACE_MI_NORM_SPIN_US)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/nfp; export TMPDIR=/tmp
B="python -u bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-extra-lines --no-bf16-line --seconds 240"
rm -f gpurun_out/nfp/lines.log
echo "on" >> gpurun_out/nfp/lines.log
ACE_MI_NORM_FUSE=1 timeout -k 10 240 $B 2>/dev/null | tail -1 >> gpurun_out/nfp/lines.log || exit 1
echo "off" >> gpurun_out/nfp/lines.log
ACE_MI_NORM_FUSE=0 timeout -k 10 240 $B 2>/dev/null | tail -1 >> gpurun_out/nfp/lines.log || exit 1
for sp in 0 5 200; do
  echo "spin=$sp" >> gpurun_out/nfp/lines.log
  ACE_MI_NORM_FUSE=1 ACE_MI_NORM_SPIN_US=$sp timeout -k 10 240 $B 2>/dev/null | tail -1 >> gpurun_out/nfp/lines.log || exit 1
done
