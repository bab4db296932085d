#!/bin/bash
# GPU box (round 6): f8c attention launch times at the DiT shapes, attn_kh_kernel (ACE_MI_ATTN_KH=1) against attn2 (0),
# then the rocprofv3 kernel trace of the self-full case for both.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6khperf; mkdir -p $out
for r in 1 2; do for kh in 1 0; do
  ACE_MI_ATTN_KH=$kh ATTN_MODES=f8c timeout -k 10 180 python -u tools/attn_bench.py >> $out/attn_bench.jsonl 2>> $out/err.txt || exit $?
done; done
for kh in 1 0; do
  ACE_MI_ATTN_KH=$kh ATTN_CASE="self_full 240s" ATTN_MODE=f8c timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_kh$kh" -o k --output-format csv -- python -u tools/attn_bench.py >> $out/prof.log 2>&1 || exit $?
done
exit 0
