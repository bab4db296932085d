#!/bin/bash
# GPU box (round 6): the per-lane MFMA block-scale probe, then the f8c kernel's error pattern with and without attn_kh.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6khdiag; mkdir -p $out
timeout -k 10 60 tools/probe/mfma_scale_lane > $out/probe_scale_lane.txt 2>&1 || exit $?
for kh in 1 0; do
  for nk in 64 300; do
    ACE_MI_ATTN_KH=$kh NK=$nk timeout -k 10 120 python -u tools/diag_kh.py >> $out/diag.jsonl 2>> $out/diag.err || exit $?
  done
done
exit 0
