#!/bin/bash
# GPU box (round 6): the two-waves-per-SIMD f8c attention kernel (attn_kh_kernel): attention tests, the one-layer
# literal parity tests, then headline-only bench lines alternating the default policy / ACE_MI_ATTN_KH=0 (attn2).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6kh; mkdir -p $out
for kh in 1 0; do ACE_MI_ATTN_KH=$kh NK=300 timeout -k 10 120 python -u tools/diag_kh.py >> $out/diag.jsonl 2>> $out/diag.err || exit $?; done
P="python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 400 $P tests/test_gpu_kernels.py -k attention > $out/test_attn.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_attn.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 400 $P tests/test_gpu_parity_strict.py > $out/test_strict.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_strict.log; [ $rc -gt 1 ] && exit $rc
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile --no-bf16-line --no-extra-lines"
for r in 1 2; do
  for kh in auto 0; do
    echo -n "kh=$kh " >> $out/lines.txt
    ACE_MI_ATTN_KH=$kh timeout -k 10 240 $B 2>> $out/bench.err | tail -1 >> $out/lines.txt || exit 1
  done
done
exit 0
