#!/bin/bash
# GPU box (round 6): mid-phase barriers + early fragment reads in attn2's f8c instances too (the build): attention and
# causal tests, then f8c launch times under the default kernel policy against lib/ab/khlate_st.so (barriers between phases).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6khab; mkdir -p $out
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k attention \
    > $out/test_attn_a2early.log 2>&1
rc=$?; echo "rc=$rc" >> $out/test_attn_a2early.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_text_encoder.py tests/test_gpu_parity_strict.py \
    > $out/test_te_strict_a2early.log 2>&1
rc=$?; echo "rc=$rc" >> $out/test_te_strict_a2early.log; [ $rc -gt 1 ] && exit $rc
KH=auto LIBS=khlate bash tools/gpu_r6_khab.sh
