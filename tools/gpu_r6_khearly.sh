#!/bin/bash
# GPU box (round 6): attn_kh_kernel with mid-phase barriers and early fragment reads (the build) -- attention and causal
# tests, then launch times against the A/B self-test library lib/ab/khlate_st.so (barriers between the phases).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6khab; mkdir -p $out
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k attention \
    > $out/test_attn_early.log 2>&1
rc=$?; echo "rc=$rc" >> $out/test_attn_early.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_text_encoder.py -k causal \
    > $out/test_causal_early.log 2>&1
rc=$?; echo "rc=$rc" >> $out/test_causal_early.log; [ $rc -gt 1 ] && exit $rc
LIBS=khlate bash tools/gpu_r6_khab.sh
