#!/bin/bash
# GPU box (round 6): the EARLY variant of attn_kh_kernel (A/B self-test library lib/ab/khearly_st.so): attention tests
# through it, then launch times against the build (tools/gpu_r6_khab.sh).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6khab; mkdir -p $out
ACE_MI_SELFTEST_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/khearly_st.so timeout -k 10 300 python -u -m pytest -q -m gpu \
    --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k attention > $out/test_attn_early.log 2>&1
rc=$?; echo "rc=$rc" >> $out/test_attn_early.log; [ $rc -gt 1 ] && exit $rc
LIBS=khearly bash tools/gpu_r6_khab.sh
