#!/bin/bash
# GPU box: attention tests with the in-kernel key-split merge (ACE_MI_ATTN_FUSED_MERGE=1, alone and with the
# short-range split ACE_MI_ATTN_KSPLIT=4), then bench lines at 60 s and 240 s against the default, interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="tests/test_gpu_kernels.py tests/test_gpu_parity_strict.py"
timeout -k 10 300 python -u -m pytest $T -k "attention or attn" -x -q -m gpu --timeout 200 --timeout-method thread \
    > gpurun_out/fm_tests_default.log 2>&1 || exit 1
ACE_MI_ATTN_FUSED_MERGE=1 timeout -k 10 300 python -u -m pytest $T -k "attention or attn" -x -q -m gpu --timeout 200 \
    --timeout-method thread > gpurun_out/fm_tests_fm.log 2>&1 || exit 1
ACE_MI_ATTN_FUSED_MERGE=1 ACE_MI_ATTN_KSPLIT=4 timeout -k 10 300 python -u -m pytest $T -k "attention or attn" -x -q -m gpu \
    --timeout 200 --timeout-method thread > gpurun_out/fm_tests_fm4.log 2>&1 || exit 1
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-lines --no-bf16-line --no-profile"
rm -f gpurun_out/fm_lines.log
for r in 1 2; do
  for sec in 60 240; do
    echo "sec=$sec base" >> gpurun_out/fm_lines.log
    timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 >> gpurun_out/fm_lines.log || exit 1
    echo "sec=$sec fm" >> gpurun_out/fm_lines.log
    ACE_MI_ATTN_FUSED_MERGE=1 timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 >> gpurun_out/fm_lines.log || exit 1
    echo "sec=$sec fm4" >> gpurun_out/fm_lines.log
    ACE_MI_ATTN_FUSED_MERGE=1 ACE_MI_ATTN_KSPLIT=4 timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 \
        >> gpurun_out/fm_lines.log || exit 1
  done
done
