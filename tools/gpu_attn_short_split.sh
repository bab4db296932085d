#!/bin/bash
# GPU box: attention tests, then the short-range key split as the default for under-filled grids against the previous
# rule (ACE_MI_ATTN_KSPLIT=3: the previous rule; the long-range rule is unchanged) at 10 s / 60 s / 240 s
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity_strict.py -k "attention or attn" -x -q -m gpu \
    --timeout 200 --timeout-method thread > gpurun_out/ss_tests.log 2>&1 || exit 1
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-lines --no-bf16-line --no-profile"
rm -f gpurun_out/ss_lines.log
for r in 1 2; do
  for sec in 10 60 240; do
    echo "sec=$sec new" >> gpurun_out/ss_lines.log
    timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 >> gpurun_out/ss_lines.log || exit 1
    echo "sec=$sec old" >> gpurun_out/ss_lines.log
    ACE_MI_ATTN_KSPLIT=3 timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 >> gpurun_out/ss_lines.log || exit 1
  done
done
