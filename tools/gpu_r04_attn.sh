#!/bin/bash
# GPU box: attention kernel tests (new kernel), attention micro-bench new vs round-3 kernel, one-layer parity per precision
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attention or attn" -x -q -m gpu --timeout 120 \
    --timeout-method thread > gpurun_out/attn_kernel_tests.log 2>&1 || { echo "kernel tests failed"; exit 1; }
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_modes_v2.jsonl 2>&1 || exit $?
ACE_MI_ATTN_V1=1 timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_modes_v1.jsonl 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_strict.py -k "one_layer and default" -v -s -m gpu --timeout 300 \
    --timeout-method thread > gpurun_out/one_layer.log 2>&1
