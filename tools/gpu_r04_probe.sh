#!/bin/bash
# GPU box: one-layer literal-bound parity in every attention precision + attention micro-bench per mode
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/attn_bench.py > gpurun_out/attn_modes.jsonl 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_strict.py -k "one_layer and default" -v -s -m gpu --timeout 300 \
    --timeout-method thread > gpurun_out/one_layer.log 2>&1
