#!/bin/bash
# GPU box: the pv8 attention mode (fp16 Q.K, f8c P.V): attention kernel tests, strict parity (one-layer literal bound,
# peaked logits) for pv8 and f8c, and the attention micro-benchmark of every mode.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pv8; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -v -m gpu -k "attention" --timeout 120 --timeout-method thread > gpurun_out/pv8/t_attn.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_strict.py -v -s -m gpu -k "pv8 or f8c" --timeout 200 --timeout-method thread > gpurun_out/pv8/t_parity.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/pv8/attn_modes.jsonl 2>&1
