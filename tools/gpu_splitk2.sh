#!/bin/bash
# GPU box: TFLOP/s of the short-sequence tiles with and without split-K (tools/gemm_msweep.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u tools/gemm_msweep.py ${SK_VARIANTS} ${SK_MS} > gpurun_out/sk_sweep2.log 2>&1
