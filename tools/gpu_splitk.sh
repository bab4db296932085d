#!/bin/bash
# GPU box: split-K GEMM correctness (kernel tests) then TFLOP/s of the split variants at the DiT shapes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/sk_test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_msweep.py ${SK_VARIANTS:-4,7,204,207,1,201} ${SK_MS:-3000,750,1500} > gpurun_out/sk_sweep.log 2>&1
