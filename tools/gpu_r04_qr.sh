#!/bin/bash
# GPU box: dequant-fused tiles after the buffer-load staging fix: the v21 Q4_K diagnostic, the quant suite (v21 Q4_K
# no longer skipped), whole-forward determinism of the forced register-dequant tiles, and the dense GEMM tests.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/qr; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/diag_v21.py > gpurun_out/qr/diag_v21.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_quant.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/qr/t_quant.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/diag_det_qr.py > gpurun_out/qr/det.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/qr/t_gemm.log 2>&1
