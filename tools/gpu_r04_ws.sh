#!/bin/bash
# GPU box: warp-specialized GEMM tile (variants 18 / 19): bit identity + GEMM tests, then the TFLOP/s table.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ws; export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "bit_identical" --timeout 60 --timeout-method thread > gpurun_out/ws/t_ident.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread > gpurun_out/ws/t_gemm.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -x -q -m gpu -k "fused_qkv_prep" --timeout 200 --timeout-method thread > gpurun_out/ws/t_prep.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/gemm_bench.py 4,7,18,19 > gpurun_out/ws/bench.jsonl 2>&1
