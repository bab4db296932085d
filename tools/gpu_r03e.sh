#!/bin/bash
# Round 3: forward state-dependence diagnostic, multi-stage short-sequence GEMM tiles, skewed quantized pipeline.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/diag_state.py > gpurun_out/diag_state.log 2>&1 || exit $?
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kernels.py -k "gemm" > gpurun_out/kernels_e.log 2>&1 || exit $?
timeout -k 10 600 $T tests/test_gpu_quant.py > gpurun_out/quant_e.log 2>&1 || exit $?
timeout -k 10 300 python tools/gemm_msweep.py 7,8,9,12,13,209,212,213 750,125 > gpurun_out/msweep_ns.jsonl 2> gpurun_out/msweep_ns.err || exit $?
timeout -k 10 300 python tools/gemm_q_bench.py 3000,750 -1,20,21,22 > gpurun_out/gemm_q_bench4.jsonl 2> gpurun_out/gemm_q_bench4.err || exit $?
