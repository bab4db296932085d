#!/bin/bash
# GPU box: dequant-fused GEMM stress (tools/diag_gemm_q.py), the quantized parity tests, and an A/B of the
# q8_0 GEMM rates between lib/ab/base.so and lib/ab/new.so.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
STRESS_REPS=${STRESS_REPS:-40} timeout -k 10 400 python -u tools/diag_gemm_q.py > gpurun_out/diag_q.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_quant.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/quant.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/quant.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
NAMES="base new" ROUNDS=2 AB_CMD="tools/gemm_bench.py 5,7 q8_0" bash tools/ab_multi.sh
