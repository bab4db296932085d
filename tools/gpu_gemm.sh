#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -q -m gpu -k gemm > gpurun_out/kg.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/kg.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python tools/gemm_bench.py ${VARIANTS:-0,1,2,3} > gpurun_out/gemm_bench.log 2>&1
