#!/bin/bash
# GPU box: quantized parity (kernel + forward tests, BASELINE configs q8_0 / q4_k), then the default bench
# line (configs[2], Q8_0, with the bf16 line beside it) and its rocprof kernel stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_quant.py -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/quant.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/quant.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -q -s -m gpu -x -k "quantized" --timeout 500 --timeout-method thread > gpurun_out/configs_q.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/configs_q.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
STEPS=${STEPS:-20} BENCH_ARGS="--no-cpu-baseline ${BENCH_ARGS}" bash tools/gpu_bench.sh
