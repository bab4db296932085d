#!/bin/bash
# GPU-box script: kernel + forward parity tests, GEMM micro-bench (dense + quantized),
# bench bf16 (+ rocprofv3 kernel stats), bench Q8_0.  Stops at the first crash/timeout.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/gemm_bench.py 1,2,3 ,q8_0,q4_k > gpurun_out/gemm_bench.log 2>&1
rc=$?; echo "gemm_bench rc=$rc" >> gpurun_out/gemm_bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_bench.sh
rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --qtype q8_0 > gpurun_out/bench_q8.json 2> gpurun_out/bench_q8.err
rc=$?; echo "bench q8 rc=$rc" >> gpurun_out/bench_q8.err
exit $rc
