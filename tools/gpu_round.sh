#!/bin/bash
# GPU-box script for one measurement round, stopping at the first crash / timeout:
#   1. parity suite, one pytest process per file (tools/gpu_tests.sh)
#   2. GEMM micro-bench, dense and dequant-fused (tools/gemm_bench.py)
#   3. bench.py line + rocprofv3 --kernel-trace --stats of the same command (tools/gpu_bench.sh)
#   4. HBM traffic from counter-only PMC passes (tools/gpu_pmc.sh)
#   5. bench.py with Q8_0 weights, end-to-end generate timing (tools/bench_generate.py), FP-vs-quantized
#      end-to-end quality (tools/eval_quant.py)
# Outputs under gpurun_out/; copy the summaries to be kept into profiles/.
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
bash tools/gpu_pmc.sh
rc=$?
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --qtype q8_0 > gpurun_out/bench_q8.json 2> gpurun_out/bench_q8.err
rc=$?; echo "bench q8 rc=$rc" >> gpurun_out/bench_q8.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python tools/bench_generate.py --seconds 10 240 --runs 2 > gpurun_out/bench_generate.json \
    2> gpurun_out/bench_generate.err
rc=$?; echo "bench_generate rc=$rc" >> gpurun_out/bench_generate.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python tools/eval_quant.py --seconds 10 > gpurun_out/eval_quant.json 2> gpurun_out/eval_quant.err
rc=$?; echo "eval_quant rc=$rc" >> gpurun_out/eval_quant.err
exit $rc
