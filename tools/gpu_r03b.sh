#!/bin/bash
# Round 3: register-dequant GEMM (kernel tests, micro-bench, Q8_0 line fused vs staged) + loop / peaked diagnostics.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_quant.py -x > gpurun_out/quant.log 2>&1; rc=$?
echo "quant rc=$rc" >> gpurun_out/quant.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/gemm_q_bench.py 3000,750,125 -1,20,21,24 > gpurun_out/gemm_q_bench.jsonl 2> gpurun_out/gemm_q_bench.err || exit $?
ACE_MI_QUANT_STAGED=0 timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_q8_fused.json 2> gpurun_out/bench_q8_fused.err || exit $?
timeout -k 10 300 python tools/diag_loop.py > gpurun_out/diag_loop.log 2>&1 || exit $?
timeout -k 10 600 python tools/diag_peaked.py > gpurun_out/diag_peaked.log 2>&1 || exit $?
exit $rc
