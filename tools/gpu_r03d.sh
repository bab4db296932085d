#!/bin/bash
# Round 3: residual-prefetch GEMM (kernel tests + sweep + bench), determinism diagnostics.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kernels.py > gpurun_out/kernels.log 2>&1; rc=$?
echo "kernels rc=$rc" >> gpurun_out/kernels.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/gemm_msweep.py 7,8,9,1 3000,750 > gpurun_out/msweep_xpf.jsonl 2> gpurun_out/msweep_xpf.err || exit $?
timeout -k 10 300 python tools/gemm_q_bench.py 3000,750,125 -1,21,22 > gpurun_out/gemm_q_bench3.jsonl 2> gpurun_out/gemm_q_bench3.err || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r03d.json 2> gpurun_out/bench_r03d.err || exit $?
timeout -k 10 300 python tools/diag_loop.py > gpurun_out/diag_loop3.log 2>&1 || exit $?
exit $rc
