#!/bin/bash
# Round 3: uncontracted Euler / rounding helpers, persistent rmsnorm_mod, multi-stage short-sequence GEMM tiles.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_quant.py > gpurun_out/quant_e.log 2>&1 || exit $?
timeout -k 10 300 python tools/diag_loop.py > gpurun_out/diag_loop4.log 2>&1 || exit $?
timeout -k 10 600 $T tests/test_gpu_kernels.py tests/test_gpu_forward.py > gpurun_out/kernels_e.log 2>&1 || exit $?
timeout -k 10 300 python tools/gemm_msweep.py 7,8,9,12,13,209,212,213 750,125 > gpurun_out/msweep_ns.jsonl 2> gpurun_out/msweep_ns.err || exit $?
timeout -k 10 900 $T tests/test_gpu_configs.py > gpurun_out/configs_e.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r03e.json 2> gpurun_out/bench_r03e.err || exit $?
