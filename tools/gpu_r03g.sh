#!/bin/bash
# Round 3: attention 4-part key split, cold-weight GEMM sweep, quantized tests, kernel-trace of the 60 s / 10 s loops (GPU busy vs wall).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kernels.py -k "attention" > gpurun_out/attn_g.log 2>&1 || exit $?
ACE_MI_BENCH_COLD=24 timeout -k 10 300 python tools/gemm_msweep.py 4,7,8,9,209 3000,750,125 > gpurun_out/msweep_cold.jsonl 2> gpurun_out/msweep_cold.err || exit $?
timeout -k 10 900 $T tests/test_gpu_quant.py > gpurun_out/quant_g.log 2>&1; rc=$?
[ $rc -gt 1 ] && exit $rc
B="bench.py --steps 27 --warmup 3 --no-extra-lines --no-bf16-line --no-cpu-baseline --qtype bf16 --no-profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof60 -o prof60 -- python $B --seconds 60 > gpurun_out/prof60.json 2> gpurun_out/prof60.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof10 -o prof10 -- python $B --seconds 10 > gpurun_out/prof10.json 2> gpurun_out/prof10.err || exit $?
exit 0
