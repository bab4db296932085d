#!/bin/bash
# GPU box: GEMM kernel tests (residual epilogues of every tile), forward / quant parity, then the bs=8 line
# (8-wave residual tiles) and the default bench line + rocprofv3 stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SUITES="kernels:400 forward:900 quant:900" bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --batch-per-gpu 8 --no-cpu-baseline > gpurun_out/bench_bs8_q8.json 2> gpurun_out/bench_bs8_q8.err || exit $?
STEPS=27 bash tools/gpu_bench.sh || exit $?
exit $rc
