#!/bin/bash
# GPU box: GEMM/forward/quant parity after the split-K + dequant changes, then the default bench line.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_forward.py tests/test_gpu_quant.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02b_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 2 > gpurun_out/r02b_bench.json 2> gpurun_out/r02b_bench.err
