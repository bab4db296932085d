#!/bin/bash
# Round 3: bf16 images of the non-block quantized weights (condition, cross k|v, proj in/out): quantized tests,
# configs tests, final bench line.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_quant.py > gpurun_out/quant_l.log 2>&1; rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 900 $T tests/test_gpu_configs.py > gpurun_out/configs_l.log 2>&1; rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_l.json 2> gpurun_out/bench_l.err || exit $?
exit 0
