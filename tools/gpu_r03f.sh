#!/bin/bash
# Round 3: determinism after the quantized picker change, short-M multi-stage tiles, bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 300 python tools/gemm_msweep.py 7,8,9,12,13,14,15,209,212,213 750,125 > gpurun_out/msweep_ns.jsonl 2> gpurun_out/msweep_ns.err || exit $?
timeout -k 10 300 python tools/gemm_msweep.py 7,14,15,4 3000 > gpurun_out/msweep_ns3000.jsonl 2> gpurun_out/msweep_ns3000.err || exit $?
timeout -k 10 300 python tools/diag_det.py > gpurun_out/diag_det2.log 2>&1 || exit $?
timeout -k 10 900 $T tests/test_gpu_quant.py tests/test_gpu_kernels.py > gpurun_out/quant_f.log 2>&1; rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r03f.json 2> gpurun_out/bench_r03f.err || exit $?
exit 0
