#!/bin/bash
# Round 3: skinny GEMM (M <= 128) tests and the 10 s / 60 s lines.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kernels.py -k "skinny or all_variants" > gpurun_out/skinny_k.log 2>&1 || exit $?
timeout -k 10 900 $T tests/test_gpu_forward.py > gpurun_out/forward_k.log 2>&1; rc=$?
[ $rc -gt 1 ] && exit $rc
B="bench.py --steps 27 --warmup 3 --no-extra-lines --no-bf16-line --no-cpu-baseline --qtype bf16"
for sec in 10 60; do
  timeout -k 10 300 python $B --seconds $sec > gpurun_out/k_${sec}.json 2> gpurun_out/k_${sec}.err || exit $?
done
ACE_MI_BENCH_COLD=24 timeout -k 10 300 python tools/gemm_msweep.py 7,9,13,208,213,214,215,408,412,413 750,500 > gpurun_out/msweep_cold60.jsonl 2> gpurun_out/msweep_cold60.err || exit $?
exit 0
