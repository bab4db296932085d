#!/bin/bash
# Round 3: in-kernel key-split merge (attention), cold sweep of the multi-stage tiles, 60 s / 10 s kernel traces.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_forward.py > gpurun_out/forward_h.log 2>&1; rc=$?
[ $rc -gt 1 ] && exit $rc
ACE_MI_BENCH_COLD=24 timeout -k 10 300 python tools/gemm_msweep.py 7,8,9,12,13,209,212,213 750,125 > gpurun_out/msweep_cold_ns.jsonl 2> gpurun_out/msweep_cold_ns.err || exit $?
B="bench.py --steps 27 --warmup 3 --no-extra-lines --no-bf16-line --no-cpu-baseline --qtype bf16 --no-profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof60b -o prof60b -- python $B --seconds 60 > gpurun_out/prof60b.json 2> gpurun_out/prof60b.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof10b -o prof10b -- python $B --seconds 10 > gpurun_out/prof10b.json 2> gpurun_out/prof10b.err || exit $?
timeout -k 10 300 python $B --seconds 60 > gpurun_out/b60_h.json 2> gpurun_out/b60_h.err || exit $?
exit 0
