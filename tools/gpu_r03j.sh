#!/bin/bash
# Round 3: cold sweep of split / multi-stage tiles at the 60 s shapes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ACE_MI_BENCH_COLD=24 timeout -k 10 300 python tools/gemm_msweep.py 7,9,13,208,213,214,215,408,412,413 750,500 > gpurun_out/msweep_cold60.jsonl 2> gpurun_out/msweep_cold60.err || exit $?
exit 0
