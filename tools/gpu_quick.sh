#!/bin/bash
# GPU-box script for a quick iteration: selected test files, attention micro-bench, bench line.
#   SUITES="kernels:400 forward:900" bash tools/gpu_quick.sh
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
SUITES=${SUITES:-"kernels:400"} bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -z "$NO_ATTN_BENCH" ]; then
    timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1
    r=$?; echo "attn_bench rc=$r" >> gpurun_out/attn_bench.log
    if [ $r -ne 0 ]; then exit $r; fi
fi
NO_PROF=${NO_PROF-1} bash tools/gpu_bench.sh
exit $?
