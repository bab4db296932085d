#!/bin/bash
# GPU box: quantized-path parity (incl. the sampling-call staging scope), then the default bench line
# (BASELINE configs[2], Q8_0, with the bf16 line beside it) + rocprofv3 kernel stats of the same command.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SUITES="quant:900 sampler:300" bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
STEPS=27 bash tools/gpu_bench.sh || exit $?
exit $rc
