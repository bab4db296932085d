#!/bin/bash
# GPU box (round 6): the whole -m gpu suite (tools/gpu_tests.sh); with BENCH=1 the driver's bench command after it.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
bash tools/gpu_tests.sh; rc=$?
[ $rc -gt 1 ] && exit $rc
if [ -n "$BENCH" ]; then
  mkdir -p gpurun_out/bench
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench/bench.json 2> gpurun_out/bench/bench.err || exit $?
fi
exit $rc
