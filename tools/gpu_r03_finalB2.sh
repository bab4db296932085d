#!/bin/bash
# Round 3 (session 2) measurement: attention wave-priority A/B (lib/ab/p0|p1|p2.so), then the default bench line
# and a rocprofv3 kernel-trace --stats pass of the same bench command.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
NAMES="p0 p1 p2" AB_CMD="tools/attn_bench.py" ROUNDS=2 bash tools/ab_multi.sh || exit $?
STEPS=10 bash tools/gpu_bench.sh
