#!/bin/bash
# GPU box: attention kernel tests, then attn_bench alternating lib/ab/base.so and lib/ab/new.so
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity_strict.py -k "attention or attn or peaked" -v -m gpu --timeout 300 \
    --timeout-method thread > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/attn_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
rm -f gpurun_out/ab.log
NAMES="base new" AB_CMD="tools/attn_bench.py" ROUNDS=3 bash tools/ab_multi.sh
