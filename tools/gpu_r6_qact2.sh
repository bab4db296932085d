#!/bin/bash
# GPU box (round 6): q8-mode GEMM unit tests + per-kernel times (bf16-MFMA Q8_0 GEMM), one run.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6qact2; mkdir -p $out
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_qact.py -k "gemm_a8" > $out/test_qact.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_qact.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/qact_bench.py > $out/qact_bf16.jsonl 2> $out/qact_bf16.err || exit $?
exit 0
