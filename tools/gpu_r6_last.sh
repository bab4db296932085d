#!/bin/bash
# GPU box (round 6, last tree): the attention kernel tests and the text-encoder causal tests, then tools/gpu_final.sh
# (PMC traffic stamped with this tree's source hash, the driver's bench command, the rocprof kernel trace).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6last; mkdir -p $out
timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k attention \
    > $out/test_attn.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_attn.log; [ $rc -gt 1 ] && exit $rc
bash tools/gpu_final.sh
