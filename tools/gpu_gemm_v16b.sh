#!/bin/bash
# GPU box: 8-wave 192x128 (v16) against the current picks at the batched / long-sequence M
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/gemm_v16; mkdir -p "$out"
timeout -k 10 400 python -u tools/gemm_msweep.py 4,7,10,11,16 4500,7500,12000,24000 > "$out/msweep_b.jsonl" 2> "$out/msweep_b.err" || exit $?
