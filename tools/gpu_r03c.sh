#!/bin/bash
# Round 3: LDS-dequant GEMM correctness matrix + micro-bench, dense split-K sweep at M = 3000, strict parity after
# the timestep / floor changes, loop determinism, the hook on hipStreamLegacy.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 600 --timeout-method thread"
timeout -k 10 300 python tools/diag_qr.py > gpurun_out/diag_qr.log 2>&1 || exit $?
timeout -k 10 300 python tools/gemm_q_bench.py 3000,750,125 -1,20,21,22 > gpurun_out/gemm_q_bench2.jsonl 2> gpurun_out/gemm_q_bench2.err || exit $?
timeout -k 10 300 python tools/gemm_msweep.py 7,4,1,104,204,107,207,11 3000 > gpurun_out/msweep_sk.jsonl 2> gpurun_out/msweep_sk.err || exit $?
timeout -k 10 300 python tools/diag_loop.py > gpurun_out/diag_loop2.log 2>&1 || exit $?
timeout -k 10 300 $T tests/test_gpu_forward.py -k "hook or golden or batched or sampler" > gpurun_out/fwd_quick.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 $T tests/test_gpu_parity_strict.py > gpurun_out/strict2.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/diag_peaked.py > gpurun_out/diag_peaked2.log 2>&1 || exit $?
exit 0
