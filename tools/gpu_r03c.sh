#!/bin/bash
# Round 3: register-dequant correctness matrix, strict parity after the timestep / floor changes, loop determinism,
# the hook on hipStreamLegacy.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 600 --timeout-method thread"
timeout -k 10 300 python tools/diag_qr.py > gpurun_out/diag_qr.log 2>&1 || exit $?
timeout -k 10 300 $T tests/test_gpu_forward.py -k "hook or golden or batched or sampler" > gpurun_out/fwd_quick.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 $T tests/test_gpu_parity_strict.py > gpurun_out/strict2.log 2>&1; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/diag_peaked.py > gpurun_out/diag_peaked2.log 2>&1 || exit $?
timeout -k 10 300 python tools/diag_loop.py > gpurun_out/diag_loop2.log 2>&1 || exit $?
exit 0
