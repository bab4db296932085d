#!/bin/bash
# GPU box: correctness of GEMM variants 16 / 17 (8-wave 192x128) and an M = 3000 / 6000 TFLOP/s sweep vs the picks
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/gemm_v16; mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "variant and (16 or 17)" -v -m gpu --timeout 120 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; echo "rc=$rc" >> "$out/pytest.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/gemm_msweep.py 7,4,1,16,17 3000,6000 > "$out/msweep.jsonl" 2> "$out/msweep.err" || exit $?
