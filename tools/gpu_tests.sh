#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/dev.txt
timeout -k 10 400 python -m pytest tests/test_gpu_kernels.py -q -m gpu > gpurun_out/k.log 2>&1
rc=$?
echo "kernels rc=$rc" >> gpurun_out/k.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -m pytest tests/test_gpu_forward.py -q -s -m "gpu" ${FWD_ARGS} > gpurun_out/f.log 2>&1
rc=$?
echo "forward rc=$rc" >> gpurun_out/f.log
exit $rc
