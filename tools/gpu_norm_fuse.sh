#!/bin/bash
# GPU box: the fused row norm (launch_gemm_resid_norm) -- its bit-identity tests, the forward / quantized parity tests
# that now run through it, then bench lines with the fusion on and off (ACE_MI_NORM_FUSE=0), interleaved
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
P="python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread"
timeout -k 10 300 $P tests/test_gpu_norm_fuse.py > gpurun_out/nf_tests.log 2>&1 || exit 1
timeout -k 10 600 $P tests/test_gpu_forward.py tests/test_gpu_quant.py > gpurun_out/nf_fwd.log 2>&1 || exit 1
B="python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extra-lines --no-bf16-line --no-profile"
rm -f gpurun_out/nf_lines.log
for r in 1 2; do
  for sec in 60 240; do
    echo "sec=$sec fused" >> gpurun_out/nf_lines.log
    ACE_MI_NORM_FUSE=1 timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 >> gpurun_out/nf_lines.log || exit 1
    echo "sec=$sec off" >> gpurun_out/nf_lines.log
    ACE_MI_NORM_FUSE=0 timeout -k 10 240 $B --seconds $sec 2>/dev/null | tail -1 >> gpurun_out/nf_lines.log || exit 1
  done
done
