#!/bin/bash
# Round 3: attention epilogue with 16-byte stores (lane-half swap): attention tests + forward tests + bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_kernels.py -k attention tests/test_gpu_forward.py > gpurun_out/attn_m.log 2>&1 || exit $?
B="bench.py --steps 27 --warmup 3 --no-extra-lines --no-bf16-line --no-cpu-baseline --qtype bf16"
for sec in 240 60 10; do
  timeout -k 10 300 python $B --seconds $sec > gpurun_out/m_${sec}.json 2> gpurun_out/m_${sec}.err || exit $?
done
exit 0
