#!/bin/bash
# GPU box: forward / BASELINE-config / sampler parity after the multi-layer cross prep, then the default
# bench line + rocprofv3 stats, the 60 s (configs[1] shape) line and the bs=8 lines.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SUITES="forward:900 configs:900 sampler:300" bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
STEPS=27 bash tools/gpu_bench.sh || exit $?
timeout -k 10 600 python bench.py --steps 27 --warmup 3 --seconds 60 --qtype bf16 --no-cpu-baseline > gpurun_out/bench_60s.json 2> gpurun_out/bench_60s.err || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --batch-per-gpu 8 --no-cpu-baseline > gpurun_out/bench_bs8_q8.json 2> gpurun_out/bench_bs8_q8.err || exit $?
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 tools/rccl_check.py > gpurun_out/rccl_check.json 2> gpurun_out/rccl_check.err || exit $?
exit $rc
