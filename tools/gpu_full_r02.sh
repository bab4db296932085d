#!/bin/bash
# GPU box: the whole -m gpu suite (one pytest process per file), then the extra bench lines of DESIGN.md §6:
# bs=8 per GPU (bf16 and Q8_0) and the 60 s configs[1] line.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SUITES="kernels:400 forward:900 lyric_timbre:300 quant:900 sampler:300 text_encoder:300 vae:600" bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --batch-per-gpu 8 --qtype bf16 --no-cpu-baseline > gpurun_out/bench_bs8.json 2> gpurun_out/bench_bs8.err || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --batch-per-gpu 8 --no-bf16-line --no-cpu-baseline > gpurun_out/bench_bs8_q8.json 2> gpurun_out/bench_bs8_q8.err || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 2 --seconds 60 --qtype bf16 --no-cpu-baseline > gpurun_out/bench_60s.json 2> gpurun_out/bench_60s.err || exit $?
exit $rc
