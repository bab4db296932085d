#!/bin/bash
# Round 3: strict parity tests (peaked attention, 1-layer literal, fault injection), configs[1] and the
# configs[2] sampling-loop test, then the 240 s bf16 bench in fp16 and split attention on one box.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 600 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_parity_strict.py > gpurun_out/strict.log 2>&1; rc=$?
echo "strict rc=$rc" >> gpurun_out/strict.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 $T tests/test_gpu_configs.py -k "config1 or config2_q8_0_sampling" > gpurun_out/cfg.log 2>&1; rc2=$?
echo "cfg rc=$rc2" >> gpurun_out/cfg.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 600 python bench.py --qtype bf16 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_fp16.json 2> gpurun_out/bench_fp16.err || exit $?
ACE_MI_ATTN_PRECISION=split timeout -k 10 600 python bench.py --qtype bf16 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_split.json 2> gpurun_out/bench_split.err || exit $?
exit $rc
