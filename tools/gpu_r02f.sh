#!/bin/bash
# GPU box: the whole -m gpu suite incl. the BASELINE-config parity file, smoke(), then the bs=8 line
# (8-wave residual tiles) and the default bench line + rocprofv3 stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SUITES="kernels:400 forward:900 quant:900 configs:900 sampler:300 lyric_timbre:300 text_encoder:300 vae:600" bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 5 --warmup 1 --batch-per-gpu 8 --no-cpu-baseline > gpurun_out/bench_bs8_q8.json 2> gpurun_out/bench_bs8_q8.err || exit $?
STEPS=27 bash tools/gpu_bench.sh || exit $?
exit $rc
