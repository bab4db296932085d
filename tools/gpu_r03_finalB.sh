#!/bin/bash
# Round 3 validation B: the default bench line, its rocprofv3 kernel-trace stats, HBM traffic PMC passes.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread tests/test_gpu_quant.py -k staged_dequant > gpurun_out/quant_staged.log 2>&1; rc=$?
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_final" -o bench --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-bf16-line --no-extra-lines > gpurun_out/bench_prof.log 2>&1 || exit $?
bash tools/gpu_pmc.sh || exit $?
exit 0
