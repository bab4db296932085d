#!/bin/bash
# GPU box: staged-dequant kernel exactness, then the Q8_0 bench line for each chunks-per-thread setting
# (ACE_MI_DEQ_CPT), and a kernel-trace of the default setting.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_quant.py -q -m gpu -x -k "staged" --timeout 200 --timeout-method thread > gpurun_out/deq_test.log 2>&1 || exit $?
for r in 1 2; do
for c in ${CPTS:-1 2 4 8}; do
    echo "== cpt $c round $r" >> gpurun_out/deq_ab.log
    ACE_MI_DEQ_CPT=$c timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-bf16-line >> gpurun_out/deq_ab.log 2>> gpurun_out/deq_ab.err || exit $?
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_deq" -o bench --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-bf16-line > gpurun_out/deq_prof.log 2>&1
