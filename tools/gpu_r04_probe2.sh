#!/bin/bash
# GPU box: fp8 block-scaled MFMA layout probe, attention kernel tests (all modes incl. f8c), attention micro-bench,
# then (kernel tests green only) the one-layer literal-bound / peaked parity in f8c mode
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
true
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attention or attn" -q -m gpu --timeout 120 \
    --timeout-method thread > gpurun_out/attn_kernel_tests.log 2>&1
krc=$?
echo "kernel tests rc=$krc" >> gpurun_out/attn_kernel_tests.log
if [ $krc -ne 0 ] && [ $krc -ne 1 ]; then exit $krc; fi   # a crash / timeout: stop here
timeout -k 10 200 python -u tools/attn_bench.py > gpurun_out/attn_modes_v3.jsonl 2>&1 || exit $?
if [ $krc -ne 0 ]; then exit 1; fi
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_strict.py -k "(one_layer and default and f8c) or (peaked_attention and f8c)" -v -s -m gpu --timeout 300 \
    --timeout-method thread > gpurun_out/one_layer_f8c.log 2>&1
for r in 1 2; do for v in ra2 ra4; do
  echo "== $v round $r" >> gpurun_out/attn_ra_ab.log
  ACE_MI_SELFTEST_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/${v}_st.so timeout -k 10 200 python -u tools/attn_bench.py >> gpurun_out/attn_ra_ab.log 2>&1 || exit $?
done; done
for m in f8c pvsplit; do
  ATTN_CASE="self_full 240s" ATTN_MODE=$m timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
      -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$m" -o p --output-format csv -- python tools/attn_bench.py > "gpurun_out/pmc_$m.log" 2>&1 || exit $?
done
