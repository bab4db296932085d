#!/bin/bash
# GPU box (round 6): the q8-mode (ggml arithmetic) tests and per-kernel times with the Q8_0 GEMM on the i8 MFMA vs on the
# bf16 MFMA (ACE_MI_QACT_GEMM=0 / default), plus the text-encoder pin.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6qact; mkdir -p $out
P="python -u -m pytest -q -m gpu --timeout 600 --timeout-method thread -s"
timeout -k 10 600 $P tests/test_gpu_qact.py > $out/test_qact.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_qact.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 $P tests/test_gpu_text_encoder.py > $out/test_text.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_text.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 env ACE_MI_QACT_GEMM=0 python -u tools/qact_bench.py > $out/qact_i8.jsonl 2> $out/qact_i8.err || exit $?
timeout -k 10 300 python -u tools/qact_bench.py > $out/qact_bf16.jsonl 2> $out/qact_bf16.err || exit $?
timeout -k 10 900 $P tests/test_gpu_quant.py -k "full_width_vs_ggml" > $out/test_quant_fw.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_quant_fw.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 900 $P tests/test_gpu_configs.py -k "quantized_configs" > $out/test_configs_q.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_configs_q.log
exit 0
