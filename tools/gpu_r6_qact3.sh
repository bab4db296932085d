#!/bin/bash
# GPU box (round 6): q8-mode tests (kernels, tiny, full width, configs), attention tests, per-kernel times, bench.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6qact3; mkdir -p $out
P="python -u -m pytest -q -m gpu --timeout 600 --timeout-method thread -s"
timeout -k 10 300 $P tests/test_gpu_qact.py > $out/test_qact.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_qact.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 $P tests/test_gpu_kernels.py -k attention > $out/test_attn.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_attn.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 $P tests/test_gpu_quant.py -k "full_width_vs_ggml" > $out/test_quant_fw.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_quant_fw.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 600 $P tests/test_gpu_configs.py -k "quantized_configs" > $out/test_configs_q.log 2>&1; rc=$?; echo "rc=$rc" >> $out/test_configs_q.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/qact_bench.py > $out/qact_bf16.jsonl 2> $out/qact_bf16.err || exit $?
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit $?
exit 0
