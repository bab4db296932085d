#!/bin/bash
# GPU box: attention micro-benchmark at the 240 s shapes, then SQ counter passes (wave parking vs issue stalls vs
# MFMA busy) for the fast-mode self (full) and cross kernels.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/attn_${1:-x}; mkdir -p "$out"
timeout -k 10 200 python -u tools/attn_bench.py > "$out/bench.jsonl" 2> "$out/bench.err" || exit $?
for c in "self_full 240s" "cross 240s" "self_sliding 240s"; do
  tag=$(echo "$c" | tr ' ' '_')
  ATTN_CASE="$c" ATTN_MODE=fast timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
      -d "$GRAFT_REPO_ROOT/$out/pmc_$tag" -o p --output-format csv -- python tools/attn_bench.py > "$out/pmc_$tag.log" 2>&1 || exit $?
done
