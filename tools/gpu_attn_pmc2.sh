#!/bin/bash
# GPU box: SQ counter passes (wave parking vs issue stalls vs MFMA busy) of the attention kernel at the 240 s full-layer
# shape in each precision mode (ATTN_MODE), one counter-only rocprofv3 pass per mode.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/attn_${1:-x}; mkdir -p "$out"
for m in fast split pvsplit; do
  ATTN_CASE="self_full 240s" ATTN_MODE=$m timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
      -d "$GRAFT_REPO_ROOT/$out/pmc_$m" -o p --output-format csv -- python tools/attn_bench.py > "$out/pmc_$m.log" 2>&1 || exit $?
done
