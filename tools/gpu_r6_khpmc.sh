#!/bin/bash
# GPU box (round 6): SQ counters of the f8c self-full attention launch at 240 s, attn_kh_kernel vs attn2 (LDS-array
# cycles and bank conflicts, MFMA busy, VALU / LDS issue), counter-only rocprofv3 passes.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6khpmc; mkdir -p $out
for kh in 1 0; do
  ACE_MI_ATTN_KH=$kh ATTN_CASE="self_full 240s" ATTN_MODE=f8c timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT \
      -d "$GRAFT_REPO_ROOT/$out/a_kh$kh" -o p --output-format csv -- python tools/attn_bench.py > $out/a_kh$kh.log 2>&1 || exit $?
  ACE_MI_ATTN_KH=$kh ATTN_CASE="self_full 240s" ATTN_MODE=f8c timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
      -d "$GRAFT_REPO_ROOT/$out/b_kh$kh" -o p --output-format csv -- python tools/attn_bench.py > $out/b_kh$kh.log 2>&1 || exit $?
done
exit 0
