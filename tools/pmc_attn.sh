cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/apmc; export TMPDIR=/tmp
export ATTN_CASE="self_full 240s"
timeout -k 10 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS -d "$GRAFT_REPO_ROOT/gpurun_out/apmc/p1" -o pmc --output-format csv -- python tools/attn_bench.py > gpurun_out/apmc/p1.log 2>&1 &&
timeout -k 10 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAVES -d "$GRAFT_REPO_ROOT/gpurun_out/apmc/p2" -o pmc --output-format csv -- python tools/attn_bench.py > gpurun_out/apmc/p2.log 2>&1
