#!/bin/bash
# GPU-box: effective shader clock under the attention and GEMM micro-benchmarks — GRBM_GUI_ACTIVE
# (GPU-busy cycles) per dispatch against the dispatch's own start/end timestamps.  Counters only.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/clk; export TMPDIR=/tmp
ATTN_CASE="self_full 240s" timeout -k 10 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES \
    -d "$GRAFT_REPO_ROOT/gpurun_out/clk/attn" -o pmc --output-format csv -- python tools/attn_bench.py \
    > gpurun_out/clk/attn.log 2>&1 &&
timeout -k 10 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES \
    -d "$GRAFT_REPO_ROOT/gpurun_out/clk/gemm" -o pmc --output-format csv -- python tools/gemm_bench.py 4 \
    > gpurun_out/clk/gemm.log 2>&1
