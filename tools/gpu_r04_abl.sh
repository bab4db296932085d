#!/bin/bash
# GPU box: GEMM loop ablations (tools/build_ab.sh: abl4 = DMA of k-tile 0 only (L2-hot bytes, issue kept), abl5 = that
# without the LDS reads) against the regular build (incl. the 3-stage 192x128 tile, 17), and the variant-21 Q4_K
# diagnostic.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abl; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/diag_v21.py > gpurun_out/diag_v21.log 2>&1
for n in base abl4 abl5; do
  if [ $n = base ]; then unset ACE_MI_SELFTEST_LIB; else export ACE_MI_SELFTEST_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/${n}_st.so; fi
  timeout -k 10 200 python -u tools/gemm_bench.py 4,17,7,14,15 > gpurun_out/abl/b_$n.jsonl 2>&1 || exit $?
done
