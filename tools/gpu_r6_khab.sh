#!/bin/bash
# GPU box (round 6): f8c attention launch times, the build vs A/B self-test libraries (LIBS="name ..." = lib/ab/<name>_st.so),
# interleaved, with ACE_MI_ATTN_KH=${KH:-1}.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6khab; mkdir -p $out
for r in 1 2; do
  for n in base ${LIBS}; do
    if [ "$n" = base ]; then unset ACE_MI_SELFTEST_LIB; else export ACE_MI_SELFTEST_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/${n}_st.so; fi
    ACE_MI_ATTN_KH=${KH:-1} ATTN_MODES=${MODES:-f8c} timeout -k 10 180 python -u tools/attn_bench.py 2>> $out/err.txt | sed "s/^/$n /" >> $out/ab.txt || exit 1
  done
done
exit 0
