#!/bin/bash
# GPU box: variant-21 Q4_K diagnostic against two diagnostic builds (tools/build_ab.sh qr1 / qr2: ACEMI_QR_DIAG 1 =
# no LDS-DMA in flight during LDS reads, 2 = q bytes by ds_read_b64).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/qr; export TMPDIR=/tmp
for n in qr3; do
  if [ $n = base ]; then unset ACE_MI_SELFTEST_LIB; else export ACE_MI_SELFTEST_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/${n}_st.so; fi
  timeout -k 10 120 python -u tools/diag_v21.py > gpurun_out/qr/diag_$n.log 2>&1 || exit $?
done
