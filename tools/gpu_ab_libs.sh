#!/bin/bash
# GPU box: run one command against the regular build and each A/B self-test library built by tools/build_ab.sh
# (ACE_MI_SELFTEST_LIB), stopping at the first crash / time limit.  Output: gpurun_out/ab/<tag>/<lib>.log.
# Usage: TAG=name LIBS="base abl1 abl2" LIMIT=200 bash tools/gpu_ab_libs.sh python -u tools/gemm_bench.py 4,7
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/ab/${TAG:-run}; mkdir -p "$out"
for n in ${LIBS:-base}; do
  if [ "$n" = base ]; then unset ACE_MI_SELFTEST_LIB; else export ACE_MI_SELFTEST_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/${n}_st.so; fi
  timeout -k 10 "${LIMIT:-300}" "$@" > "$out/$n.log" 2>&1 || exit $?
done
