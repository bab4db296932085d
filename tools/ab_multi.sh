#!/bin/bash
# GPU-box A/B/C..: alternate several builds of the library (ACE_MI_LIB = lib/ab/<name>.so) over the same
# micro-benchmark, ROUNDS times, one process per run.  Usage: NAMES="base e1 e2" AB_CMD="tools/gemm_bench.py 10" bash tools/ab_multi.sh
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LIBDIR=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab
for r in $(seq 1 "${ROUNDS:-2}"); do
    for v in ${NAMES:-base new}; do
        echo "== $v round $r" >> gpurun_out/ab.log
        ACE_MI_LIB="$LIBDIR/$v.so" timeout -k 10 "${AB_LIMIT:-200}" python -u $AB_CMD >> gpurun_out/ab.log 2>&1 || exit $?
    done
done
