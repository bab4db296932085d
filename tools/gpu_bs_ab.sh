#!/bin/bash
# GPU box: 240 s DiT line at 2 / 4 / 8 items per GPU (M = 6000 / 12000 / 24000), new GEMM picks vs the previous
# library (ab_lib/libacestep_mi355x_prev.so), alternating.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/bs_ab${TAG}; mkdir -p "$out"
for b in ${BS:-2 4 8}; do
  for lib in new prev new prev; do
    if [ $lib = prev ]; then export ACE_MI_LIB=$GRAFT_REPO_ROOT/ab_lib/libacestep_mi355x_prev.so; else unset ACE_MI_LIB; fi
    timeout -k 10 300 python -u bench.py --batch-per-gpu $b --seconds ${SECONDS_:-240} --qtype bf16 --no-cpu-baseline --no-extra-lines --no-bf16-line \
        --steps 6 --warmup 2 >> "$out/bench_b${b}_${lib}.jsonl" 2>> "$out/bench.err" || exit $?
  done
done
