#!/bin/bash
# GPU box (round 6): the driver's bench command, then the 240 s VAE decode against an A/B product library
# (LIBS, lib/ab/<name>.so), interleaved.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; out=gpurun_out/r6bench; mkdir -p $out
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit $?
for r in 1 2; do
  for n in base ${LIBS}; do
    if [ "$n" = base ]; then unset ACE_MI_LIB; else export ACE_MI_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/$n.so; fi
    echo -n "$n " >> $out/vae.txt
    timeout -k 10 240 python -u tools/vae_profile.py --frames 6000 --runs 3 2>> $out/vae.err | tail -1 >> $out/vae.txt || exit 1
  done
done
