#!/bin/bash
# GPU box (round 6): the kernel / quant / VAE test files, then headline-only bench lines against A/B product libraries
# (tools/build_ab.sh PRODUCT=1), interleaved: base (the build), LIBS="slp noguard ..." (lib/ab/<name>.so).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r6ab
for t in ${TESTS:-kernels quant vae}; do
  timeout -k 10 600 python -u -m pytest "tests/test_gpu_${t}.py" -q -m gpu -x --timeout 300 --timeout-method thread \
      > "gpurun_out/r6ab/test_${t}.log" 2>&1
  rc=$?; echo "rc=$rc" >> "gpurun_out/r6ab/test_${t}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
B="python -u bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-profile --no-bf16-line --no-extra-lines ${BARGS}"
for r in $(seq ${REPS:-2}); do
  for n in base ${LIBS}; do
    if [ "$n" = base ]; then unset ACE_MI_LIB; else export ACE_MI_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/$n.so; fi
    echo -n "$n " >> gpurun_out/r6ab/lines.txt
    timeout -k 10 240 $B 2>> gpurun_out/r6ab/bench.err | tail -1 >> gpurun_out/r6ab/lines.txt || exit 1
  done
done
