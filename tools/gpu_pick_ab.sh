#!/bin/bash
# GPU box: parity of the long-sequence GEMM picks, then the 600 s DiT line with the new picks vs the previous
# library (ACE_MI_LIB=ab_lib/libacestep_mi355x_prev.so), alternating.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/pick_ab${TAG}; mkdir -p "$out"
rc=0
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_configs.py -k "qkv_prep or 600 or q4_k" \
    -v -s -m gpu --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
[ -n "$SKIP_TESTS" ] || { rc=$?; echo "rc=$rc" >> "$out/pytest.log"; }
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in new prev new prev; do
  if [ $lib = prev ]; then export ACE_MI_LIB=$GRAFT_REPO_ROOT/ab_lib/libacestep_mi355x_prev.so; else unset ACE_MI_LIB; fi
  for q in bf16 q4_k; do
    timeout -k 10 300 python -u bench.py --seconds 600 --qtype $q --no-cpu-baseline --no-extra-lines --no-bf16-line --no-profile \
        --steps 8 --warmup 2 >> "$out/bench_${lib}_$q.jsonl" 2>> "$out/bench.err" || exit $?
  done
done
exit $rc
