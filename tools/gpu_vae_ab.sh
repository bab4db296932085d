#!/bin/bash
# GPU box: VAE quick parity (-k selection) then an A/B of one env switch on the 240 s decode (timing + per-stage
# kernel trace for each side).  Usage: tools/gpu_vae_ab.sh <tag> <VAR> <valueA> <valueB> [pytest -k expr]
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/vae_ab_$1; mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_vae.py -k "${5:-phase or halo or odd_stride}" -v -s -m gpu --timeout 300 \
    --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; echo "rc=$rc" >> "$out/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "$3" "$4" "$3" "$4"; do
  env "$2=$v" timeout -k 10 200 python -u tools/vae_profile.py --frames 6000 --runs 3 >> "$out/time_$v.json" 2>> "$out/time.err" || exit $?
done
for v in "$3" "$4"; do
  env "$2=$v" timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/p_$v" -o vae --output-format csv -- \
      python tools/vae_profile.py --frames 6000 --runs 1 > "$out/prof_$v.log" 2>&1 || exit $?
  python tools/vae_profile.py --summarize "$(ls $out/p_$v/*kernel_trace.csv | head -1)" --frames 6000 > "$out/stages_$v.json" || exit $?
  rm -rf "$out/p_$v"
done
exit $rc
