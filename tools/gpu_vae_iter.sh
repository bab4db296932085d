#!/bin/bash
# GPU box: VAE parity (tiny + full-size + the windowed 192-frame decode) then the per-stage profile at 240 s.
# Usage: tools/gpu_vae_iter.sh <tag>   (outputs under gpurun_out/vae_<tag>/)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/vae_${1:-x}; mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_vae.py "tests/test_gpu_configs.py::test_config4_vae_decode_192_frames_windowed" \
    -v -s -m gpu --timeout 300 --timeout-method thread > "$out/pytest.log" 2>&1
rc=$?; echo "rc=$rc" >> "$out/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/vae_profile.py --frames 6000 --runs 3 > "$out/time_6000.json" 2> "$out/time.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o vae --output-format csv -- \
    python tools/vae_profile.py --frames 6000 --runs 1 > "$out/prof.log" 2>&1 || exit $?
python tools/vae_profile.py --summarize "$(ls $out/prof/*kernel_trace.csv | head -1)" --frames 6000 > "$out/stages_6000.json"
exit $rc
