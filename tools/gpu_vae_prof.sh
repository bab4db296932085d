#!/bin/bash
# GPU box: VAE decode timing at 240 s / 600 s of audio and a rocprofv3 kernel trace of the 240 s decode, joined
# with the launch plan into per-stage TFLOP/s (tools/vae_profile.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/vae; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/vae_profile.py --frames 6000 --runs 3 > gpurun_out/vae/time_6000.json 2> gpurun_out/vae/time.err || exit $?
timeout -k 10 300 python -u tools/vae_profile.py --frames 15000 --runs 3 > gpurun_out/vae/time_15000.json 2>> gpurun_out/vae/time.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/vae/prof" -o vae --output-format csv -- python tools/vae_profile.py --frames 6000 --runs 1 > gpurun_out/vae/prof.log 2>&1 || exit $?
python tools/vae_profile.py --summarize "$(ls gpurun_out/vae/prof/*kernel_trace.csv | head -1)" --frames 6000 > gpurun_out/vae/stages_6000.json
