#!/bin/bash
# GPU box: VAE parity (decode / encode / windowed 192-frame full-width decode) then the VAE profile.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_vae.py tests/test_gpu_configs.py -k "vae" -q -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/vae_tests.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/vae_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_vae_prof.sh
