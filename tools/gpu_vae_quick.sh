cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/vae_e4
timeout -k 10 300 python -u -m pytest tests/test_gpu_vae.py -k "halo or odd_stride" -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/vae_e4/pytest.log 2>&1
rc=$?; echo rc=$rc >> gpurun_out/vae_e4/pytest.log; exit $rc
