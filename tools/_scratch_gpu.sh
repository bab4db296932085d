cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SUITES="forward:900 text_encoder:400" bash tools/gpu_tests.sh; r=$?
if [ $r -gt 1 ]; then exit $r; fi
timeout -k 10 1500 python -u -m pytest tests/test_gpu_configs.py -v -s -m gpu --timeout 1200 --timeout-method thread > gpurun_out/configs.log 2>&1; r=$?
echo "configs rc=$r" >> gpurun_out/configs.log
exit $r
