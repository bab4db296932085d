cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SUITES="forward:900" bash tools/gpu_tests.sh; r=$?
if [ $r -gt 1 ]; then exit $r; fi
bash tools/gpu_bench.sh
