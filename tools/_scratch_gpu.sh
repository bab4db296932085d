cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SUITES="kernels:400 forward:900" bash tools/gpu_tests.sh; r=$?
if [ $r -gt 1 ]; then exit $r; fi
for ks in 1 2; do ACE_MI_ATTN_KSPLIT=$ks timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench_ks$ks.log 2>&1 || exit 3; done
timeout -k 10 300 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1 || exit 4
NO_PROF=1 bash tools/gpu_bench.sh
