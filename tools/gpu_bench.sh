#!/bin/bash
# GPU-box script: bench line + rocprofv3 kernel-trace stats of the same command.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
timeout -k 10 900 python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$NO_PROF" ]; then exit 0; fi
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench --output-format csv -- python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline --no-profile --no-bf16-line ${BENCH_ARGS} > gpurun_out/bench_prof.log 2>&1
rc=$?
echo "rocprof rc=$rc" >> gpurun_out/bench_prof.log
exit $rc
