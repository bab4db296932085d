#!/bin/bash
# GPU-box script: HBM traffic of the bench's kernels from PMC counters, one counter group per pass
# (MI355X_MICROARCH.md "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE cannot share a pass), counters
# only — no trace domains in these runs.  Summaries land in gpurun_out/pmc/; tools/pmc_summary.py turns
# them into per-launch bytes (FETCH_SIZE doubled for gfx950's 128-B requests tallied at 64 B).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-bf16-line ${BENCH_ARGS}"
for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/$ctr" -o pmc --output-format csv \
        -- python bench.py $ARGS > "gpurun_out/pmc/$ctr.log" 2>&1
    rc=$?
    echo "pmc $ctr rc=$rc" >> "gpurun_out/pmc/$ctr.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
done
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/FETCH_SIZE.log > gpurun_out/pmc/summary.json
