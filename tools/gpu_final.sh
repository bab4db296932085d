#!/bin/bash
# GPU box: the HBM-traffic PMC passes of the bench workload (FETCH_SIZE, WRITE_SIZE; separate counter-only runs) ->
# tools/pmc_summary.py (stamped with acestep_mi355x.source_hash(); copied to profiles/pmc_traffic.json on the box so the
# bench line below reports `traffic` -- commit that summary from gpurun_out/pmc/summary.json), then the driver's bench
# command, then the rocprofv3 kernel-trace summary of a short run of the same workload.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/final gpurun_out/pmc; export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/$ctr" -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-bf16-line --no-extra-lines > "gpurun_out/pmc/$ctr.log" 2>&1 || exit $?
done
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/FETCH_SIZE.log > gpurun_out/pmc/summary.json || exit $?
cp gpurun_out/pmc/summary.json profiles/pmc_traffic.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/final/prof" -o bench --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-profile --no-bf16-line --no-extra-lines > gpurun_out/final/bench_prof.log 2>&1 || exit $?
