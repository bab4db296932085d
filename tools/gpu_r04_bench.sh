#!/bin/bash
# GPU box: the driver's bench command (default workload, every extra line) and the variant-21 Q4_K diagnostic
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/diag_v21.py > gpurun_out/diag_v21.log 2>&1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r04.json 2> gpurun_out/bench_r04.err
