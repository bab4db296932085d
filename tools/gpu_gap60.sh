#!/bin/bash
# GPU box: 60 s (configs[1] shape) bf16 bench line and a kernel trace of it (launch-gap analysis).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --seconds 60 --qtype bf16 --no-bf16-line --no-cpu-baseline --steps 27 --warmup 3 > gpurun_out/b60.json 2> gpurun_out/b60.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof60" -o b60 --output-format csv -- python bench.py --seconds 60 --qtype bf16 --no-bf16-line --no-cpu-baseline --no-profile --steps 27 --warmup 3 > gpurun_out/b60_prof.log 2>&1
