#!/bin/bash
# GPU box: the whole -m gpu suite (one pytest process per file), then the counter-only PMC passes
# (FETCH_SIZE, WRITE_SIZE) of the default bench workload for the roofline's `traffic`.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_pmc.sh || exit $?
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc/FETCH_SIZE.log > gpurun_out/pmc/summary.json || exit $?
exit $rc
