#!/bin/bash
# tests then bench; stop on a crash/timeout (rc other than 0/1)
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests.sh
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_bench.sh
