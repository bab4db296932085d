#!/bin/bash
# Round 3 validation A: the whole -m gpu suite (one pytest process per file) and smoke().
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_tests.sh; rc=$?
echo "suite rc=$rc" > gpurun_out/suite_rc.txt
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
exit $rc
