#!/bin/bash
# GPU-box parity suite, one pytest process per file (dense paths first), each under its own time
# limit.  Stops at the first crash / timeout (rc other than 0 = pass, 1 = test failures).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m2 -E "gfx950|Marketing" > gpurun_out/dev.txt
worst=0
for spec in ${SUITES:-kernels:400 forward:900 parity_strict:900 configs:900 lyric_timbre:300 quant:900 qact:300 sampler:300 text_encoder:300 vae:600}; do
    name=${spec%%:*}
    lim=${spec##*:}
    timeout -k 10 "$lim" python -u -m pytest "tests/test_gpu_${name}.py" -v -s -m gpu --timeout 300 --timeout-method thread ${FWD_ARGS} \
        > "gpurun_out/${name}.log" 2>&1
    rc=$?
    echo "${name} rc=$rc" >> "gpurun_out/${name}.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    if [ $rc -gt $worst ]; then worst=$rc; fi
done
exit $worst
