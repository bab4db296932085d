#!/bin/bash
# GPU box: the variant-21 diagnostic build (qr3: scale pieces first) and the pv8 attention validation.
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r04_qrdiag.sh || exit $?
bash tools/gpu_r04_pv8.sh
