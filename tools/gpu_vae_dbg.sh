#!/bin/bash
# GPU box: VAE decode kernel traces with the timing-experiment switches (ACE_MI_VAE_DBG) -> per-stage tables
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/vae_dbg_${1:-x}; mkdir -p "$out"
for dbg in ${DBGS:-0 1 2 4 6 7}; do
  ACE_MI_VAE_DBG=$dbg timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/p$dbg" -o vae --output-format csv -- \
      python tools/vae_profile.py --frames 6000 --runs 1 > "$out/prof$dbg.log" 2>&1 || exit $?
  python tools/vae_profile.py --summarize "$(ls $out/p$dbg/*kernel_trace.csv | head -1)" --frames 6000 > "$out/stages_$dbg.json" || exit $?
  rm -rf "$out/p$dbg"
done
