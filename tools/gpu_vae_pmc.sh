#!/bin/bash
# GPU box: HBM bytes per VAE conv launch at 240 s (rocprofv3 --pmc, one counter per pass, counters only), joined
# with the launch plan by tools/vae_pmc_summary.py.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/vae_pmc; mkdir -p "$out"
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$GRAFT_REPO_ROOT/$out/$ctr" -o p --output-format csv -- \
      python tools/vae_profile.py --frames 6000 --runs 1 > "$out/$ctr.log" 2>&1 || exit $?
done
python tools/vae_pmc_summary.py "$out" 6000 > "$out/summary.json"
