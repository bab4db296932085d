#!/bin/bash
# GPU box: in-loop A/B of GEMM tile picks at the 240 s bs=1 workload through ACE_MI_GEMM_OVERRIDE (N:K:variant),
# whole bench lines (bf16 weights), the unmodified picks interleaved as the reference.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/pick_inloop${TAG}; mkdir -p "$out"
ARGS="--qtype bf16 --no-cpu-baseline --no-extra-lines --no-bf16-line --steps 10 --warmup 2 ${BENCH_ARGS}"
run() {  # $1 = label, $2 = override
  ACE_MI_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/libacestep_mi355x_selftest.so ACE_MI_GEMM_OVERRIDE="$2" timeout -k 10 200 python -u bench.py $ARGS > "$out/tmp.json" 2>> "$out/bench.err" || exit $?
  python -c "import json,sys; d=json.load(open('$out/tmp.json')); print(json.dumps({'label': '$1', 'override': '$2', 'value': d['value'], 'ms': d['ms_per_step'], 'bl': d.get('breakdown', {}).get('_dit_block_linears', {}).get('frac_of_bf16_peak')}))" >> "$out/results.jsonl"
}
run base ""
for ov in ${OVS}; do
  run "$ov" "$ov"
  if [ $(( RANDOM % 3 )) -eq 0 ]; then run base ""; fi
done
run base ""
