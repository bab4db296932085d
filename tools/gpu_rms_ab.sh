cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=gpurun_out/rms_ab; mkdir -p "$out"
ARGS="--qtype bf16 --no-cpu-baseline --no-extra-lines --no-bf16-line --steps 10 --warmup 2"
for s in 60 240; do
for cfg in "P2" "P0" "P0R1" "P4" "P1" "P2"; do
  case $cfg in P2) E="ACE_MI_RMSNORM_PERSIST=2";; P0) E="ACE_MI_RMSNORM_PERSIST=0";; P0R1) E="ACE_MI_RMSNORM_PERSIST=0 ACE_MI_RMSNORM_ROWS=1";; P4) E="ACE_MI_RMSNORM_PERSIST=4";; P1) E="ACE_MI_RMSNORM_PERSIST=1";; esac
  env $E timeout -k 10 200 python -u bench.py $ARGS --seconds $s > "$out/tmp.json" 2>> "$out/err" || exit $?
  python -c "import json; d=json.load(open('$out/tmp.json')); print(json.dumps({'s': $s, 'cfg': '$cfg', 'value': d['value'], 'rms_ms': d.get('breakdown',{}).get('rmsnorm_mod')}))" >> "$out/results.jsonl"
done
done
