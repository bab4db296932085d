#!/bin/bash
# Round 3: cold-aware short-sequence tiles, side-stream weight prefetch A/B at 60 s / 10 s.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_forward.py tests/test_gpu_kernels.py > gpurun_out/fk_i.log 2>&1; rc=$?
[ $rc -gt 1 ] && exit $rc
B="bench.py --steps 27 --warmup 3 --no-extra-lines --no-bf16-line --no-cpu-baseline --qtype bf16"
for pf in 0 32 96 0; do
  for sec in 60 10; do
    ACE_MI_WEIGHT_PREFETCH=$pf timeout -k 10 300 python $B --seconds $sec > gpurun_out/pf${pf}_${sec}.json 2> gpurun_out/pf${pf}_${sec}.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/pf${pf}_${sec}.json'));print('pf=$pf sec=$sec', d['value'], d['ms_per_step'], d['breakdown'].get('_dit_block_linears'))" >> gpurun_out/pf_summary.txt
  done
done
exit 0
