cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; L=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab
for v in base new base new; do
  ACE_MI_LIB=$L/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/abp/$v$((n++))" -o s --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/abp_$v.log 2>&1 || exit $?
done
