#!/bin/bash
# A/B build (CPU side): a library whose listed kernel sources are compiled with extra flags (e.g. -DACEMI_GEMM_ABLATE=1);
# every other object is the regular build's.  Default: a self-test library lib/ab/<name>_st.so, loaded on the GPU box with
# ACE_MI_SELFTEST_LIB=...; PRODUCT=1: a product library lib/ab/<name>.so (ACE_MI_LIB=..., what bench.py loads).
# NOSLP: the kernels built with -fno-slp-vectorize (default: the Makefile's KFLAGS_*: gemm gemm_q gemm_a8 ops).
# Usage: [PRODUCT=1] [NOSLP="gemm_q gemm_a8"] tools/build_ab.sh NAME "EXTRA FLAGS" gemm [attention ...]
set -e
name=$1; flags=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/ace-step-1.5-ggml_amd/csrc; bld=$root/ace-step-1.5-ggml_amd/build; out=$root/ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab
make -C "$src" -j8 >/dev/null  # (run the A/B builds one at a time: concurrent runs race on the regular objects)
mkdir -p "$bld/ab_$name" "$out"
noslp=" ${NOSLP-gemm gemm_q gemm_a8 ops} "
objs=()
for k in gemm gemm_q gemm_a8 attention ops vae; do
    if [[ " $* " == *" $k "* ]]; then
        kf=""; [[ "$noslp" == *" $k "* ]] && kf="-fno-slp-vectorize"
        (cd "$bld/ab_$name" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -save-temps=obj -std=c++17 -fPIC -fvisibility=hidden \
            -Wall -Wno-unused-result -ffp-contract=fast-honor-pragmas -munsafe-fp-atomics $kf $flags -c "$src/kernels/$k.hip" \
            -o "$bld/ab_$name/k_$k.o")
        objs+=("$bld/ab_$name/k_$k.o")
    else
        objs+=("$bld/k_$k.o")
    fi
done
if [ -n "$PRODUCT" ]; then
    rt=$(ls "$bld"/r_*.o | grep -v "r_test_hooks_st.o\|r_selftest.o")
    lib="$out/${name}.so"
else
    rt=$(ls "$bld"/r_*.o | grep -v "r_test_hooks.o")
    lib="$out/${name}_st.so"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o "$lib" "${objs[@]}" $rt
echo "$lib"
