#!/bin/bash
# A/B build (CPU side): a self-test library lib/ab/<name>_st.so whose listed kernel sources are compiled with extra
# flags (e.g. -DACEMI_GEMM_ABLATE=1); every other object is the regular build's.  Load it on the GPU box with
# ACE_MI_SELFTEST_LIB=ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab/<name>_st.so.
# Usage: tools/build_ab.sh NAME "EXTRA FLAGS" gemm [attention ...]
set -e
name=$1; flags=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/ace-step-1.5-ggml_amd/csrc; bld=$root/ace-step-1.5-ggml_amd/build; out=$root/ace-step-1.5-ggml_amd/acestep_mi355x/lib/ab
make -C "$src" -j8 >/dev/null  # (run the A/B builds one at a time: concurrent runs race on the regular objects)
mkdir -p "$bld/ab_$name" "$out"
objs=()
for k in gemm gemm_q attention ops vae; do
    if [[ " $* " == *" $k "* ]]; then
        kf=""; [ "$k" = gemm_q ] || [ "$k" = gemm ] || [ "$k" = ops ] && kf="-fno-slp-vectorize"  # (as the Makefile's KFLAGS_gemm*)
        (cd "$bld/ab_$name" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -save-temps=obj -std=c++17 -fPIC -fvisibility=hidden \
            -Wall -Wno-unused-result -ffp-contract=fast-honor-pragmas -munsafe-fp-atomics $kf $flags -c "$src/kernels/$k.hip" \
            -o "$bld/ab_$name/k_$k.o")
        objs+=("$bld/ab_$name/k_$k.o")
    else
        objs+=("$bld/k_$k.o")
    fi
done
rt=$(ls "$bld"/r_*.o | grep -v "r_test_hooks.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o "$out/${name}_st.so" "${objs[@]}" $rt
echo "$out/${name}_st.so"
