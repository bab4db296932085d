#!/bin/bash
# Build an A/B variant of the library: gemm.hip recompiled with extra defines, linked with the other
# objects of the current build.  Usage: bash tools/build_ab.sh NAME "-DFOO=1"   -> lib/ab/NAME.so
set -e
cd "$(dirname "$0")/../ace-step-1.5-ggml_amd/csrc"
NAME=$1; DEFS=$2
B=../build; OUT=../acestep_mi355x/lib/ab; mkdir -p $OUT $B/ab_$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unused-result \
    -munsafe-fp-atomics $DEFS -c kernels/gemm.hip -o $B/ab_$NAME/k_gemm.o
OBJS=$(ls $B/k_*.o $B/r_*.o | grep -v "/k_gemm.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o $OUT/$NAME.so $B/ab_$NAME/k_gemm.o $OBJS
