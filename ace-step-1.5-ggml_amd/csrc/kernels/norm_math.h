// RMSNorm + AdaLN modulation (acestep_dit_model.cpp:1097-1106 rms_norm, :1477-1481 / :1522-1526 / :1545-1549
// modulate): y = ((x * 1/sqrt(mean(x^2) + eps)) * w) * (1 + scale) + shift, each op rounded once.
// One fixed summation order for sum(x^2), shared by the standalone kernel (ops.hip rmsnorm_mod_canon_kernel) and
// the residual GEMM epilogue that produces the row and normalises it in place (gemm_common.h norm_fuse), so a
// row's activation has the same bits whichever of the two wrote it:
//   chunk q = columns 16q .. 16q+15: each x^2 rounded, summed by a butterfly over 16 lanes (xor 1, 2, 4, 8 -- a
//   perfect binary tree in column order, the same value in every lane);
//   row = a perfect binary tree over the chunks in column order, padded with zero leaves to a power of two (a
//   zero leaf adds nothing, so any zero-padded size gives the same sum: the GEMM tiles combine whole aligned
//   subtrees of 16 * 2^k columns and the reader finishes the tree over the tiles' partials).
#pragma once

#include "prep_math.h"

namespace acemi {
namespace normc {

// sum of v over the 16 lanes sharing lane >> 4
__device__ __forceinline__ float chunk16(float v) {
    v = rn_add(v, __shfl_xor(v, 1));
    v = rn_add(v, __shfl_xor(v, 2));
    v = rn_add(v, __shfl_xor(v, 4));
    v = rn_add(v, __shfl_xor(v, 8));
    return v;
}

constexpr int pow2_ceil(int n) { return n <= 1 ? 1 : 2 * pow2_ceil((n + 1) / 2); }

// perfect binary tree over a[0..N) in order, zero-padded to a power of two
template <int N>
__device__ __forceinline__ float tree(const float (&a)[N]) {
    constexpr int P = pow2_ceil(N);
    float t[P];
#pragma unroll
    for (int i = 0; i < P; ++i) t[i] = i < N ? a[i] : 0.f;
#pragma unroll
    for (int s = 1; s < P; s *= 2)
#pragma unroll
        for (int i = 0; i < P; i += 2 * s) t[i] = rn_add(t[i], t[i + s]);
    return t[0];
}

__device__ __forceinline__ float rms_scale(float ss, int H, float eps) {
    return 1.0f / sqrtf(rn_add(rn_div(ss, (float)H), eps));
}

// ((x * sc) * w) * s1 + shift, s1 = 1 + scale (rounded once, by the caller); mod = false: (x * sc) * w
__device__ __forceinline__ float modulate(float x, float sc, float w, bool mod, float s1, float sh) {
    float t = rn_mul(rn_mul(x, sc), w);
    if (mod) t = rn_add(rn_mul(t, s1), sh);
    return t;
}

}  // namespace normc
}  // namespace acemi
