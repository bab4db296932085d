// Per-token attention operand preparation shared by attn_prep_kernel (ops.hip) and the QKV GEMM's fused
// epilogue (gemm.hip, EPI_QKV_PREP), so both produce the same bits:
//   q/k heads: per-head RMSNorm over D = 128 with the q_norm / k_norm weights, then NEOX RoPE
//              (acestep_dit_model.cpp:1198-1210), fp16 hi (+ lo = fp16(x - hi)) rows [b][head][n][128];
//   v heads:   V^T [b][kvh][d][n] in the attention kernel's key order (vperm inside groups of 16).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace acemi {

// Separately rounded f32 operations (the reference's ggml ops round after every op).  HIP's __fmul_rn /
// __fadd_rn are plain operators, and hipcc's default -ffp-contract=fast fuses a product into a following add
// even across them (one rounding instead of two: the device Euler update x - v*dt came out 1 ulp off torch's
// and the oracle's).  The kernels build with -ffp-contract=fast-honor-pragmas, so contract(off) here holds.
__device__ __forceinline__ float rn_mul(float a, float b) {
#pragma clang fp contract(off)
    return a * b;
}
__device__ __forceinline__ float rn_add(float a, float b) {
#pragma clang fp contract(off)
    return a + b;
}
__device__ __forceinline__ float rn_sub(float a, float b) {
#pragma clang fp contract(off)
    return a - b;
}
__device__ __forceinline__ float rn_div(float a, float b) {
#pragma clang fp contract(off)
    return a / b;
}

namespace prep {

__device__ __forceinline__ uint16_t f16_bits(float f) {
    _Float16 h = (_Float16)f;
    return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float f16_lo(float v) { return v - (float)__builtin_bit_cast(_Float16, f16_bits(v)); }
__device__ __forceinline__ uint2 pk4(float p, float q, float r, float t) {
    return make_uint2((uint32_t)f16_bits(p) | ((uint32_t)f16_bits(q) << 16),
                      (uint32_t)f16_bits(r) | ((uint32_t)f16_bits(t) << 16));
}

// Key order of V^T inside a group of 16: the attention kernel's P^T registers hold keys
// (r & 3) + 8 * (r >> 2) + 4 * half, so the 4-key sub-groups 1 and 2 trade places.
__device__ __forceinline__ int vperm(int k) {
    const int w = k & 15;
    const int g = w >> 2;
    const int gp = (g == 1) ? 2 : (g == 2 ? 1 : g);
    return (k & ~15) | (gp << 2) | (w & 3);
}

// ---- fp8 (OCP e4m3) operand planes of the f8c attention mode (attention.hip, AttnArgs::f8): the lo plane of a
// q / k head row holds 256 bytes instead of 128 fp16 lo values -- Q: [fp8(x) | fp8(2^11 (x - f16(x)))],
// K: [fp8(2^11 (x - f16(x))) | fp8(x)] (d order), so that one K=256 block-scaled fp8 MFMA chain forms
// Kl.Qh + Kh.Ql (the 2^-11 goes into the MFMA's block scale); V^T's lo plane holds, per 64-key tile of a d row,
// [fp8(2^11 (v - f16(v))) | fp8(v)] (64 bytes each) in the P^T register order of the attention kernel (v8pos).
constexpr float F8_LO_SCALE = 2048.0f;  // 2^11: lo parts of fp16-rounded values back into e4m3's normal range
__device__ __forceinline__ uint32_t f8_pack4(float a, float b, float c, float d) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
    return (uint32_t)w;
}
__device__ __forceinline__ uint32_t f8_lo_pack4(float a, float b, float c, float d) {
    return f8_pack4(f16_lo(a) * F8_LO_SCALE, f16_lo(b) * F8_LO_SCALE, f16_lo(c) * F8_LO_SCALE, f16_lo(d) * F8_LO_SCALE);
}
// byte position inside a 64-key tile's 64-byte fp8 V segment of key w (0..15) of 16-key group G (0..3): the
// attention kernel's lane half h = (w >> 2) & 1 holds the 32 keys 32 (c >> 4) + 8 ((c >> 2) & 3) + 4 h + (c & 3)
// (its S^T accumulator registers c = 16 t + r) as bytes c of its fp8 B operand
__device__ __forceinline__ int v8pos(int G, int w) {
    return 32 * ((w >> 2) & 1) + 16 * (G >> 1) + 8 * (G & 1) + 4 * (w >> 3) + (w & 3);
}

// One token's head row, 16 lanes per token (lane & 15 = d / 4): y[0..3] = dims d..d+3, y[4..7] = dims
// 64+d..64+d+3 (the NEOX rotation pairs d with d+64 inside the lane).  has_w: RMSNorm with weights w0 / w1
// (dims d.. / 64+d..); has_rope: rotate by the position's c4 / s4 (dims d..d+3 of its RoPE row).  Writes fp16
// hi into dst[0..127] and, when plane > 0, lo into dst[plane..].
__device__ __forceinline__ void head_row_v(float (&y)[8], bool has_w, const float4& w0, const float4& w1, int d,
                                           float eps, bool has_rope, const float4& c4, const float4& s4,
                                           uint16_t* dst, int64_t plane, int f8 = 0) {
    if (has_w) {
        float ss = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += y[j] * y[j];
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);  // the token's 16 lanes
        const float sc = 1.0f / sqrtf(ss / 128.0f + eps);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) y[j] = rn_mul(rn_mul(y[j], sc), wv[j]);
    }
    float r[8];
    if (has_rope) {
        const float c[4] = {c4.x, c4.y, c4.z, c4.w}, s[4] = {s4.x, s4.y, s4.z, s4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            r[j] = rn_sub(rn_mul(y[j], c[j]), rn_mul(y[4 + j], s[j]));
            r[4 + j] = rn_add(rn_mul(y[j], s[j]), rn_mul(y[4 + j], c[j]));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = y[j];
    }
    *(uint2*)(dst + d) = pk4(r[0], r[1], r[2], r[3]);
    *(uint2*)(dst + 64 + d) = pk4(r[4], r[5], r[6], r[7]);
    if (plane > 0 && f8) {  // f8 = 1: q row [hi8 | lo8], 2: k row [lo8 | hi8]
        uint8_t* row8 = reinterpret_cast<uint8_t*>(dst + plane);
        const int hoff = f8 == 1 ? 0 : 128, loff = 128 - hoff;
        *(uint32_t*)(row8 + hoff + d) = f8_pack4(r[0], r[1], r[2], r[3]);
        *(uint32_t*)(row8 + hoff + 64 + d) = f8_pack4(r[4], r[5], r[6], r[7]);
        *(uint32_t*)(row8 + loff + d) = f8_lo_pack4(r[0], r[1], r[2], r[3]);
        *(uint32_t*)(row8 + loff + 64 + d) = f8_lo_pack4(r[4], r[5], r[6], r[7]);
    } else if (plane > 0) {
        *(uint2*)(dst + plane + d) = pk4(f16_lo(r[0]), f16_lo(r[1]), f16_lo(r[2]), f16_lo(r[3]));
        *(uint2*)(dst + plane + 64 + d) = pk4(f16_lo(r[4]), f16_lo(r[5]), f16_lo(r[6]), f16_lo(r[7]));
    }
}

// head_row_v with the weights and RoPE row read here: w = norm weights or null (plain copy), cs / sn = the
// position's RoPE row (+ d) or null
__device__ __forceinline__ void head_row(float (&y)[8], const float* w, int d, float eps, const float* cs,
                                         const float* sn, uint16_t* dst, int64_t plane, int f8 = 0) {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    head_row_v(y, w != nullptr, w ? *(const float4*)(w + d) : z, w ? *(const float4*)(w + 64 + d) : z, d, eps,
               cs != nullptr, cs ? *(const float4*)cs : z, cs ? *(const float4*)sn : z, dst, plane, f8);
}

// 16 values of one V^T row segment (keys g0 + vperm(k), k = 0..15) as fp16 hi / lo words.
__device__ __forceinline__ void v_words(const float (&v)[16], uint32_t (&wv)[8], uint32_t (&wl)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint16_t h0 = f16_bits(v[2 * j]), h1 = f16_bits(v[2 * j + 1]);
        wv[j] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        wl[j] = (uint32_t)f16_bits(v[2 * j] - (float)__builtin_bit_cast(_Float16, h0)) |
                ((uint32_t)f16_bits(v[2 * j + 1] - (float)__builtin_bit_cast(_Float16, h1)) << 16);
    }
}

// The f8 V^T lo plane of one 16-key group (natural-order values vn[w] = key g0 + w, g0 % 16 == 0) of the d row
// whose fp16 image starts at vrow (uint16 units, key 0): fp8 lo / hi bytes at v8pos inside the group's 64-key
// tile; `have` (bit w) selects the keys this caller owns (all 16: four dword stores per half)
__device__ __forceinline__ void v_store8(const float (&vn)[16], uint16_t* vrow, int64_t plane, int g0, uint32_t have) {
    uint8_t* tile8 = reinterpret_cast<uint8_t*>(vrow + plane) + 2 * (g0 & ~63);
    const int G = (g0 >> 4) & 3;
    if (have == 0xffffu) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {  // q = (w >> 3, (w >> 2) & 1): keys 8 (q >> 1) + 4 (q & 1) + 0..3
            const int w0 = 8 * (q >> 1) + 4 * (q & 1);
            const int pos = v8pos(G, w0);
            *(uint32_t*)(tile8 + pos) = f8_lo_pack4(vn[w0], vn[w0 + 1], vn[w0 + 2], vn[w0 + 3]);
            *(uint32_t*)(tile8 + 64 + pos) = f8_pack4(vn[w0], vn[w0 + 1], vn[w0 + 2], vn[w0 + 3]);
        }
    } else {
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            if (!((have >> w) & 1u)) continue;
            const uint32_t lo = f8_lo_pack4(vn[w], 0.f, 0.f, 0.f), hi = f8_pack4(vn[w], 0.f, 0.f, 0.f);
            tile8[v8pos(G, w)] = (uint8_t)lo;
            tile8[64 + v8pos(G, w)] = (uint8_t)hi;
        }
    }
}

}  // namespace prep
}  // namespace acemi
