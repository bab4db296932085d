// ggml-faithful quantized-activation linears (ACE_MI_QUANT_ACT=q8, DitEngine::forward_qact).
//
// ggml's mul_mat(W, x) with W in a block format converts the f32 activation rows x to W's vec_dot_type before the
// dot product (Q8_0 weights: Q8_0 blocks, x86 quantize_row_q8_0; Q4_K / Q6_K: Q8_K blocks, quantize_row_q8_K_ref;
// block layouts ggml-metal-embed.metal:222-227, quantize :3110-3128) and sums d_w * d_a * (integer dot of the two
// blocks) in f32 (vec_dot_q8_0_q8_0 / vec_dot_q4_K_q8_K / vec_dot_q6_K_q8_K).  The product path multiplies bf16
// activations with bf16(dequant(W)) instead (kernels/gemm_q.hip); this file is the arithmetic ggml actually runs,
// for parity against the oracle's ggml semantics (oracle/ggml_numerics.py: convert_activation + mul_mat).
//
// The GEMM takes one 32-value block per step: v_mfma_i32_16x16x32_i8 gives the exact integer dot of an activation
// block with a weight block (Q6_K: two MFMAs, one per 16-value half, each with the other half's weights zeroed), and
// the f32 accumulator adds isum * (d_w * d_a) (Q4_K: d_a * (d*sc * isum - dmin*m * bsum_a)).  Operands come straight
// from global memory into the MFMA registers (no LDS staging): this is a parity mode, not a throughput path.
#include "gemm_common.h"

namespace acemi {
namespace {
using namespace gemm_detail;

typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int A8_BM = 128, A8_BN = 128;
constexpr int A8_PREP_SMEM = 64 * PREP_LD * 4;  // EPI_QKV_PREP: the 128 x 128 tile in two 64-row chunks

struct A8Params {
    GemmParams g;  // M, N, K and the epilogue
    const int8_t* aq;
    const float* as;
    const float* ab;
    int64_t ld_s;
    const void* wq;
    const float* ws;
};

// ---------------------------------------------------------------- activation quantization
// Q8_0 (x86 quantize_row_q8_0): per 32 values amax = max|x|, d = amax / 127 stored as fp16, id = 127 / amax (0 for
// an all-zero block), q = round-half-even(x * id).  One thread per block.
__global__ void __launch_bounds__(256) quantize_q8_0_kernel(const float* __restrict__ x, int64_t ldx, int M, int K,
                                                            bool silu_in, int8_t* __restrict__ q, uint16_t* __restrict__ q16,
                                                            float* __restrict__ s, int64_t ld_s) {
    const int nb = K >> 5;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= (int64_t)M * nb) return;
    const int m = (int)(t / nb), b = (int)(t - (int64_t)m * nb);
    const float* xr = x + (int64_t)m * ldx + b * 32;
    float v[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float4 f = *(const float4*)(xr + 4 * i);
        v[4 * i] = f.x;
        v[4 * i + 1] = f.y;
        v[4 * i + 2] = f.z;
        v[4 * i + 3] = f.w;
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        if (silu_in) v[i] = silu_f(v[i]);
        amax = fmaxf(amax, fabsf(v[i]));
    }
    const float d = amax / 127.0f;
    const float id = amax != 0.0f ? 127.0f / amax : 0.0f;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t p = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) p |= ((uint32_t)(int)__builtin_rintf(rn_mul(v[4 * i + j], id)) & 0xffu) << (8 * j);
        w[i] = p;
    }
    if (q) {
        int8_t* qr = q + (int64_t)m * K + b * 32;
        *(uint4*)qr = make_uint4(w[0], w[1], w[2], w[3]);
        *(uint4*)(qr + 16) = make_uint4(w[4], w[5], w[6], w[7]);
    }
    if (q16) {  // bf16(q): the integers exactly (the bf16-MFMA Q8_0 GEMM's A operand)
        uint16_t* hr = q16 + (int64_t)m * K + b * 32;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            uint32_t h[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t p = w[2 * i + (j >> 1)];
                const int q0 = (int)(int8_t)((p >> (16 * (j & 1))) & 0xff), q1 = (int)(int8_t)((p >> (16 * (j & 1) + 8)) & 0xff);
                h[j] = (__float_as_uint((float)q0) >> 16) | (__float_as_uint((float)q1) & 0xffff0000u);
            }
            *(uint4*)(hr + 8 * i) = make_uint4(h[0], h[1], h[2], h[3]);
        }
    }
    s[(int64_t)b * ld_s + m] = (float)(_Float16)d;
}

// Q8_K (quantize_row_q8_K_ref): per 256 values max = the value of largest magnitude (first one on ties),
// iscale = -127 / max, q = min(127, nearest_int(iscale * x)), d = 1 / iscale; an all-zero block is d = 0, q = 0.
// Eight lanes per block, 32 values each; the lane's block sum feeds the Q4_K min term (ggml's bsums per 16, summed
// in pairs by vec_dot_q4_K_q8_K).
__global__ void __launch_bounds__(256) quantize_q8_k_kernel(const float* __restrict__ x, int64_t ldx, int M, int K,
                                                            bool silu_in, int8_t* __restrict__ q, float* __restrict__ s,
                                                            float* __restrict__ bs, int64_t ld_s) {
    const int nb = K >> 8;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool live = t < (int64_t)M * nb * 8;  // whole 8-lane groups are live or dead together
    const int64_t blk = live ? t >> 3 : 0;
    const int part = (int)(t & 7);
    const int m = (int)(blk / nb), b = (int)(blk - (int64_t)m * nb);
    const float* xr = x + (int64_t)m * ldx + b * 256 + part * 32;
    float v[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float4 f = *(const float4*)(xr + 4 * i);
        v[4 * i] = f.x;
        v[4 * i + 1] = f.y;
        v[4 * i + 2] = f.z;
        v[4 * i + 3] = f.w;
    }
    float amax = 0.f, mx = 0.f;
    int idx = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        if (silu_in) v[i] = silu_f(v[i]);
        const float ax = fabsf(v[i]);
        if (ax > amax) {
            amax = ax;
            mx = v[i];
            idx = i;
        }
    }
    idx += part * 32;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
        const float a2 = __shfl_xor(amax, o), m2 = __shfl_xor(mx, o);
        const int i2 = __shfl_xor(idx, o);
        if (a2 > amax || (a2 == amax && i2 < idx)) {
            amax = a2;
            mx = m2;
            idx = i2;
        }
    }
    if (!live) return;
    int8_t* qr = q + (int64_t)m * K + b * 256 + part * 32;
    const int64_t so = (int64_t)(b * 8 + part) * ld_s + m;
    if (amax == 0.0f) {
        *(uint4*)qr = make_uint4(0, 0, 0, 0);
        *(uint4*)(qr + 16) = make_uint4(0, 0, 0, 0);
        s[so] = 0.f;
        bs[so] = 0.f;
        return;
    }
    const float iscale = -127.0f / mx;
    uint32_t w[8];
    int sum = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t p = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int qi = min(127, (int)__builtin_rintf(rn_mul(iscale, v[4 * i + j])));
            sum += qi;
            p |= ((uint32_t)qi & 0xffu) << (8 * j);
        }
        w[i] = p;
    }
    *(uint4*)qr = make_uint4(w[0], w[1], w[2], w[3]);
    *(uint4*)(qr + 16) = make_uint4(w[4], w[5], w[6], w[7]);
    s[so] = 1.0f / iscale;
    bs[so] = (float)sum;
}

// ---------------------------------------------------------------- f32 producers
// launch_rmsnorm_mod's arithmetic (ops.hip rmsnorm_mod_kernel), f32 out
template <int VPT>
__global__ void __launch_bounds__(256) rmsnorm_mod_f32_kernel(const float* __restrict__ x, int H, const float* __restrict__ w,
                                                              const float* __restrict__ scale, const float* __restrict__ shift,
                                                              int64_t mod_stride, int rows_per_item, float eps,
                                                              float* __restrict__ out) {
    const int m = blockIdx.x;
    const float* xr = x + (int64_t)m * H;
    __shared__ float red[4];
    float4 v[VPT];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const int i = (threadIdx.x + k * 256) * 4;
        v[k] = i < H ? *(const float4*)(xr + i) : make_float4(0.f, 0.f, 0.f, 0.f);
        ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const float tot = red[0] + red[1] + red[2] + red[3];
    const float sc = 1.0f / sqrtf(tot / (float)H + eps);
    const int item = m / rows_per_item;
    const float* scp = scale ? scale + (int64_t)item * mod_stride : nullptr;
    const float* shp = shift ? shift + (int64_t)item * mod_stride : nullptr;
    float* orow = out + (int64_t)m * H;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const int i = (threadIdx.x + k * 256) * 4;
        if (i >= H) break;
        const float4 wv = *(const float4*)(w + i);
        const float y[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        const float ww[4] = {wv.x, wv.y, wv.z, wv.w};
        float s4[4] = {0.f, 0.f, 0.f, 0.f}, h4[4] = {0.f, 0.f, 0.f, 0.f};
        if (scp) {
            const float4 a4 = *(const float4*)(scp + i);
            const float4 b4 = *(const float4*)(shp + i);
            s4[0] = a4.x; s4[1] = a4.y; s4[2] = a4.z; s4[3] = a4.w;
            h4[0] = b4.x; h4[1] = b4.y; h4[2] = b4.z; h4[3] = b4.w;
        }
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float t = rn_mul(rn_mul(y[j], sc), ww[j]);
            if (scp) t = rn_add(rn_mul(t, rn_add(s4[j], 1.0f)), h4[j]);
            o[j] = t;
        }
        *(float4*)(orow + i) = make_float4(o[0], o[1], o[2], o[3]);
    }
}

// input pack + patchify (acestep_dit_model.cpp:1350-1380), f32 out (ops.hip pack_input_kernel's indexing)
__global__ void pack_input_f32_kernel(const float* __restrict__ hidden, const float* __restrict__ context, int B, int T,
                                      int Np, int P, int audio, int cdim, float* __restrict__ out) {
    const int cin = audio + cdim;
    const int64_t total = (int64_t)B * Np * P * cin;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % cin);
        int64_t r = i / cin;
        const int k = (int)(r % P);
        r /= P;
        const int p = (int)(r % Np);
        const int b = (int)(r / Np);
        const int t = p * P + k;
        float v = 0.f;
        if (t < T) {
            if (c < cdim) {
                if (context) v = context[((int64_t)b * T + t) * cdim + c];
            } else {
                if (hidden) v = hidden[((int64_t)b * T + t) * audio + (c - cdim)];
            }
        }
        out[i] = v;
    }
}

// The epilogues of both Q8 GEMMs, on a wave's 4 x 4 grid of 16 x 16 accumulators (the bf16 form's C/D map)
template <int EPI, int SMEM, int TN = 4>
__device__ __forceinline__ void a8_epilogue(const GemmParams& p, f32x4 (&acc)[4][TN], int m0, int n0, int wm0, int wn0,
                                            int tid, char* smem) {
    static_assert(EPI != EPI_QKV_PREP || TN == 4, "the prep epilogue takes whole 128-column heads");
    const int lane = tid & 63, g = lane >> 4, c = lane & 15;
    const GemmEpilogue& e = p.e;
    if constexpr (EPI == EPI_QKV_PREP) {
        qkv_prep_tile<A8_BM, 4, 4, TN, SMEM>(p, acc, m0, n0, wm0, wn0, tid, smem);
    } else if constexpr (EPI == EPI_SWIGLU_F32) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm0 + i * 16 + 4 * g + r;
                if (m >= p.M) continue;
#pragma unroll
                for (int j = 0; j < TN; j += 2) {
                    const int n = n0 + wn0 + j * 16;  // gate columns n .. n + 15, up columns n + 16 .. n + 31
                    e.c_f32[(int64_t)m * e.ldc + (n >> 1) + c] = rn_mul(silu_f(acc[i][j][r]), acc[i][j + 1][r]);
                }
            }
    } else {
        if constexpr (EPI == EPI_RESID || EPI == EPI_RESID_GATED) {
            if (e.bias) {  // x + (W x_a + b): the bias joins the product before the residual add
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const float bj = e.bias[n0 + wn0 + j * 16 + c];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[i][j][r] = rn_add(acc[i][j][r], bj);
                }
            }
        }
        gemm_epilogue<4, TN, false, EPI, 1024>(p, acc, m0 + wm0, n0 + wn0, lane);
    }
}

// ---------------------------------------------------------------- the GEMM
// 256 threads, a 128 x 128 tile as 2 x 2 waves of 64 x 64 (4 x 4 accumulators of 16 x 16).  i8 MFMA 16x16x32
// operands: lane l holds A row l & 15 / B column l & 15, k = 8 (l >> 4) .. + 7; result row 4 (l >> 4) + r,
// column l & 15 (the bf16 form's map).
template <int WQ, int EPI>
__global__ void __launch_bounds__(256) gemm_a8_kernel(A8Params p) {
    __shared__ __attribute__((aligned(16))) char smem[EPI == EPI_QKV_PREP ? A8_PREP_SMEM : 16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int M = p.g.M, K = p.g.K;
    int m0, n0;
    block_tile<A8_BM, A8_BN>(p.g, m0, n0);
    const int wm0 = (wid >> 1) * 64, wn0 = (wid & 1) * 64;
    const int g = lane >> 4, c = lane & 15;
    const int nb = K >> 5;
    const int8_t* arow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) arow[i] = p.aq + (int64_t)min(m0 + wm0 + i * 16 + c, M - 1) * K + 8 * g;
    const float* asb = p.as + m0 + wm0 + 4 * g;
    const float* abb = WQ == WF_Q4_K ? p.ab + m0 + wm0 + 4 * g : nullptr;
    int64_t wrow[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wrow[j] = n0 + wn0 + j * 16 + c;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const i32x4 zero = {0, 0, 0, 0};

    // one 32-value block's operands, loaded raw (the Q4_K unpack and the Q6_K half masks run at compute time, so the
    // next block's loads are in flight while this one's MFMAs and scaling run: a two-block software pipeline)
    struct Ops {
        long av[4], wv[4];
        float s0[4], s1[4];
        float4 sa[4], sb[4];
    };
    auto load = [&](int b, Ops& o) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o.av[i] = *(const long*)(arow[i] + b * 32);
            o.sa[i] = *(const float4*)(asb + (int64_t)b * p.ld_s + i * 16);
            if constexpr (WQ == WF_Q4_K) o.sb[i] = *(const float4*)(abb + (int64_t)b * p.ld_s + i * 16);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (WQ == WF_Q4_K) {
                // 16 bytes per block; byte i: low nibble k = 8 (i / 4) + i % 4, high nibble k + 4 (runtime/quant.h)
                o.wv[j] = (long)*(const uint32_t*)(static_cast<const uint8_t*>(p.wq) + wrow[j] * (K / 2) + b * 16 + 4 * g);
                const float2 sc = *(const float2*)(p.ws + (wrow[j] * nb + b) * 2);  // (d*sc, dmin*m)
                o.s0[j] = sc.x;
                o.s1[j] = sc.y;
            } else {
                o.wv[j] = *(const long*)(static_cast<const int8_t*>(p.wq) + wrow[j] * K + b * 32 + 8 * g);
                if constexpr (WQ == WF_Q6_K) {
                    const float2 sc = *(const float2*)(p.ws + (wrow[j] * nb + b) * 2);  // d*sc of the two 16-halves
                    o.s0[j] = sc.x;
                    o.s1[j] = sc.y;
                } else {
                    o.s0[j] = p.ws[wrow[j] * nb + b];
                }
            }
        }
    };
    auto compute = [&](Ops& o) {
        long wv[4], wv2[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if constexpr (WQ == WF_Q4_K) {
                const uint32_t u = (uint32_t)o.wv[j];
                const uint64_t lo = u & 0x0f0f0f0fu, hi = (u >> 4) & 0x0f0f0f0fu;
                wv[j] = (long)(lo | (hi << 32));
            } else if constexpr (WQ == WF_Q6_K) {
                wv2[j] = g < 2 ? 0 : o.wv[j];  // second half: k 16..31 (lanes 32..63)
                wv[j] = g < 2 ? o.wv[j] : 0;
            } else {
                wv[j] = o.wv[j];
            }
        }
        mfma_war_guard();  // the operands' VALU writes are done before the MFMAs read them
        i32x4 is[4][4], is2[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                is[i][j] = __builtin_amdgcn_mfma_i32_16x16x32_i8(o.av[i], wv[j], zero, 0, 0, 0);
                if constexpr (WQ == WF_Q6_K) is2[i][j] = __builtin_amdgcn_mfma_i32_16x16x32_i8(o.av[i], wv2[j], zero, 0, 0, 0);
            }
        mfma_war_guard();  // no operand register is rewritten while an MFMA may still read it
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float a4[4] = {o.sa[i].x, o.sa[i].y, o.sa[i].z, o.sa[i].w};
            const float b4[4] = {o.sb[i].x, o.sb[i].y, o.sb[i].z, o.sb[i].w};
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (WQ == WF_Q8_0) {
                        // acc += sumi * (d_w * d_a) as one FMA: ggml's AVX2 vec_dot_q8_0_q8_0 (_mm256_fmadd_ps)
                        acc[i][j][r] = __builtin_fmaf((float)is[i][j][r], rn_mul(o.s0[j], a4[r]), acc[i][j][r]);
                    } else if constexpr (WQ == WF_Q4_K) {
                        const float v = rn_mul(a4[r], rn_sub(rn_mul(o.s0[j], (float)is[i][j][r]), rn_mul(o.s1[j], b4[r])));
                        acc[i][j][r] = rn_add(acc[i][j][r], v);
                    } else {
                        const float v =
                            rn_mul(a4[r], rn_add(rn_mul(o.s0[j], (float)is[i][j][r]), rn_mul(o.s1[j], (float)is2[i][j][r])));
                        acc[i][j][r] = rn_add(acc[i][j][r], v);
                    }
                }
        }
    };
    Ops o0, o1;
    o0.sb[0] = o0.sb[1] = o0.sb[2] = o0.sb[3] = make_float4(0.f, 0.f, 0.f, 0.f);
    o1.sb[0] = o1.sb[1] = o1.sb[2] = o1.sb[3] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 4; ++j) o0.s1[j] = o1.s1[j] = 0.f;
    load(0, o0);
    for (int b = 0; b < nb; b += 2) {
        if (b + 1 < nb) load(b + 1, o1);
        compute(o0);
        if (b + 1 < nb) {
            if (b + 2 < nb) load(b + 2, o0);
            compute(o1);
        }
    }

    a8_epilogue<EPI, (EPI == EPI_QKV_PREP ? A8_PREP_SMEM : 16)>(p.g, acc, m0, n0, wm0, wn0, tid, smem);
}

// ---------------------------------------------------------------- Q8_0 on the bf16 MFMA (round 6)
// ggml's Q8_0 block dot is exact in a bf16 MFMA: every q of an activation or weight block is an integer in [-127, 127]
// (exact in bf16), each product is exact in f32 and so is the 32-term block sum (|sum| <= 32 * 127^2 < 2^24).  So
// v_mfma_f32_16x16x32_bf16 over ONE 32-value block, accumulator zero, returns the block's integer dot already in f32 --
// the value v_mfma_i32_16x16x32_i8 returns, with no convert -- and the per-block scaling is acc = fma(dot, d_w * d_a,
// acc) in block order, exactly the kernel above (same bits).  The operands are the activation quantizer's bf16(q)
// rows and a bf16(q) image of the weight plane (launch_q8_image; the q8 mode keeps one per matrix), so the dense
// GEMM's machinery applies: 128 x 128 tiles of 2 x 2 waves (64 x 64 each), BK = 64 (two blocks), both operands staged
// by LDS-DMA into a double-buffered, XOR-swizzled LDS image (released early: every fragment is read before the
// barrier) and the two blocks' d_a [2][128] and d_w [128][2] into a three-slot ring read during the MFMAs, fragment
// reads as inline asm with one counted vmcnt (block 1's fragments read under block 0's MFMAs), two workgroups per CU.
// Per block and 16 x 16 tile: one MFMA
// and, per output, one multiply (d_w * d_a) and one FMA.
constexpr int A8S_STAGE = (A8_BM + A8_BN) * 128;  // A and W k-tiles, 128-byte rows (two buffers; BN = 64 uses less)
constexpr int A8S_SC = 2 * A8_BM * 4 + A8_BN * 2 * 4;  // d_a [2][BM] + d_w [BN][2] of one k-tile (a three-slot ring)
constexpr int A8S_DA = 0, A8S_DW = 2 * A8_BM * 4;
constexpr int A8S_SMEM = 2 * A8S_STAGE + 3 * A8S_SC;  // 71 680 B: two workgroups per CU
static_assert(A8S_SMEM >= A8_PREP_SMEM, "the prep epilogue reuses the stage buffers");

struct A8SParams {
    GemmParams g;        // M, N, K and the epilogue
    const uint16_t* a;   // bf16(q) activation rows [M][K]
    const uint16_t* w;   // bf16(q) weight image [N][K]
    const float* as;     // d_a [K/32][ld_s]
    int64_t ld_s;
    const float* ws;     // d_w [N][K/32]
};

template <int OFF>
__device__ __forceinline__ uint2 ds_read_b64_off(uint32_t addr) {
    typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
    u32x2_t v;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return make_uint2(v[0], v[1]);
}

// BN = 128 (2 x 2 waves of 64 x 64) or 64 (waves of 64 x 32: grids that a 128-wide tile leaves under one round of two
// workgroups per CU, e.g. the N = 2048 projections at M = 3000: 384 tiles for 512 slots)
template <int EPI, int BN = 128>
__global__ void __launch_bounds__(256, 2) gemm_a8s_kernel(A8SParams p) {
    constexpr int TM = 4, TN = BN / 32, BK = 64, ROWB = 128;
    constexpr int GA = A8_BM / 32, GW = BN / 32;  // 1 KiB A / W pieces per wave per k-tile
    constexpr int G_AW = GA + GW;
    constexpr int G = G_AW + 2;                    // + one d_a and one d_w dword piece
    constexpr int STAGE = (A8_BM + BN) * ROWB;
    __shared__ __attribute__((aligned(16))) char smem[A8S_SMEM];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int M = p.g.M, K = p.g.K;
    const int nb = K >> 5, nk = K / BK;
    int m0, n0;
    block_tile<A8_BM, BN>(p.g, m0, n0);
    const int wm0 = (wid >> 1) * 64, wn0 = (wid & 1) * (BN / 2);
    const int g = lane >> 4, c = lane & 15;

    // LDS-DMA sources as 32-bit element offsets (pieces j < G_AW / 2 are A rows, the rest W rows): 64-bit pointers
    // cost the registers that keep this kernel at two workgroups per CU without scratch
    int src[G_AW];
#pragma unroll
    for (int j = 0; j < G_AW; ++j) {
        const int row = (wid + 4 * j) * 8 + (lane >> 3);
        const int ch = (lane & 7) ^ swz(row);
        src[j] = j < GA ? min(m0 + row, M - 1) * K + ch * 8 : (n0 + row - A8_BM) * K + ch * 8;
    }
    // scale pieces: element e = 64 wid + lane of d_a [2][BM] (block e / BM, row e % BM; rows past M read the zero-padded
    // plane, ld_s >= M rounded up to 128) and of d_w [BN][2] (column e / 2, block e % 2; BN = 64: waves 2, 3 re-read
    // column BN - 1 into the unused half of the slot's d_w region)
    const int e = 64 * wid + lane;
    const float* sa = p.as + (int64_t)(e / A8_BM) * p.ld_s + m0 + e % A8_BM;
    const int ew = min(e, 2 * BN - 1);
    const float* sw = p.ws + (int64_t)(n0 + (ew >> 1)) * nb + (ew & 1);
    auto stage = [&](int buf, int kt) {
        char* base = smem + buf * STAGE;
#pragma unroll
        for (int j = 0; j < G_AW; ++j)
            __builtin_amdgcn_global_load_lds((const void*)((j < GA ? p.a : p.w) + (src[j] + kt * BK)),
                                             (lds_void*)(base + (wid + 4 * j) * 1024), 16, 0, 0);
        char* sc = smem + 2 * STAGE + (kt % 3) * A8S_SC;
        __builtin_amdgcn_global_load_lds((const void*)(sa + (int64_t)(2 * kt) * p.ld_s), (lds_void*)(sc + A8S_DA + wid * 256),
                                         4, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(sw + 2 * kt), (lds_void*)(sc + A8S_DW + wid * 256), 4, 0, 0);
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const int lrow = lane & 15, lchunk = lane >> 4;
    uint4 a[2][TM], b[2][TN];  // the two blocks' fragments (block 1's are read under block 0's MFMAs)
    uint4 da[2][TM];           // d_a of this lane's 4 rows of each 16-row tile, per block
    uint2 dw[TN];        // d_w of this lane's column of each 16-column tile, both blocks
    auto read_frags = [&](int buf, auto kk_c) {
        constexpr int kk = decltype(kk_c)::value;
        const uint32_t sbase = lds0 + buf * STAGE;
        const int ch = (kk * 4 + lchunk) ^ ((lrow >> 1) & 7);
        const uint32_t bb = sbase + A8_BM * ROWB + (wn0 + lrow) * ROWB + ch * 16;
        const uint32_t ab = sbase + (wm0 + lrow) * ROWB + ch * 16;
        static_for<0, TN>([&](auto j_c) {
            constexpr int j = decltype(j_c)::value;
            b[kk][j] = ds_read_b128_off<j * 16 * ROWB>(bb);
        });
        static_for<0, TM>([&](auto i_c) {
            constexpr int i = decltype(i_c)::value;
            a[kk][i] = ds_read_b128_off<i * 16 * ROWB>(ab);
        });
    };
    auto read_dw = [&](int kt) {
        const uint32_t dwb = lds0 + 2 * STAGE + (kt % 3) * A8S_SC + A8S_DW + (wn0 + c) * 8;
        static_for<0, TN>([&](auto j_c) {
            constexpr int j = decltype(j_c)::value;
            dw[j] = ds_read_b64_off<j * 128>(dwb);
        });
    };
    auto read_da = [&](int kt, auto kk_c) {
        constexpr int kk = decltype(kk_c)::value;
        const uint32_t dab = lds0 + 2 * STAGE + (kt % 3) * A8S_SC + A8S_DA + (kk * A8_BM + wm0 + 4 * g) * 4;
        da[kk][0] = ds_read_b128_off<0 * 64>(dab);
        da[kk][1] = ds_read_b128_off<1 * 64>(dab);
        da[kk][2] = ds_read_b128_off<2 * 64>(dab);
        da[kk][3] = ds_read_b128_off<3 * 64>(dab);
    };
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    // One block (kk): row group i's four MFMAs are issued in step i and scaled into acc in step i + 1, under the next
    // group's MFMAs.  Empty asm statements pin the order (hipcc otherwise hoists all sixteen MFMAs of both blocks and
    // sinks the scaling behind them, holding 32 results at once: spills): step i's MFMAs read a[i] after an asm that
    // "writes" it, and the FMAs of step i produce acc rows that an asm "reads" in the same step.
    auto block = [&](auto kk_c) {
        constexpr int kk = decltype(kk_c)::value;
        f32x4 tp[TN], tc[TN];
        static_for<0, TM + 1>([&](auto i_c) {
            constexpr int i = decltype(i_c)::value;
            if constexpr (i < TM) {
                u32x4 ai = __builtin_bit_cast(u32x4, a[kk][i]);
                asm volatile("" : "+v"(ai));
                a[kk][i] = __builtin_bit_cast(uint4, ai);
#pragma unroll
                for (int j = 0; j < TN; ++j) tc[j] = mfma16<false>(a[kk][i], b[kk][j], zero);
            }
            if constexpr (i > 0) {
                const uint4 dv = da[kk][i - 1];
                const float d4[4] = {__uint_as_float(dv.x), __uint_as_float(dv.y), __uint_as_float(dv.z),
                                     __uint_as_float(dv.w)};
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const float dwj = __uint_as_float(kk == 0 ? dw[j].x : dw[j].y);
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[i - 1][j][r] = __builtin_fmaf(tp[j][r], rn_mul(dwj, d4[r]), acc[i - 1][j][r]);
                    asm volatile("" : "+v"(acc[i - 1][j]));
                }
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) tp[j] = tc[j];
        });
    };
    auto wait_retire = [&](int younger) {
        if (younger >= 1)
            wait_vmcnt<G>();
        else
            wait_vmcnt<0>();
    };

    // Double buffer, one k-tile ahead: tile kt + 2 is staged into buffer kt & 1 once every wave has finished reading it
    // (the barrier that ends iteration kt), so each tile has the whole next iteration to land; the fragments of each
    // block are read right before its MFMAs (one block's operands live at a time).
    using K0 = std::integral_constant<int, 0>;
    using K1 = std::integral_constant<int, 1>;
    stage(0, 0);
    if (nk > 1) stage(1, 1);
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        wait_retire(kt + 1 < nk ? 1 : 0);  // tile kt landed (tile kt + 1 may stay in flight)
        __builtin_amdgcn_s_barrier();       // ... for every wave's pieces
        read_frags(cur, K0{});
        read_dw(kt);
        read_da(kt, K0{});
        lds_wait_all();
        read_frags(cur, K1{});  // in flight under block 0
        read_da(kt, K1{});
        block(K0{});
        mfma_war_retire(a[0], b[0]);
        lds_wait_all();
        block(K1{});
        mfma_war_retire(a[1], b[1]);
        __builtin_amdgcn_s_barrier();  // every wave is done with buffer `cur` and scale slot kt % 3
        if (kt + 2 < nk) stage(cur, kt + 2);
    }
    a8_epilogue<EPI, A8S_SMEM, TN>(p.g, acc, m0, n0, wm0, wn0, tid, smem);
}

template <int EPI>
void launch_a8s_epi(const A8SParams& p, hipStream_t s) {
    const int nbm = (p.g.M + A8_BM - 1) / A8_BM;
    // a 128-wide tile grid under half a round of two workgroups per CU takes the 64-wide tile (twice the tiles, each
    // half the work); the prep epilogue needs whole 128-column heads.  Measured (tools/qact_bench.py, 240 s): the
    // N = 2048 projections (384 tiles of 128 for 512 slots) are slower on 64-wide tiles (o 80 -> 86 us, down 214 ->
    // 227), the small grids faster (proj_out 64 -> 48, condition 50 -> 38): hence half a round, not one.
    static int n_cu = 0;
    if (n_cu == 0) {
        int dev = 0;
        ACEMI_HIP(hipGetDevice(&dev));
        ACEMI_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    }
    if constexpr (EPI != EPI_QKV_PREP) {
        if ((int64_t)nbm * (p.g.N / 128) < n_cu && p.g.N % 64 == 0) {
            hipLaunchKernelGGL((gemm_a8s_kernel<EPI, 64>), dim3(nbm * (p.g.N / 64)), dim3(256), 0, s, p);
            return;
        }
    }
    hipLaunchKernelGGL((gemm_a8s_kernel<EPI, 128>), dim3(nbm * (p.g.N / 128)), dim3(256), 0, s, p);
}

// int8 plane -> its bf16 image (exact integers), 16 values per thread
__global__ void __launch_bounds__(256) q8_image_kernel(const int8_t* __restrict__ q, int64_t n16, uint16_t* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= n16) return;
    const uint4 v = *(const uint4*)(q + t * 16);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int x0 = (int)(int8_t)(w[i] & 0xff), x1 = (int)(int8_t)((w[i] >> 8) & 0xff);
        const int x2 = (int)(int8_t)((w[i] >> 16) & 0xff), x3 = (int)(int8_t)(w[i] >> 24);
        o[2 * i] = (__float_as_uint((float)x0) >> 16) | (__float_as_uint((float)x1) & 0xffff0000u);
        o[2 * i + 1] = (__float_as_uint((float)x2) >> 16) | (__float_as_uint((float)x3) & 0xffff0000u);
    }
    *(uint4*)(out + t * 16) = make_uint4(o[0], o[1], o[2], o[3]);
    *(uint4*)(out + t * 16 + 8) = make_uint4(o[4], o[5], o[6], o[7]);
}

template <int WQ>
void launch_wq(const A8Params& p, dim3 grid, hipStream_t s) {
    switch (p.g.e.kind) {
        case EPI_STORE_F32: hipLaunchKernelGGL((gemm_a8_kernel<WQ, EPI_STORE_F32>), grid, dim3(256), 0, s, p); break;
        case EPI_STORE_ACT: hipLaunchKernelGGL((gemm_a8_kernel<WQ, EPI_STORE_ACT>), grid, dim3(256), 0, s, p); break;
        case EPI_RESID_GATED: hipLaunchKernelGGL((gemm_a8_kernel<WQ, EPI_RESID_GATED>), grid, dim3(256), 0, s, p); break;
        case EPI_RESID: hipLaunchKernelGGL((gemm_a8_kernel<WQ, EPI_RESID>), grid, dim3(256), 0, s, p); break;
        case EPI_SWIGLU: hipLaunchKernelGGL((gemm_a8_kernel<WQ, EPI_SWIGLU>), grid, dim3(256), 0, s, p); break;
        case EPI_PROJ_OUT: hipLaunchKernelGGL((gemm_a8_kernel<WQ, EPI_PROJ_OUT>), grid, dim3(256), 0, s, p); break;
        case EPI_QKV_PREP: hipLaunchKernelGGL((gemm_a8_kernel<WQ, EPI_QKV_PREP>), grid, dim3(256), 0, s, p); break;
        case EPI_SWIGLU_F32: hipLaunchKernelGGL((gemm_a8_kernel<WQ, EPI_SWIGLU_F32>), grid, dim3(256), 0, s, p); break;
        default: throw std::runtime_error("gemm_a8: unknown epilogue");
    }
}

dim3 grid_1d(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

}  // namespace

void launch_quantize_act(int kind, const float* x, int64_t ldx, int M, int K, bool silu_in, int8_t* q, float* s,
                         float* bsum, int64_t ld_s, hipStream_t st, uint16_t* q16) {
    ACEMI_CHECK(M >= 1 && ld_s >= M && ldx >= K && ldx % 4 == 0, "quantize_act: bad shape");
    if (kind == QACT_Q8_0) {
        ACEMI_CHECK(K % 32 == 0 && (q || q16), "quantize_act: Q8_0 needs K % 32 == 0 and an output");
        hipLaunchKernelGGL(quantize_q8_0_kernel, grid_1d((int64_t)M * (K / 32)), dim3(256), 0, st, x, ldx, M, K, silu_in,
                           q, q16, s, ld_s);
    } else {
        ACEMI_CHECK(q != nullptr && q16 == nullptr, "quantize_act: Q8_K has the int8 form only");
        ACEMI_CHECK(K % 256 == 0 && bsum != nullptr, "quantize_act: Q8_K needs K % 256 == 0 and a block-sum plane");
        hipLaunchKernelGGL(quantize_q8_k_kernel, grid_1d((int64_t)M * (K / 256) * 8), dim3(256), 0, st, x, ldx, M, K,
                           silu_in, q, s, bsum, ld_s);
    }
    ACEMI_HIP(hipGetLastError());
}

static int g_a8_mode = -1;
void gemm_a8_mode(int mode) { g_a8_mode = mode; }
bool gemm_a8_bf16_path(int fmt, int K) {
    static const int env = [] {
        const char* e = std::getenv("ACE_MI_QACT_GEMM");
        return (e && e[0] == '0') ? 0 : 1;
    }();
    const int mode = g_a8_mode >= 0 ? g_a8_mode : env;
    return mode == 1 && fmt == WF_Q8_0 && K % 64 == 0;
}

void launch_q8_image(const int8_t* q, int64_t n, uint16_t* out, hipStream_t s) {
    ACEMI_CHECK(n % 16 == 0, "q8_image: n % 16 == 0");
    hipLaunchKernelGGL(q8_image_kernel, grid_1d(n / 16), dim3(256), 0, s, q, n / 16, out);
    ACEMI_HIP(hipGetLastError());
}

void launch_gemm_a8(const QAct& a, const WeightView& W, int M, int N, int K, const GemmEpilogue& epi, hipStream_t s,
                    const uint16_t* w16) {
    ACEMI_CHECK(weight_quantized(W.fmt) && W.q && W.s, "gemm_a8: the weight must be in a ggml block format");
    if (a.q16 && w16) {  // Q8_0 on the bf16 MFMA (gemm_a8s_kernel)
        ACEMI_CHECK(W.fmt == WF_Q8_0 && a.kind == QACT_Q8_0 && K % 64 == 0 && K >= 64 && M >= 1 && N % A8_BN == 0,
                    "gemm_a8: the bf16-MFMA form is Q8_0 with K % 64 == 0, N % 128 == 0");
        ACEMI_CHECK(a.s && a.ld_s >= (int64_t)(M + A8_BM - 1) / A8_BM * A8_BM, "gemm_a8: activation scale plane too small");
        A8SParams p{};
        p.g.M = M;
        p.g.N = N;
        p.g.K = K;
        p.g.e = epi;
        p.a = a.q16;
        p.w = w16;
        p.as = a.s;
        p.ld_s = a.ld_s;
        p.ws = W.s;
        switch (epi.kind) {
            case EPI_STORE_F32: launch_a8s_epi<EPI_STORE_F32>(p, s); break;
            case EPI_STORE_ACT: launch_a8s_epi<EPI_STORE_ACT>(p, s); break;
            case EPI_RESID_GATED: launch_a8s_epi<EPI_RESID_GATED>(p, s); break;
            case EPI_RESID: launch_a8s_epi<EPI_RESID>(p, s); break;
            case EPI_SWIGLU: launch_a8s_epi<EPI_SWIGLU>(p, s); break;
            case EPI_PROJ_OUT: launch_a8s_epi<EPI_PROJ_OUT>(p, s); break;
            case EPI_QKV_PREP: launch_a8s_epi<EPI_QKV_PREP>(p, s); break;
            case EPI_SWIGLU_F32: launch_a8s_epi<EPI_SWIGLU_F32>(p, s); break;
            default: throw std::runtime_error("gemm_a8: unknown epilogue");
        }
        ACEMI_HIP(hipGetLastError());
        return;
    }
    ACEMI_CHECK(a.q != nullptr, "gemm_a8: the i8 kernel needs the int8 activation blocks");
    ACEMI_CHECK(a.kind == qact_kind_for(W.fmt), "gemm_a8: activation blocks do not match the weight's vec_dot_type");
    ACEMI_CHECK(M >= 1 && N % A8_BN == 0 && K % (W.fmt == WF_Q8_0 ? 32 : 256) == 0, "gemm_a8: bad shape");
    ACEMI_CHECK(a.q && a.s && a.ld_s >= (int64_t)(M + A8_BM - 1) / A8_BM * A8_BM && a.ld_s % 4 == 0,
                "gemm_a8: activation scale plane too small");
    ACEMI_CHECK(W.fmt != WF_Q4_K || a.bsum, "gemm_a8: Q4_K needs the activation block sums");
    ACEMI_CHECK(epi.kind != EPI_QKV_PREP || N % 128 == 0, "gemm_a8: prep epilogue on 128-column heads");
    A8Params p{};
    p.g.M = M;
    p.g.N = N;
    p.g.K = K;
    p.g.e = epi;
    p.aq = a.q;
    p.as = a.s;
    p.ab = a.bsum;
    p.ld_s = a.ld_s;
    p.wq = W.q;
    p.ws = W.s;
    const dim3 grid((unsigned)(((M + A8_BM - 1) / A8_BM) * (N / A8_BN)));
    switch (W.fmt) {
        case WF_Q8_0: launch_wq<WF_Q8_0>(p, grid, s); break;
        case WF_Q4_K: launch_wq<WF_Q4_K>(p, grid, s); break;
        default: launch_wq<WF_Q6_K>(p, grid, s); break;
    }
    ACEMI_HIP(hipGetLastError());
}

void launch_rmsnorm_mod_f32(const float* x, int M, int H, const float* w, const float* scale, const float* shift,
                            int64_t mod_stride, int rows_per_item, float eps, float* out, hipStream_t s) {
    ACEMI_CHECK(H % 4 == 0 && H <= 4096 && M >= 1, "rmsnorm_mod_f32: H % 4 == 0 and H <= 4096");
#define ACEMI_RMSF(V)                                                                                               \
    hipLaunchKernelGGL(rmsnorm_mod_f32_kernel<V>, dim3(M), dim3(256), 0, s, x, H, w, scale, shift, mod_stride, \
                       rows_per_item, eps, out)
    if (H <= 1024)
        ACEMI_RMSF(1);
    else if (H <= 2048)
        ACEMI_RMSF(2);
    else
        ACEMI_RMSF(4);
#undef ACEMI_RMSF
    ACEMI_HIP(hipGetLastError());
}

void launch_pack_input_f32(const float* hidden, const float* context, int B, int T, int Np, int P, int audio_dim,
                           int ctx_dim, float* out, hipStream_t s) {
    const int64_t n = (int64_t)B * Np * P * (audio_dim + ctx_dim);
    hipLaunchKernelGGL(pack_input_f32_kernel, dim3((unsigned)std::min<int64_t>((n + 255) / 256, 16384)), dim3(256), 0,
                       s, hidden, context, B, T, Np, P, audio_dim, ctx_dim, out);
    ACEMI_HIP(hipGetLastError());
}

}  // namespace acemi
