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
                                                            bool silu_in, int8_t* __restrict__ q, float* __restrict__ s,
                                                            int64_t ld_s) {
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
    int8_t* qr = q + (int64_t)m * K + b * 32;
    *(uint4*)qr = make_uint4(w[0], w[1], w[2], w[3]);
    *(uint4*)(qr + 16) = make_uint4(w[4], w[5], w[6], w[7]);
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

    const GemmEpilogue& e = p.g.e;
    if constexpr (EPI == EPI_QKV_PREP) {
        qkv_prep_tile<A8_BM, 4, 4, 4, A8_PREP_SMEM>(p.g, acc, m0, n0, wm0, wn0, tid, smem);
    } else if constexpr (EPI == EPI_SWIGLU_F32) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm0 + i * 16 + 4 * g + r;
                if (m >= M) continue;
#pragma unroll
                for (int j = 0; j < 4; j += 2) {
                    const int n = n0 + wn0 + j * 16;  // gate columns n .. n + 15, up columns n + 16 .. n + 31
                    e.c_f32[(int64_t)m * e.ldc + (n >> 1) + c] = rn_mul(silu_f(acc[i][j][r]), acc[i][j + 1][r]);
                }
            }
    } else {
        if constexpr (EPI == EPI_RESID || EPI == EPI_RESID_GATED) {
            if (e.bias) {  // x + (W x_a + b): the bias joins the product before the residual add
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float bj = e.bias[n0 + wn0 + j * 16 + c];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc[i][j][r] = rn_add(acc[i][j][r], bj);
                }
            }
        }
        gemm_epilogue<4, 4, false, EPI, 1024>(p.g, acc, m0 + wm0, n0 + wn0, lane);
    }
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
                         float* bsum, int64_t ld_s, hipStream_t st) {
    ACEMI_CHECK(M >= 1 && ld_s >= M && ldx >= K && ldx % 4 == 0, "quantize_act: bad shape");
    if (kind == QACT_Q8_0) {
        ACEMI_CHECK(K % 32 == 0, "quantize_act: Q8_0 needs K % 32 == 0");
        hipLaunchKernelGGL(quantize_q8_0_kernel, grid_1d((int64_t)M * (K / 32)), dim3(256), 0, st, x, ldx, M, K, silu_in,
                           q, s, ld_s);
    } else {
        ACEMI_CHECK(K % 256 == 0 && bsum != nullptr, "quantize_act: Q8_K needs K % 256 == 0 and a block-sum plane");
        hipLaunchKernelGGL(quantize_q8_k_kernel, grid_1d((int64_t)M * (K / 256) * 8), dim3(256), 0, st, x, ldx, M, K,
                           silu_in, q, s, bsum, ld_s);
    }
    ACEMI_HIP(hipGetLastError());
}

void launch_gemm_a8(const QAct& a, const WeightView& W, int M, int N, int K, const GemmEpilogue& epi, hipStream_t s) {
    ACEMI_CHECK(weight_quantized(W.fmt) && W.q && W.s, "gemm_a8: the weight must be in a ggml block format");
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
