// Flash-style attention for the DiT self/cross attention (gfx950 / CDNA4).
//
// Replaces the materialised ggml graph of attention()
// (acestep_dit_model.cpp:1212-1256): kq = K.Q (F32), *1/sqrt(D), + mask,
// soft_max, V.attn, with GQA head h -> kv head h / n_rep
// (repeat_kv_interleave :1118-1130) and the additive mask of
// build_attention_mask (:1132-1173: key padding, bidirectional sliding window
// |q-k| <= w), plus the causal mask of the Qwen3 text encoder
// (qwen_model.cpp:618-637).  Scores never touch HBM; the sliding layers visit
// only the key tiles inside the window, causal blocks stop at their last query.
//
// Numerics: the reference runs attention in F32.  SPLIT=true (default) keeps
// every operand as an fp16 pair x = hi + lo (hi = fp16(x), lo = fp16(x - hi))
// and forms each product as hi*hi + hi*lo + lo*hi with three
// v_mfma_f32_32x32x16_f16 (f32 accumulate) -> ~22-bit operands, so the bf16
// rounding of the attention output (the o_proj vec_dot conversion) flips
// almost never relative to the F32 reference.  SPLIT=false is the plain fp16
// fast path (ACE_MI_ATTN_FAST=1).  P is formed as exp2(s - m + 12) (scaled by
// 2^12 so its lo part stays a normal fp16; O and l carry the same factor).
// Online softmax in f32 (exp2 domain).  A row whose keys are all masked
// yields 0/0 = NaN exactly like ggml's soft_max of an all -inf row.
//
// Structure: one workgroup = 4 waves = (batch item, kv head, 128 query rows
// spread over the n_rep q heads sharing that kv head), so each K/V tile is
// staged once for all heads of the group.  Each wave owns 32 query rows and
// computes S^T = K.Q^T (swapped), so a lane holds one query's scores in
// registers: row max / sum are in-register + one cross-half shuffle.  The
// S^T accumulator registers are, after f16 packing, directly the B operand of
// O^T = V^T . P^T (the k order inside a 16-key step is permuted; V^T is stored
// with the matching permutation by the prep kernel), so P never goes through
// LDS and the per-row rescale factor is lane-local.  K/V^T tiles arrive by
// global_load_lds into a double-buffered, XOR-swizzled LDS image.
#include "../kernels.h"
#include "lds_asm.h"

namespace acemi {
namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int D = 128;
constexpr int KT = 64;                    // keys per tile
constexpr int K_BYTES = KT * D * 2;       // 16 KiB
constexpr int V_BYTES = D * KT * 2;       // 16 KiB
constexpr float PSCALE_LOG2 = 12.0f;

template <bool SPLIT>
struct Stage {
    static constexpr int K_HI = 0;
    static constexpr int K_LO = K_BYTES;
    static constexpr int V_HI = SPLIT ? 2 * K_BYTES : K_BYTES;
    static constexpr int V_LO = V_HI + V_BYTES;
    static constexpr int KB = SPLIT ? 2 * (K_BYTES + V_BYTES) : K_BYTES + V_BYTES;
    static constexpr int BYTES = KB + KT * 4;
};

__device__ __forceinline__ f32x16 mfma32(const uint4& a, const uint4& b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0,
                                                  0, 0);
}

__device__ __forceinline__ uint32_t pack_f16x2(float a, float b) {
    _Float16 ha = (_Float16)a, hb = (_Float16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, ha) | ((uint32_t)__builtin_bit_cast(uint16_t, hb) << 16);
}

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 64u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

template <bool F16OUT>
__device__ __forceinline__ uint16_t to_act(float f) {
    if constexpr (F16OUT) {
        _Float16 h = (_Float16)f;
        return __builtin_bit_cast(uint16_t, h);
    } else {
        return f32_to_bf16_rne(f);
    }
}

__device__ __forceinline__ uint32_t pack_f16x2_lo(float a, float b) {
    const _Float16 ha = (_Float16)a, hb = (_Float16)b;
    return pack_f16x2(a - (float)ha, b - (float)hb);
}

template <bool F16OUT, bool SPLIT>
__global__ void __launch_bounds__(256) attn_kernel(AttnArgs a) {
    using ST = Stage<SPLIT>;
    constexpr int STAGE = ST::BYTES;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int h = lane >> 5;     // lane half
    const int lq = lane & 31;

    const int rep = a.Hq / a.Hkv;
    const int qpb = 128 / rep;   // query rows per head in this block
    const int n_qt = (a.nq + qpb - 1) / qpb;
    int bid = blockIdx.x;
    const int qt = bid % n_qt;
    bid /= n_qt;
    const int kvh = bid % a.Hkv;
    const int b = bid / a.Hkv;
    const int waves_per_head = 4 / rep;
    const int head = kvh * rep + wid / waves_per_head;
    const int q0 = qt * qpb;
    const int qw0 = q0 + (wid % waves_per_head) * 32;  // this wave's first row
    const int qrow = qw0 + lq;

    // ---- key tile range
    int klo = 0, khi = a.nk;
    if (a.window > 0) {
        klo = max(0, q0 - a.window);
        khi = min(a.nk, q0 + qpb - 1 + a.window + 1);
    }
    if (a.causal) khi = min(khi, q0 + qpb);  // no key after the block's last query
    const int kt_begin = klo / KT;
    const int kt_end = (khi + KT - 1) / KT;

    // ---- Q fragments (B operand of S^T = K Q^T): Q[q][16ks + 8h + j]
    const uint16_t* qptr = a.q + (((int64_t)b * a.Hq + head) * a.nq_pad + qrow) * D + 8 * h;
    uint4 qf[8], qfl[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *(const uint4*)(qptr + 16 * ks);
    if constexpr (SPLIT) {
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) qfl[ks] = *(const uint4*)(qptr + a.q_plane + 16 * ks);
    }

    const uint16_t* kbase = a.k + ((int64_t)b * a.Hkv + kvh) * a.nk_pad * D;
    const uint16_t* vbase = a.vt + ((int64_t)b * a.Hkv + kvh) * D * a.nk_pad;
    const float* kb = a.kbias ? a.kbias + (int64_t)b * a.nk_pad : nullptr;

    auto stage = [&](int buf, int kt) {
        char* base = smem + buf * STAGE;
        const int k0 = kt * KT;
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // K: 16 instr of 4 rows
            const int g = wid + 4 * j;
            const int row = 4 * g + (lane >> 4);
            const int ch = (lane & 15) ^ (row & 15);
            const uint16_t* src = kbase + (int64_t)(k0 + row) * D + ch * 8;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + ST::K_HI + g * 1024), 16, 0, 0);
            if constexpr (SPLIT)
                __builtin_amdgcn_global_load_lds((const void*)(src + a.k_plane), (lds_void*)(base + ST::K_LO + g * 1024),
                                                 16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // V^T: 16 instr of 8 d-rows
            const int g = wid + 4 * j;
            const int d = 8 * g + (lane >> 3);
            const int ch = (lane & 7) ^ ((d >> 1) & 7);
            const uint16_t* src = vbase + (int64_t)d * a.nk_pad + k0 + ch * 8;
            __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + ST::V_HI + g * 1024), 16, 0, 0);
            if constexpr (SPLIT)
                __builtin_amdgcn_global_load_lds((const void*)(src + a.v_plane), (lds_void*)(base + ST::V_LO + g * 1024),
                                                 16, 0, 0);
        }
        if (kb && wid == 0) {
            __builtin_amdgcn_global_load_lds((const void*)(kb + k0 + lane), (lds_void*)(base + ST::KB), 4, 0, 0);
        }
    };

    const float c_log2 = a.scale * 1.4426950408889634f;
    float m_run = -INFINITY;
    float l_run = 0.f;
    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;

    if (kt_begin < kt_end) {
        stage(0, kt_begin);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // Per-lane LDS read addressing.  K rows are 256 B with 16-B chunk c stored at c ^ (key & 15); the
    // fragment chunk of k-step ks is 2*ks + h, so its physical chunk is (2*ks) ^ cK (cK lane constant).
    // V^T rows are 128 B with chunk c at c ^ ((d >> 1) & 7): chunk of key-step g is (2*g) ^ cV.
    const int cK = h ^ (lq & 15);
    const int cV = h ^ ((lq >> 1) & 7);
    const uint32_t smem_l = lds_addr(smem);

    for (int kt = kt_begin; kt < kt_end; ++kt) {
        const int cur = (kt - kt_begin) & 1;
        if (kt + 1 < kt_end) stage(cur ^ 1, kt + 1);
        const uint32_t st = smem_l + cur * STAGE;
        const int k0 = kt * KT;

        // ---- S^T = K . Q^T (two 32-key tiles); SPLIT: Kh.Qh + Kh.Ql + Kl.Qh
        f32x16 s[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int r = 0; r < 16; ++r) s[t][r] = 0.f;
            const uint32_t rowk = st + ST::K_HI + (32 * t + lq) * 256;
            uint4 kf[8], kfl[8];
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) kf[ks] = ds_read_b128_v(rowk + (((2 * ks) ^ cK) << 4));
            if constexpr (SPLIT) {
#pragma unroll
                for (int ks = 0; ks < 8; ++ks)
                    kfl[ks] = ds_read_b128_v(rowk + (ST::K_LO - ST::K_HI) + (((2 * ks) ^ cK) << 4));
            }
            lds_wait_all();
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                s[t] = mfma32(kf[ks], qf[ks], s[t]);
                if constexpr (SPLIT) {
                    s[t] = mfma32(kf[ks], qfl[ks], s[t]);
                    s[t] = mfma32(kfl[ks], qf[ks], s[t]);
                }
            }
        }

        // ---- scale, mask, online softmax (this lane: query qrow, 32 of the 64 keys)
        float kbv[2][16];
        if (kb) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int g4 = 0; g4 < 4; ++g4) {
                    const uint4 v = ds_read_b128_v(st + ST::KB + (32 * t + 8 * g4 + 4 * h) * 4);
                    kbv[t][4 * g4 + 0] = __uint_as_float(v.x);
                    kbv[t][4 * g4 + 1] = __uint_as_float(v.y);
                    kbv[t][4 * g4 + 2] = __uint_as_float(v.z);
                    kbv[t][4 * g4 + 3] = __uint_as_float(v.w);
                }
            lds_wait_all();
        }
        const bool need_window = a.window > 0 && (k0 < qw0 + 31 - a.window || k0 + KT - 1 > qw0 + a.window);
        const bool need_causal = a.causal && k0 + KT - 1 > qw0;
        float mloc = -INFINITY;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int krel = 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
                float x = s[t][r] * c_log2;
                if (kb) x += kbv[t][r];
                if (need_window) {
                    const int d = qrow - (k0 + krel);
                    if (d > a.window || d < -a.window) x = -INFINITY;
                }
                if (need_causal && k0 + krel > qrow) x = -INFINITY;
                s[t][r] = x;
                mloc = fmaxf(mloc, x);
            }
        }
        mloc = fmaxf(mloc, __shfl_xor(mloc, 32));
        const float m_new = fmaxf(m_run, mloc);
        const float m_use = ((m_new == -INFINITY) ? 0.f : m_new) - PSCALE_LOG2;
        const float alpha = __builtin_amdgcn_exp2f(m_run - PSCALE_LOG2 - m_use);
        // alpha is exp2(0) = 1 for every row whose running max did not move; once the maxima settle
        // (after the first few key tiles) whole waves skip the O rescale below
        const bool rescale = __ballot(m_new != m_run) != 0;
        m_run = m_new;
        float lsum = 0.f;
        uint4 pf[4], pfl[4];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float pr = __builtin_amdgcn_exp2f(s[t][r] - m_use);
                s[t][r] = pr;
                lsum += pr;
            }
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                uint4 f;
                f.x = pack_f16x2(s[t][8 * ss + 0], s[t][8 * ss + 1]);
                f.y = pack_f16x2(s[t][8 * ss + 2], s[t][8 * ss + 3]);
                f.z = pack_f16x2(s[t][8 * ss + 4], s[t][8 * ss + 5]);
                f.w = pack_f16x2(s[t][8 * ss + 6], s[t][8 * ss + 7]);
                pf[2 * t + ss] = f;
                if constexpr (SPLIT) {
                    uint4 fl;
                    fl.x = pack_f16x2_lo(s[t][8 * ss + 0], s[t][8 * ss + 1]);
                    fl.y = pack_f16x2_lo(s[t][8 * ss + 2], s[t][8 * ss + 3]);
                    fl.z = pack_f16x2_lo(s[t][8 * ss + 4], s[t][8 * ss + 5]);
                    fl.w = pack_f16x2_lo(s[t][8 * ss + 6], s[t][8 * ss + 7]);
                    pfl[2 * t + ss] = fl;
                }
            }
        }
        l_run = (rescale ? l_run * alpha : l_run) + lsum;  // O and l always scaled together
        if (rescale) {
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        }

        // ---- O^T += V^T . P^T ; SPLIT: Vh.Ph + Vh.Pl + Vl.Ph
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
            const uint32_t rowv = st + ST::V_HI + (32 * dt + lq) * 128;
            uint4 vf[4], vfl[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) vf[g] = ds_read_b128_v(rowv + (((2 * g) ^ cV) << 4));
            if constexpr (SPLIT) {
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    vfl[g] = ds_read_b128_v(rowv + (ST::V_LO - ST::V_HI) + (((2 * g) ^ cV) << 4));
            }
            lds_wait_all();
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                o[dt] = mfma32(vf[g], pf[g], o[dt]);
                if constexpr (SPLIT) {
                    o[dt] = mfma32(vf[g], pfl[g], o[dt]);
                    o[dt] = mfma32(vfl[g], pf[g], o[dt]);
                }
            }
        }
        if (kt + 1 < kt_end) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt+1 landed (issued a whole tile ago)
            __builtin_amdgcn_s_barrier();                     // ... for every wave; buffer `cur` released
        }
    }

    // ---- normalise and store O[q][head*128 + d]
    const float l = l_run + __shfl_xor(l_run, 32);
    const float inv = 1.0f / l;
    if (qrow < a.nq) {
        uint16_t* op = a.out + ((int64_t)b * a.nq + qrow) * (a.Hq * D) + head * D;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int d = 32 * dt + 8 * g4 + 4 * h;
                uint2 w;
                w.x = (uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 0] * inv) |
                      ((uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 1] * inv) << 16);
                w.y = (uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 2] * inv) |
                      ((uint32_t)to_act<F16OUT>(o[dt][4 * g4 + 3] * inv) << 16);
                *(uint2*)(op + d) = w;
            }
        }
    }
}

}  // namespace

void launch_attention(ActType out_t, const AttnArgs& a, hipStream_t s) {
    ACEMI_CHECK(a.Hkv > 0 && a.Hq % a.Hkv == 0, "attention: Hq must be a multiple of Hkv");
    const int rep = a.Hq / a.Hkv;
    ACEMI_CHECK(rep == 1 || rep == 2 || rep == 4, "attention: n_rep must be 1, 2 or 4");
    ACEMI_CHECK(a.nk_pad % KT == 0 && a.nk_pad >= a.nk, "attention: nk_pad");
    const int qpb = 128 / rep;
    const int n_qt = (a.nq + qpb - 1) / qpb;
    ACEMI_CHECK(a.nq_pad >= n_qt * qpb, "attention: nq_pad too small");
    const dim3 grid(a.B * a.Hkv * n_qt);
    if (a.split) {
        ACEMI_CHECK(a.q_plane > 0 && a.k_plane > 0 && a.v_plane > 0, "attention: split mode needs lo planes");
        const size_t lds = 2 * Stage<true>::BYTES;
        if (out_t == ActType::F16)
            hipLaunchKernelGGL((attn_kernel<true, true>), grid, dim3(256), lds, s, a);
        else
            hipLaunchKernelGGL((attn_kernel<false, true>), grid, dim3(256), lds, s, a);
    } else {
        const size_t lds = 2 * Stage<false>::BYTES;
        if (out_t == ActType::F16)
            hipLaunchKernelGGL((attn_kernel<true, false>), grid, dim3(256), lds, s, a);
        else
            hipLaunchKernelGGL((attn_kernel<false, false>), grid, dim3(256), lds, s, a);
    }
    ACEMI_HIP(hipGetLastError());
}

}  // namespace acemi
