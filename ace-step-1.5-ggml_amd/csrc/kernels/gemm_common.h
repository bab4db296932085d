// Shared device-side pieces of the DiT GEMM kernels (gemm.hip: dense bf16 / fp16 tiles; gemm_q.hip: the
// quantized-weight kernels and the staged dequant): operand types, the swizzled LDS image helpers, the
// XCD-aware tile order, the fused epilogues and the split-K join.  Header-only (inline device functions and
// templates), so each translation unit compiles its own instances in parallel.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "../kernels.h"
#include "prep_math.h"
#include "mfma_guard.h"

namespace acemi {
namespace gemm_detail {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

typedef __attribute__((address_space(3))) void lds_void;

struct GemmParams {
    const uint16_t* A;
    const uint16_t* W;   // dense weight
    const void* Wq;      // quantized weight planes (runtime/quant.h)
    const float* Ws;
    int lda, ldw, M, N, K;
    GemmEpilogue e;
    // split-K (gemm_kernel only): ksplit blocks per output tile, each over a contiguous 1/ksplit of the
    // K-tiles; the last adds the others' partial tiles (sk_ws, slot = K part) in K order and runs the
    // epilogue.  sk_cnt / sk_ready: per-tile ticket / ready counters, zero between launches (splitk_join).
    int ksplit;
    f32x4* sk_ws;
    unsigned* sk_cnt;
    unsigned* sk_ready;
    unsigned* sk_err;  // per-device host-pinned word, set to 1 when a join's bounded wait timed out (gemm_splitk_check)
};

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 64u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

template <bool F16>
__device__ __forceinline__ uint16_t to_act(float f) {
    if constexpr (F16) {
        _Float16 h = (_Float16)f;
        return __builtin_bit_cast(uint16_t, h);
    } else {
        return f32_to_bf16_rne(f);
    }
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

template <bool F16>
__device__ __forceinline__ f32x4 mfma16(const uint4& a, const uint4& b, f32x4 c) {
    if constexpr (F16) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                      0, 0, 0);
    } else {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                       __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
}

// chunk swizzle of a 128-byte LDS row
__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

// ds_read_b128 hidden from the compiler's waitcnt pass (it would otherwise drain every in-flight
// LDS-DMA with vmcnt(0) before the read, serialising the prefetch).  The caller waits with
// lds_wait_all() + sched_barrier before consuming the registers (guide §5.7 item 1, rule 18).
template <int OFF>
__device__ __forceinline__ uint4 ds_read_b128_off(uint32_t addr) {
    u32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void lds_wait_all() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

template <int I, int N, int STRIDE>
struct ReadRows {  // dst[i] = 16 bytes at base + i*STRIDE, i = I..N-1 (compile-time offsets)
    __device__ __forceinline__ static void run(uint32_t base, uint4 (&dst)[N][2], int kk) {
        if (kk == 0)
            dst[I][0] = ds_read_b128_off<I * STRIDE>(base);
        else
            dst[I][1] = ds_read_b128_off<I * STRIDE>(base);
        ReadRows<I + 1, N, STRIDE>::run(base, dst, kk);
    }
};
template <int N, int STRIDE>
struct ReadRows<N, N, STRIDE> {
    __device__ __forceinline__ static void run(uint32_t, uint4 (&)[N][2], int) {}
};

// f(std::integral_constant<int, I>) for I = B..E-1
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// s_waitcnt vmcnt(N) with N a compile-time constant (lgkmcnt/expcnt untouched)
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// block -> tile: XCD-aware bijective remap (blocks b, b+8 share an XCD), then M-grouped order
template <int BM, int BN>
__device__ __forceinline__ void block_tile(const GemmParams& p, int& m0, int& n0, int bid = -1, int nwg = 0) {
    const int nbm = (p.M + BM - 1) / BM;
    const int nbn = p.N / BN;
    if (bid < 0) {
        bid = blockIdx.x;
        nwg = gridDim.x;
    }
    {
        const int xcd = bid & 7;
        const int q = nwg >> 3, r = nwg & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    }
#ifndef ACEMI_GEMM_GM
#define ACEMI_GEMM_GM 8
#endif
    constexpr int GM = ACEMI_GEMM_GM;  // M blocks per group of the tile order
    const int group = bid / (GM * nbn);
    const int first_m = group * GM;
    const int gm = min(nbm - first_m, GM);
    const int bm = first_m + (bid % (GM * nbn)) % gm;
    const int bn = (bid % (GM * nbn)) / gm;
    m0 = bm * BM;
    n0 = bn * BN;
}

// Fused epilogue of one wave's TM x TN grid of 16x16 accumulators at (mw, nw).
// C/D map of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + r.
template <int TM, int TN, bool F16, int EPI, int PRE>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, f32x4 (&acc)[TM][TN], int mw, int nw, int lane) {
    const GemmEpilogue& e = p.e;
    const int M = p.M;
    const int ccol = lane & 15;
    const int crow = (lane >> 4) * 4;
    if constexpr (EPI == EPI_RESID_GATED || EPI == EPI_RESID) {
        // Residual read-modify-write: the old x (and gate) values of a chunk of GI 16-row groups are all
        // loaded before the chunk's first store.  Interleaved, the compiler cannot move a load of x above
        // an earlier store to x (same pointer), so each element paid a full memory round trip in
        // sequence.  A whole-tile preload (PRE = 1024 values) fits the 512-register budget of the 4-wave
        // tiles; the 8-wave tiles (256 registers, accumulators included) preload 64 values per chunk
        // instead of spilling, the 256-register split-K instances 32.
        constexpr int PER_I = 4 * TN * (EPI == EPI_RESID_GATED ? 2 : 1);
        constexpr int GI0 = PRE / PER_I;
        constexpr int GI = GI0 < 1 ? 1 : (GI0 > TM ? TM : GI0);
#pragma unroll
        for (int i0 = 0; i0 < TM; i0 += GI) {
            float xo[GI][4][TN], gt[GI][4][TN];
#pragma unroll
            for (int ii = 0; ii < GI; ++ii)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = mw + (i0 + ii) * 16 + crow + r;
                    const bool ok = i0 + ii < TM && m < M;
                    const int item = EPI == EPI_RESID_GATED ? m / e.rows_per_item : 0;
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const int n = nw + j * 16 + ccol;
                        xo[ii][r][j] = ok ? e.c_f32[(int64_t)m * e.ldc + n] : 0.f;
                        if constexpr (EPI == EPI_RESID_GATED)
                            gt[ii][r][j] = ok ? e.gate[(int64_t)item * e.gate_stride + n] : 0.f;
                    }
                }
#pragma unroll
            for (int ii = 0; ii < GI; ++ii) {
                if (i0 + ii >= TM) break;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = mw + (i0 + ii) * 16 + crow + r;
                    if (m >= M) continue;
#pragma unroll
                    for (int j = 0; j < TN; ++j) {
                        const int n = nw + j * 16 + ccol;
                        float v = acc[i0 + ii][j][r];
                        if constexpr (EPI == EPI_RESID_GATED) v = rn_mul(v, gt[ii][r][j]);
                        e.c_f32[(int64_t)m * e.ldc + n] = rn_add(xo[ii][r][j], v);
                    }
                }
            }
        }
        return;
    }
    float bias_j[TN];  // a thread's columns are fixed: their bias is loaded once, before any store
#pragma unroll
    for (int j = 0; j < TN; ++j)
        bias_j[j] = ((EPI == EPI_STORE_F32 || EPI == EPI_STORE_ACT) && e.bias) ? e.bias[nw + j * 16 + ccol] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = mw + i * 16 + crow + r;
            if (m >= M) continue;
            if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
                for (int j = 0; j < TN; j += 2) {
                    const int n = nw + j * 16;  // multiple of 32
                    const float g = acc[i][j][r];
                    const float u = acc[i][j + 1][r];
                    e.c_act[(int64_t)m * e.ldc + (n >> 1) + ccol] = to_act<F16>(silu_f(g) * u);
                }
            } else {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = nw + j * 16 + ccol;
                    float v = acc[i][j][r];
                    if constexpr (EPI == EPI_STORE_F32) {
                        if (e.bias) v = v + bias_j[j];
                        e.c_f32[(int64_t)m * e.ldc + n] = v;
                    } else if constexpr (EPI == EPI_STORE_ACT) {
                        if (e.bias) v = v + bias_j[j];
                        e.c_act[(int64_t)m * e.ldc + n] = to_act<F16>(v);
                    } else if constexpr (EPI == EPI_PROJ_OUT) {
                        const int item = m / e.rows_per_item;
                        const int pp = m - item * e.rows_per_item;
                        const int kpos = n / e.out_ch;
                        const int c = n - kpos * e.out_ch;
                        const int t = pp * e.patch + kpos;
                        if (t < e.out_T) {
                            e.c_f32[((int64_t)item * e.out_T + t) * e.out_ch + c] = rn_add(v, e.bias[c]);
                        }
                    }
                }
            }
        }
    }
}

// Residual epilogue in two halves (gemm_kernel's XPF path): resid_prefetch issues every load of the wave tile's old
// x values (TM x 4 x TN, rows past M read as 0) and, for the gated form, the gate rows of the first and last item
// the tile touches (2 x TN) -- exactly NX loads, issued early and consumed later by resid_apply, which adds and
// stores with the arithmetic of gemm_epilogue (x + acc (* gate), each product / sum rounded once).  A wave tile
// spanning more than two items (rows_per_item < wave rows) falls back to per-element gate loads in the apply.
template <int TM, int TN, int EPI>
__device__ __forceinline__ void resid_prefetch(const GemmParams& p, int mw, int nw, int lane, int wrows,
                                               float (&xo)[TM][4][TN], float (&g0)[TN], float (&g1)[TN]) {
    const GemmEpilogue& e = p.e;
    const int ccol = lane & 15, crow = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = min(mw + i * 16 + crow + r, p.M - 1);  // rows past M: a valid row, never stored
#pragma unroll
            for (int j = 0; j < TN; ++j) xo[i][r][j] = e.c_f32[(int64_t)m * e.ldc + nw + j * 16 + ccol];
        }
    if constexpr (EPI == EPI_RESID_GATED) {
        const int i0 = min(mw, p.M - 1) / e.rows_per_item, i1 = min(mw + wrows - 1, p.M - 1) / e.rows_per_item;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = nw + j * 16 + ccol;
            g0[j] = e.gate[(int64_t)i0 * e.gate_stride + n];
            g1[j] = e.gate[(int64_t)i1 * e.gate_stride + n];
        }
    }
}

template <int TM, int TN, int EPI>
__device__ __forceinline__ void resid_apply(const GemmParams& p, f32x4 (&acc)[TM][TN], int mw, int nw, int lane,
                                            int wrows, const float (&xo)[TM][4][TN], const float (&g0)[TN],
                                            const float (&g1)[TN]) {
    const GemmEpilogue& e = p.e;
    const int ccol = lane & 15, crow = (lane >> 4) * 4;
    const int i0 = min(mw, p.M - 1) / e.rows_per_item;
    // the wave tile touches at most two items: gate rows from the prefetch (two separate arrays, so the select
    // stays a v_cndmask -- a [2][TN] array indexed by the comparison went to scratch); otherwise (short items,
    // tests) per-element gate loads.  The branch is uniform and outside the store loops, so the fast path
    // issues its stores back to back (a load between stores makes hipcc wait for every store, vmcnt(0)).
    if (EPI != EPI_RESID_GATED || e.rows_per_item >= wrows) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = mw + i * 16 + crow + r;
                if (m >= p.M) continue;
                const bool first = m / e.rows_per_item == i0;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    float v = acc[i][j][r];
                    if constexpr (EPI == EPI_RESID_GATED) v = rn_mul(v, first ? g0[j] : g1[j]);
                    e.c_f32[(int64_t)m * e.ldc + nw + j * 16 + ccol] = rn_add(xo[i][r][j], v);
                }
            }
    } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = mw + i * 16 + crow + r;
                if (m >= p.M) continue;
                const int item = m / e.rows_per_item;
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = nw + j * 16 + ccol;
                    const float v = rn_mul(acc[i][j][r], e.gate[(int64_t)item * e.gate_stride + n]);
                    e.c_f32[(int64_t)m * e.ldc + n] = rn_add(xo[i][r][j], v);
                }
            }
    }
}

// EPI_QKV_PREP: the block's BM x 128 f32 accumulator tile (one head of the [q | k | v] projection) goes
// through LDS in row chunks (rows 144 floats apart: the 16x4 accumulator writes are conflict-free) and is
// written straight into the attention operand layouts with attn_prep's arithmetic (prep_math.h): 16
// lanes per token for q / k (QK-RMSNorm, RoPE, fp16 hi/lo), one lane per (d, 16-key group) for V^T.
// This removes the f32 [M][4096] round trip through HBM and the separate prep launch.
constexpr int PREP_LD = 144;  // LDS row stride (floats) of the accumulator tile in the fused prep

// `fill(tile, c0, CH)` writes the block's accumulators of tile rows [c0, c0 + CH) of head `hd` (128 columns)
// into the LDS tile (row stride PREP_LD)
template <int BM, int NW, int SMEM, class Fill>
__device__ __forceinline__ void qkv_prep_head(const GemmParams& p, int m0, int hd, int tid, char* smem, Fill fill) {
    constexpr int LD = PREP_LD;
    constexpr int CH = (BM * LD * 4 <= SMEM) ? BM : ((BM / 2) * LD * 4 <= SMEM ? BM / 2 : BM / 4);
    static_assert(CH * LD * 4 <= SMEM && BM % CH == 0 && CH % 16 == 0, "qkv prep chunking");
    constexpr int NT = NW * 64;
    const PrepArgs& a = p.e.prep;
    float* tile = reinterpret_cast<float*>(smem);
    const int nq = a.q_col >= 0 ? a.hq : 0;
    const int nk = a.k_col >= 0 ? a.hkv : 0;
    for (int c0 = 0; c0 < BM; c0 += CH) {
        const int mc0 = m0 + c0;
        if (mc0 >= p.M) break;
        __syncthreads();  // the main loop's (or the previous chunk's) LDS readers are done
        fill(tile, c0, CH);
        __syncthreads();
        const int rows = min(CH, p.M - mc0);
        if (hd < nq + nk) {
            const bool isq = hd < nq;
            const int head = isq ? hd : hd - nq;
            const float* w = isq ? a.q_norm : a.k_norm;
            uint16_t* base = isq ? a.qh + (int64_t)head * a.n_pad * 128 : a.kh + (int64_t)head * a.n_pad * 128;
            const int64_t bstride = (int64_t)(isq ? a.hq : a.hkv) * a.n_pad * 128;
            const int64_t plane = isq ? a.q_plane : a.k_plane;
            const int d = (tid & 15) * 4;
            for (int t = tid >> 4; t < rows; t += NT / 16) {
                const int m = mc0 + t;
                const int b = m / a.n_tok, n = m - b * a.n_tok;
                const float4 x0 = *(const float4*)(tile + t * LD + d), x1 = *(const float4*)(tile + t * LD + 64 + d);
                float y[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
                prep::head_row(y, w, d, a.eps, a.rope_cos ? a.rope_cos + (int64_t)n * 64 + d : nullptr,
                               a.rope_cos ? a.rope_sin + (int64_t)n * 64 + d : nullptr,
                               base + b * bstride + (int64_t)n * 128, plane, a.f8 ? (isq ? 1 : 2) : 0);
            }
        } else {
            // V^T: groups of 16 keys of one item; a group cut by the chunk edge is written key by key
            // (its other keys belong to the neighbouring chunk or tile), padding keys as zeros, and the
            // tile holding an item's last token also zero-fills the item's groups up to n_pad
            const int hk = hd - nq - nk;
            const int d = tid & 127;
            const int b_lo = mc0 / a.n_tok, b_hi = (mc0 + rows - 1) / a.n_tok;
            for (int b = b_lo; b <= b_hi; ++b) {
                const int n_lo = max(0, mc0 - b * a.n_tok), n_hi = min(a.n_tok, mc0 + rows - b * a.n_tok);
                uint16_t* vdst = a.vt + (((int64_t)b * a.hkv + hk) * 128 + d) * a.n_pad;
                const int g_end = n_hi == a.n_tok ? a.n_pad / 16 : ((n_hi - 1) >> 4) + 1;
                for (int g = (n_lo >> 4) + (tid >> 7); g < g_end; g += NT / 128) {
                    const int g0 = g * 16;
                    float v[16];
                    uint32_t have = 0;
#pragma unroll
                    for (int k = 0; k < 16; ++k) {
                        const int n = g0 + prep::vperm(k);
                        const bool mine = n >= n_lo && n < n_hi;
                        v[k] = mine ? tile[(b * a.n_tok + n - mc0) * LD + d] : 0.f;
                        have |= (mine || n >= a.n_tok) ? (1u << k) : 0u;
                    }
                    uint32_t wv[8], wl[8];
                    prep::v_words(v, wv, wl);
                    if (a.f8 && a.v_plane > 0) {  // natural key order for the fp8 plane (vperm is an involution)
                        float vn[16];
                        uint32_t hn = 0;
#pragma unroll
                        for (int w = 0; w < 16; ++w) {
                            vn[w] = v[prep::vperm(w)];
                            hn |= ((have >> prep::vperm(w)) & 1u) << w;
                        }
                        prep::v_store8(vn, vdst, a.v_plane, g0, hn);
                    }
                    if (have == 0xffffu) {
                        *(uint4*)(vdst + g0) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                        *(uint4*)(vdst + g0 + 8) = make_uint4(wv[4], wv[5], wv[6], wv[7]);
                        if (a.v_plane > 0 && !a.f8) {
                            *(uint4*)(vdst + a.v_plane + g0) = make_uint4(wl[0], wl[1], wl[2], wl[3]);
                            *(uint4*)(vdst + a.v_plane + g0 + 8) = make_uint4(wl[4], wl[5], wl[6], wl[7]);
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < 16; ++k) {
                            if (!((have >> k) & 1u)) continue;
                            vdst[g0 + k] = (uint16_t)(wv[k >> 1] >> (16 * (k & 1)));
                            if (a.v_plane > 0 && !a.f8) vdst[a.v_plane + g0 + k] = (uint16_t)(wl[k >> 1] >> (16 * (k & 1)));
                        }
                    }
                }
            }
        }
    }
}

// the 4-wave kernels' fused prep: the block's BM x 128 tile is one head, wave tile TM x TN at (wm0, wn0)
template <int BM, int NW, int TM, int TN, int SMEM>
__device__ __forceinline__ void qkv_prep_tile(const GemmParams& p, f32x4 (&acc)[TM][TN], int m0, int n0, int wm0,
                                              int wn0, int tid, char* smem) {
    const int lane = tid & 63;
    const int ccol = lane & 15, crow = (lane >> 4) * 4;
    qkv_prep_head<BM, NW, SMEM>(p, m0, n0 >> 7, tid, smem, [&](float* tile, int c0, int CH) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int rb = wm0 + i * 16 - c0;
            if (rb < 0 || rb >= CH) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int j = 0; j < TN; ++j) tile[(rb + crow + r) * PREP_LD + wn0 + j * 16 + ccol] = acc[i][j][r];
        }
    });
}

constexpr int CPOL_SC1 = 16;  // cache-policy bit of buffer / global ops: device-scope coherent (gfx94x/gfx950)

// largest split-K factor of a tile: the last block gathers the other parts through its LDS share
template <int BM, int BN>
struct SplitKMax {
    static constexpr int value = BM * BN >= 128 * 128 ? 2 : 4;
};

// Split-K: block -> (tile, K part).  When the tile count is a multiple of 8 the S parts of a tile are
// blocks 8 apart (same XCD: the partial tiles stay in that XCD's L2); otherwise adjacent blocks.
__device__ __forceinline__ void splitk_block(int S, int& tile, int& part, int& ntiles) {
    const int b = blockIdx.x;
    ntiles = gridDim.x / S;
    if ((ntiles & 7) == 0) {
        part = (b >> 3) % S;
        tile = (b / (8 * S)) * 8 + (b & 7);
    } else {
        part = b % S;
        tile = b / S;
    }
}

// The last block of a split-K tile adds the other parts' partial tiles: each wave brings its own fragments
// of the S-1 other slots into its share of the (now free) LDS by LDS-DMA (no VGPRs held by loads in flight),
// CH fragments at a time, then acc = ((part_0 + part_1) + ...) in K order, its own sum at index `part`.
template <int TM, int TN, int NW, int SS, int SMEM>
__device__ __forceinline__ void splitk_gather(f32x4 (&acc)[TM][TN], const f32x4* slot0, int64_t slot_stride,
                                              int part, char* smem, int wid, int lane) {
    constexpr int F = TM * TN;
    constexpr int LDSW = SMEM / NW;  // bytes of LDS per wave
    constexpr int CH0 = LDSW / ((SS - 1) * 1024);
    constexpr int CH = CH0 < F ? CH0 : F;
    static_assert(CH >= 1, "split-K gather: LDS share too small");
    char* wl = smem + wid * LDSW;
#pragma unroll
    for (int f0 = 0; f0 < F; f0 += CH) {
        if (f0 > 0) lds_wait_all();  // the previous chunk's LDS reads are done before it is overwritten
#pragma unroll
        for (int f = f0; f < f0 + CH && f < F; ++f)
#pragma unroll
            for (int qi = 0; qi < SS - 1; ++qi) {
                const int q = qi < part ? qi : qi + 1;
                __builtin_amdgcn_global_load_lds((const void*)(slot0 + q * slot_stride + f * 64),
                                                 (lds_void*)(wl + ((f - f0) * (SS - 1) + qi) * 1024), 16, 0,
                                                 CPOL_SC1);  // device-coherent load
            }
        wait_vmcnt<0>();
#pragma unroll
        for (int f = f0; f < f0 + CH && f < F; ++f) {
            if ((f - f0) % 4 == 0) __builtin_amdgcn_sched_barrier(0);  // LDS reads in groups of 4 fragments
            const f32x4* l = reinterpret_cast<const f32x4*>(wl + (f - f0) * (SS - 1) * 1024) + lane;
            const int i = f / TN, j = f % TN;
            if constexpr (SS == 2) {
                acc[i][j] += l[0];  // two parts: a + b == b + a, whichever is this block's
            } else {
                f32x4 t = part == 0 ? acc[i][j] : l[0];
#pragma unroll
                for (int q = 1; q < SS; ++q) t += q == part ? acc[i][j] : l[(q < part ? q : q - 1) * 64];
                acc[i][j] = t;
            }
        }
    }
}

// Join of the S blocks of one tile after their main loops.  Each block takes a ticket (atomic add on
// sk_cnt[tile]) when it starts (taken after the main loop, the returned value live across the loop made
// hipcc rotate the accumulators through AGPRs, > 256 VGPRs); the S-1 first write their accumulators to slot `part` of the tile's workspace (in the
// MFMA register layout: coalesced, device-coherent 16-byte stores), wait for their completion, and bump
// sk_ready[tile], then exit.  The last
// waits until the S-1 writes are visible and adds the slots into its accumulators in K order
// (deterministic: the same sum whichever block arrives last), then runs the epilogue.  Deadlock-free for
// any residency: a waiting block only waits for blocks that already took their ticket, i.e. are resident
// and finish without waiting on anything.  The last block resets the tile's two counters once the others
// are in, so every launch starts from zero whatever the split factor of the previous one.  Returns false
// for the blocks that exit.
template <int TM, int TN, int NW, int SKMAX, int SMEM>
__device__ __forceinline__ bool splitk_join(const GemmParams& p, f32x4 (&acc)[TM][TN], int S, int tile, int part,
                                           int tid, char* smem, unsigned ticket0) {
    __syncthreads();  // every wave is past its main loop's LDS reads: LDS is free
    if (tid == 0) *reinterpret_cast<unsigned*>(smem) = ticket0;  // (a separate __shared__ word would cost
    __syncthreads();                                               //  the 192x128 tile its second block per CU)
    const unsigned ticket = *reinterpret_cast<const unsigned*>(smem);
    __syncthreads();
    const bool last = ticket == (unsigned)(S - 1);
    const int wid = tid >> 6, lane = tid & 63;
    constexpr int PER_TILE = NW * TM * TN * 64;  // f32x4 per (tile, part) slot
    f32x4* slot0 = p.sk_ws + (int64_t)tile * S * PER_TILE + (wid * TM * TN) * 64 + lane;
    if (!last) {
        // device-coherent (sc1) stores of the partial tile, completed (vmcnt 0) before the ready count: no
        // device-scope fence, whose L2 write-back / invalidate (per block, or per spin) cost ~4x the GEMM
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(slot0 - lane + (int64_t)part * PER_TILE), 0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                                       ((i * TN + j) * 64 + lane) * 16, 0, CPOL_SC1);
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(p.sk_ready + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
    }
    if (tid == 0) {
        // bounded (~0.2 s; a real wait is a few microseconds): a protocol bug never hangs the GPU.  On a timeout
        // the error word is raised for the host (gemm_splitk_check: the library then fails loudly) and the
        // counters are left as they are -- the late parts still bump them, so resetting here would start the
        // next launch on this stream from nonzero counts
        bool done = false;
        for (int it = 0; it < (1 << 22) && !done; ++it) {
            done = __hip_atomic_load(p.sk_ready + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(S - 1);
            if (!done) __builtin_amdgcn_s_sleep(2);
        }
        if (done) {
            // every ticket of this tile is taken and every ready count is in: reset both for the next launch
            // on this stream (ordered after this kernel)
            __hip_atomic_store(p.sk_cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(p.sk_ready + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(p.sk_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // host-pinned word
        }
    }
    __syncthreads();
    if (S == 2 || SKMAX == 2) {
        splitk_gather<TM, TN, NW, 2, SMEM>(acc, slot0, PER_TILE, part, smem, wid, lane);
    } else if constexpr (SKMAX >= 4) {
        if (S == 3)
            splitk_gather<TM, TN, NW, 3, SMEM>(acc, slot0, PER_TILE, part, smem, wid, lane);
        else
            splitk_gather<TM, TN, NW, 4, SMEM>(acc, slot0, PER_TILE, part, smem, wid, lane);
    }
    return true;
}

// split-K workspace for `ntiles` tiles of `tile_bytes` each, S parts, on stream s (gemm.hip)
void splitk_setup(GemmParams& p, int ntiles, int S, size_t tile_bytes, hipStream_t s);
// quantized-weight GEMM launch for an already picked variant (gemm_q.hip)
void dispatch_quant(int fmt, int variant, const GemmParams& p, hipStream_t s);

}  // namespace gemm_detail
}  // namespace acemi
