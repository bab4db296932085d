// LDS-staged MFMA GEMM for the DiT block linears (gfx950 / CDNA4).
//
// Replaces every `ggml_mul_mat(W, x)` of `ace_dit::forward_dit`
// (acestep_dit_model.cpp:1194-1196,1257,1381,1412,1528-1531,1551) whose
// weights are BF16/F16: ggml rounds the f32 activation to the weight type
// (vec_dot_type) and accumulates in f32 — here the producer kernels already
// write the activation in that type and the MFMA accumulates in f32.
//
// Layout: A [M][K] and W [N][K] are both K-contiguous (the safetensors
// [out][in] layout is kept as-is), so both operands feed
// v_mfma_f32_16x16x32_{bf16,f16} straight from LDS with ds_read_b128.
// Staging: global_load_lds_dwordx4 (1 KiB per wave instruction) into a
// double-buffered LDS image of 128-byte rows whose 16-byte chunks are XOR
// swizzled with f(row) = (row >> 1) & 7 — the swizzle is applied to the
// per-lane SOURCE address (glds writes LDS lane-linearly) and undone on the
// ds_read, which makes every ds_read_b128 lane group conflict-free.
// Blocks are remapped XCD-aware (blocks b, b+8 share an XCD) and grouped
// along M so co-resident tiles share weight panels in L2.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "../kernels.h"
#include "prep_math.h"

namespace acemi {
namespace {

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
                        if constexpr (EPI == EPI_RESID_GATED) v = __fmul_rn(v, gt[ii][r][j]);
                        e.c_f32[(int64_t)m * e.ldc + n] = __fadd_rn(xo[ii][r][j], v);
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
                            e.c_f32[((int64_t)item * e.out_T + t) * e.out_ch + c] = __fadd_rn(v, e.bias[c]);
                        }
                    }
                }
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
                               base + b * bstride + (int64_t)n * 128, plane);
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
                    if (have == 0xffffu) {
                        *(uint4*)(vdst + g0) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
                        *(uint4*)(vdst + g0 + 8) = make_uint4(wv[4], wv[5], wv[6], wv[7]);
                        if (a.v_plane > 0) {
                            *(uint4*)(vdst + a.v_plane + g0) = make_uint4(wl[0], wl[1], wl[2], wl[3]);
                            *(uint4*)(vdst + a.v_plane + g0 + 8) = make_uint4(wl[4], wl[5], wl[6], wl[7]);
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < 16; ++k) {
                            if (!((have >> k) & 1u)) continue;
                            vdst[g0 + k] = (uint16_t)(wv[k >> 1] >> (16 * (k & 1)));
                            if (a.v_plane > 0) vdst[a.v_plane + g0 + k] = (uint16_t)(wl[k >> 1] >> (16 * (k & 1)));
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
        // bounded (~0.2 s; a real wait is a few microseconds): a protocol bug gives wrong tiles, never a hung GPU
        for (int it = 0; it < (1 << 22); ++it) {
            if (__hip_atomic_load(p.sk_ready + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(S - 1))
                break;
            __builtin_amdgcn_s_sleep(2);
        }
        // every ticket of this tile is taken and every ready count is in: reset both for the next launch
        // on this stream (ordered after this kernel)
        __hip_atomic_store(p.sk_cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(p.sk_ready + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// PIPE 0: stage(t+1) ; compute(t) ; vmcnt(0) ; __syncthreads        (2 LDS buffers)
// PIPE 1: compute first half of tile t from registers read up front, release the LDS buffer with
//         a raw s_barrier, stage tile t+2 into it, compute the second half, then a COUNTED
//         vmcnt(G) retires tile t+1 while t+2 stays in flight across the next barrier.
// SK: split-K instance, held to 256 VGPRs (two blocks per CU where their LDS fits) with a chunked residual preload
template <int BM, int BN, int WM, int WN, bool F16, int EPI, int PIPE, bool SK = false>
__global__ void __launch_bounds__(WM * WN * 64, SK && (BM + BN) * 512 <= 160 * 1024 ? 2 : 1) gemm_kernel(GemmParams p) {
    constexpr int NW = WM * WN;
    constexpr int WTM = BM / WM;
    constexpr int WTN = BN / WN;
    constexpr int TM = WTM / 16;
    constexpr int TN = WTN / 16;
    constexpr int BK = 64;
    constexpr int ROWB = BK * 2;
    constexpr int STAGE = (BM + BN) * ROWB;
    constexpr int G_PER_WAVE = (BM + BN) / 8 / NW;
    static_assert((BM + BN) % (8 * NW) == 0, "staging split");
    static_assert(EPI != EPI_SWIGLU || (TN % 2 == 0), "swiglu needs column pairs");

    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;

    const int S = SK ? p.ksplit : 1;
    int m0, n0, sk_tile = 0, sk_part = 0;
    unsigned ticket0 = 0;  // thread 0's split-K ticket
    if constexpr (SK) {
        int ntiles;
        splitk_block(S, sk_tile, sk_part, ntiles);
        block_tile<BM, BN>(p, m0, n0, sk_tile, ntiles);
        if (tid == 0) ticket0 = __hip_atomic_fetch_add(p.sk_cnt + sk_tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        block_tile<BM, BN>(p, m0, n0);
    }

    const int wm = wid / WN;
    const int wn = wid % WN;
    const int wm0 = wm * WTM;
    const int wn0 = wn * WTN;

    const int nk_all = p.K / BK;
    const int kt_begin = sk_part * nk_all / S;  // this block's K-tiles [kt_begin, kt_end)
    const int kt_end = (sk_part + 1) * nk_all / S;
    const uint16_t* __restrict__ A = p.A + kt_begin * BK;
    const uint16_t* __restrict__ W = p.W + kt_begin * BK;
    const int M = p.M;
    const int lda = p.lda, ldw = p.ldw;

    // per-lane staging source rows (fixed over K)
    const uint16_t* src[G_PER_WAVE];
#pragma unroll
    for (int j = 0; j < G_PER_WAVE; ++j) {
        const int g = wid + NW * j;
        const int row = g * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swz(row);
        if (row < BM) {
            const int gr = min(m0 + row, M - 1);
            src[j] = A + (int64_t)gr * lda + c * 8;
        } else {
            const int gr = n0 + row - BM;
            src[j] = W + (int64_t)gr * ldw + c * 8;
        }
    }

    auto stage = [&](int buf, int kt) {
        char* base = smem + buf * STAGE;
#pragma unroll
        for (int j = 0; j < G_PER_WAVE; ++j) {
            const int g = wid + NW * j;
            __builtin_amdgcn_global_load_lds((const void*)(src[j] + kt * BK), (lds_void*)(base + g * 1024), 16, 0,
                                             0);
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = kt_end - kt_begin;
    const int lrow = lane & 15;
    const int lchunk = lane >> 4;

    auto read_frags = [&](int buf, uint4 (&a)[TM][2], uint4 (&b)[TN][2]) {
        const char* As = smem + buf * STAGE;
        const char* Bs = As + BM * ROWB;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = wn0 + j * 16 + lrow;
                const int ch = (kk * 4 + lchunk) ^ swz(row);
                b[j][kk] = *(const uint4*)(Bs + row * ROWB + ch * 16);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm0 + i * 16 + lrow;
                const int ch = (kk * 4 + lchunk) ^ swz(row);
                a[i][kk] = *(const uint4*)(As + row * ROWB + ch * 16);
            }
        }
    };
    // asm variant: row = w0 + i*16 + lrow has swz(row) = (lrow >> 1) & 7 for every i (w0, i*16 are
    // multiples of 16), so fragment i sits at a lane base + i * 16 rows: one base per (operand, kk).
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    auto read_frags_asm = [&](int buf, uint4 (&a)[TM][2], uint4 (&b)[TN][2]) {
        const uint32_t sbase = lds0 + buf * STAGE;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = (kk * 4 + lchunk) ^ ((lrow >> 1) & 7);
            const uint32_t bb = sbase + BM * ROWB + (wn0 + lrow) * ROWB + ch * 16;
            const uint32_t ab = sbase + (wm0 + lrow) * ROWB + ch * 16;
            ReadRows<0, TN, 16 * ROWB>::run(bb, b, kk);
            ReadRows<0, TM, 16 * ROWB>::run(ab, a, kk);
        }
        lds_wait_all();
    };

    if constexpr (PIPE == 0) {
        stage(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            const int cur = kt & 1;
            if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
            uint4 a[TM][2], b[TN][2];
            read_frags(cur, a, b);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<F16>(a[i][kk], b[j][kk], acc[i][j]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    } else {
        stage(0, 0);
        if (nk > 1) {
            stage(1, 1);
            wait_vmcnt<G_PER_WAVE>();
        } else {
            wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        // MFMAs issued before the buffer-release barrier: the first half of the tile for the SwiGLU
        // (gate|up) instances, none elsewhere (240 s step, tools/ab_multi.sh: qkv with the fused prep 66.5
        // -> 61.6 us, the N = 2048 projections ~1 % faster; gate|up 1 % slower with none).  For the plain
        // stores the half split also made the register allocator rotate that half's accumulators through
        // VGPRs every iteration (48 v_accvgpr copies per 32 MFMAs in the 128x128 ISA).  The split-K
        // instances (held to 256 VGPRs) issue all of them before it: with the half split, hipcc rotated
        // that half through AGPRs there.
        // The 2x4-wave tiles (256x256, 192x256: batched sequences only) keep the round-1 rule (half before
        // the barrier for every non-store epilogue), the state they were measured in.
        constexpr int I_EARLY = SK ? TM
                                   : (EPI == EPI_SWIGLU ||
                                      (WN == 4 && EPI != EPI_STORE_F32 && EPI != EPI_STORE_ACT)) ? TM / 2 : 0;
        for (int kt = 0; kt < nk; ++kt) {
            const int cur = kt & 1;
            uint4 a[TM][2], b[TN][2];
            read_frags_asm(cur, a, b);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = 0; i < I_EARLY; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<F16>(a[i][kk], b[j][kk], acc[i][j]);
            __builtin_amdgcn_s_barrier();  // every wave has its fragments of tile kt: buffer `cur` is free
            const bool more = kt + 2 < nk;
            if (more) stage(cur, kt + 2);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = I_EARLY; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<F16>(a[i][kk], b[j][kk], acc[i][j]);
            if (kt + 1 < nk) {
                if (more)
                    wait_vmcnt<G_PER_WAVE>();  // tile kt+1 landed, kt+2 still in flight
                else
                    wait_vmcnt<0>();
                __builtin_amdgcn_s_barrier();
            }
        }
    }

    if constexpr (SK)
        if (!splitk_join<TM, TN, NW, SplitKMax<BM, BN>::value, 2 * STAGE>(p, acc, S, sk_tile, sk_part, tid, smem,
                                                                                ticket0))
            return;
    if constexpr (EPI == EPI_QKV_PREP)
        qkv_prep_tile<BM, NW, TM, TN, 2 * STAGE>(p, acc, m0, n0, wm0, wn0, tid, smem);
    else
        // residual preload chunk: whole tile for the 4-wave tiles; the 8-wave (2x4) tiles keep the round-1
        // one-row-group chunks (a whole-tile preload spilled 796 B per lane in the 256x256 gated residual)
        gemm_epilogue<TM, TN, F16, EPI, (SK ? 32 : (NW > 4 ? NW : 1024))>(p, acc, m0 + wm0, n0 + wn0, lane);
}


// ---------------------------------------------------------------------------------------------
// 8-wave ping-pong GEMM: BM x 256 tile, 512 threads as 2 (M) x 4 (N) waves, two wave groups
// (wr = 0 / 1, one wave of each on every SIMD) offset by one barrier, so one group's MFMA segment
// runs while the other group issues its LDS reads and LDS-DMA (CDNA guide §5, "256² 8-phase
// template": 8 barrier-separated segments per K-tile pair, counted vmcnt, raw s_barrier, setprio).
//
// A K-tile (64 deep) lives in one of two LDS buffers as four half-tiles: A0 / A1 (rows [0, BM/2),
// [BM/2, BM)) and B0 / B1 (columns [0, 128), [128, 256)).  A wave owns rows wr*QM*16.. of each A half
// and columns wc*32.. of each B half, i.e. four QM x 2 quadrants of 16x16 accumulators, one per phase:
//   ph1: read A0, B0 -> acc[0][0]   stage B1(t+1)
//   ph2: read B1     -> acc[0][1]   stage A1(t+1)
//   ph3: read A1     -> acc[1][1]   stage A0(t+2)
//   ph4: (no reads)  -> acc[1][0]   stage B0(t+2)
// Each phase: ds_reads, one half-tile of LDS-DMA, vmcnt(keep the 4 youngest half-tiles), barrier,
// lgkmcnt(0), MFMAs, barrier.  A half-tile is re-staged >= 2 phases after its last read (WAR across
// the staggered groups) and read >= 1 phase after the wait that retires it (RAW); stages past the
// last K-tile go to a scratch LDS region so the per-phase vmcnt counts stay uniform.
template <int BM, bool F16, int EPI>
__global__ void __launch_bounds__(512) gemm8_kernel(GemmParams p) {
    constexpr int BN = 256, BK = 64, ROWB = BK * 2;
    constexpr int HA = BM / 2;         // rows per A half-tile
    constexpr int QM = BM / 64;        // 16-row tiles per wave per A half
    constexpr int QN = 2;              // 16-col tiles per wave per B half
    constexpr int PA = HA / 8;         // 1 KiB LDS-DMA pieces per A half (B half: 16)
    constexpr int STAGE = (BM + BN) * ROWB;
    constexpr int SCRATCH = 2 * STAGE;
    static_assert(BM == 256 || BM == 192, "gemm8 tile rows");
    static_assert(EPI != EPI_SWIGLU || (QN % 2 == 0), "swiglu needs column pairs");

    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE + 16 * 1024];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    const int wr = wid >> 2, wc = wid & 3;
    int m0, n0;
    block_tile<BM, BN>(p, m0, n0);
    const int M = p.M;
    const int nk = p.K / BK;

    // LDS-DMA sources: this wave stages pieces wid and wid + 8 of every half-tile (A halves of BM = 192
    // have 12 pieces: waves 4..7 stage one).  Piece rows are wid*8 + (lane >> 3) (+ 64, + half offset),
    // all with the same chunk swizzle since the offsets are multiples of 16 rows.
    constexpr bool A2 = PA == 16;
    const bool a_second = A2 || wid + 8 < PA;
    const int prow = wid * 8 + (lane >> 3);
    const int pch = (lane & 7) ^ swz(prow);
    const uint16_t* srcA[2][2];
    const uint16_t* srcB[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ra = min(m0 + h * HA + j * 64 + prow, M - 1);
            srcA[h][j] = p.A + (int64_t)ra * p.lda + pch * 8;
            srcB[h][j] = p.W + (int64_t)(n0 + h * 128 + j * 64 + prow) * p.ldw + pch * 8;
        }
    auto stage_a = [&](int h, int t) {
        char* dst = t < nk ? smem + (t & 1) * STAGE + h * HA * ROWB : smem + SCRATCH;
        const int kt = min(t, nk - 1);
        __builtin_amdgcn_global_load_lds((const void*)(srcA[h][0] + kt * BK), (lds_void*)(dst + wid * 1024), 16, 0, 0);
        if (a_second)
            __builtin_amdgcn_global_load_lds((const void*)(srcA[h][1] + kt * BK), (lds_void*)(dst + (wid + 8) * 1024),
                                             16, 0, 0);
    };
    auto stage_b = [&](int h, int t) {
        char* dst = t < nk ? smem + (t & 1) * STAGE + (BM + h * 128) * ROWB : smem + SCRATCH;
        const int kt = min(t, nk - 1);
        __builtin_amdgcn_global_load_lds((const void*)(srcB[h][0] + kt * BK), (lds_void*)(dst + wid * 1024), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(srcB[h][1] + kt * BK), (lds_void*)(dst + (wid + 8) * 1024), 16,
                                         0, 0);
    };
    // retire all but the 4 youngest half-tiles (2 A + 2 B in any 4 consecutive phases) of this wave
    auto wait_stages = [&]() {
        if (a_second)
            wait_vmcnt<8>();
        else
            wait_vmcnt<6>();
    };

    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const int lrow = lane & 15, lchunk = lane >> 4;
    const int rsw = (lrow >> 1) & 7;
    auto read_a = [&](int buf, int h, uint4 (&a)[QM][2]) {
        const uint32_t base = lds0 + buf * STAGE + (h * HA + wr * QM * 16 + lrow) * ROWB;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) ReadRows<0, QM, 16 * ROWB>::run(base + (((kk * 4 + lchunk) ^ rsw) * 16), a, kk);
    };
    auto read_b = [&](int buf, int h, uint4 (&b)[QN][2]) {
        const uint32_t base = lds0 + buf * STAGE + (BM + h * 128 + wc * 32 + lrow) * ROWB;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) ReadRows<0, QN, 16 * ROWB>::run(base + (((kk * 4 + lchunk) ^ rsw) * 16), b, kk);
    };

    f32x4 acc[2][2][QM][QN];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int i = 0; i < QM; ++i)
#pragma unroll
                for (int j = 0; j < QN; ++j) acc[x][y][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto mma = [&](const uint4 (&a)[QM][2], const uint4 (&b)[QN][2], f32x4 (&c)[QM][QN]) {
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < QM; ++i)
#pragma unroll
                for (int j = 0; j < QN; ++j) c[i][j] = mfma16<F16>(a[i][kk], b[j][kk], c[i][j]);
        __builtin_amdgcn_s_setprio(0);
    };
    // segment boundary: the barrier that hands over to the other group
    auto seg = [&]() { __builtin_amdgcn_s_barrier(); };

    // prologue: A0 B0 B1 A1 of tile 0, A0 B0 of tile 1 (the steady-state stage order)
    stage_a(0, 0);
    stage_b(0, 0);
    stage_b(1, 0);
    stage_a(1, 0);
    stage_a(0, 1);
    stage_b(0, 1);
    wait_stages();
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one segment behind group 0

    uint4 a[QM][2], b0[QN][2], b1[QN][2];
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        // ph1
        read_a(buf, 0, a);
        read_b(buf, 0, b0);
        stage_b(1, kt + 1);
        wait_stages();
        seg();
        lds_wait_all();
        mma(a, b0, acc[0][0]);
        seg();
        // ph2
        read_b(buf, 1, b1);
        stage_a(1, kt + 1);
        wait_stages();
        seg();
        lds_wait_all();
        mma(a, b1, acc[0][1]);
        seg();
        // ph3: ph4 reads nothing, so no stage has to retire here (a wait here measured neutral)
        read_a(buf, 1, a);
        stage_a(0, kt + 2);
        seg();
        lds_wait_all();
        mma(a, b1, acc[1][1]);
        seg();
        // ph4
        stage_b(0, kt + 2);
        wait_stages();
        seg();
        __builtin_amdgcn_sched_barrier(0);
        mma(a, b0, acc[1][0]);
        seg();
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // both groups now at the same barrier count
    wait_vmcnt<0>();                            // the scratch-region stages of the last tiles

    if constexpr (EPI == EPI_QKV_PREP) {
        const int ccol = lane & 15, crow = (lane >> 4) * 4;
#pragma unroll
        for (int hb = 0; hb < 2; ++hb)
            qkv_prep_head<BM, 8, 2 * STAGE>(p, m0, (n0 >> 7) + hb, tid, smem, [&](float* tile, int c0, int CH) {
#pragma unroll
                for (int ha = 0; ha < 2; ++ha)
#pragma unroll
                    for (int i = 0; i < QM; ++i) {
                        const int rb = ha * HA + wr * QM * 16 + i * 16 - c0;
                        if (rb < 0 || rb >= CH) continue;
#pragma unroll
                        for (int r = 0; r < 4; ++r)
#pragma unroll
                            for (int j = 0; j < QN; ++j)
                                tile[(rb + crow + r) * PREP_LD + wc * 32 + j * 16 + ccol] = acc[ha][hb][i][j][r];
                    }
            });
    } else {
#pragma unroll
        for (int ha = 0; ha < 2; ++ha)
#pragma unroll
            for (int hb = 0; hb < 2; ++hb)
                gemm_epilogue<QM, QN, F16, EPI, 64>(p, acc[ha][hb], m0 + ha * HA + wr * QM * 16,
                                                   n0 + hb * 128 + wc * 32, lane);
    }
}

// ---------------------------------------------------------------------------------------------
// Dequant-fused variant: W arrives as a ggml block format re-laid out at load (runtime/quant.h).
// Each thread owns one 32-value block of the BN x 64 weight tile (BN*2 == threads): it loads the
// block's bytes + scale(s) into registers one k-tile ahead, turns them into bf16 with the exact
// ggml dequant arithmetic (q*d, d*sc*q - dmin*m, (d*sc)*q; one f32 rounding, then RNE bf16) and
// writes the bf16 image into the same swizzled LDS layout the dense kernel reads.  A (bf16
// activations) is still staged by LDS-DMA.  Pipeline (PIPE 1 shape): fragments of tile t are read
// up front, a raw barrier frees the buffer, A(t+2) is DMA'd and W(t+2) dequantized into it while
// the second half of tile t's MFMAs runs, and W(t+3)'s bytes are requested.
struct WRaw {
    u32x4 q0, q1;
    float s0, s1;
};

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
    bf16x2_t v;
    v[0] = (__bf16)lo;
    v[1] = (__bf16)hi;
    return __builtin_bit_cast(uint32_t, v);
}

// A compiler-visible LDS store, not inline asm: the hazard recognizer does not cover an asm
// ds_write_b128's data VGPRs, and on gfx950 the VALU overwrote them before the DS unit had read the
// last lanes (lanes 48-63 of the dequantized W rows came out wrong on the GPU).
__device__ __forceinline__ void ds_write_b128_v(uint32_t addr, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
    *(lds_u32x4*)(uintptr_t)addr = u32x4{a, b, c, d};
}

// Weight bytes are plain (compiler-tracked) loads issued one k-tile ahead; the loop consumes them
// BEFORE it issues the next A DMA, so the vmcnt the compiler places at that use only drains what
// must have landed by the end of the iteration anyway (tile kt+1's A, issued earlier).
template <int WQ>
__device__ __forceinline__ WRaw load_wq(const char* qbase, const float* sbase, int kt) {
    WRaw r;
    if constexpr (WQ == WF_Q4_K) {
        r.q0 = *(const u32x4*)(qbase + kt * 32);
        const float2 sm = *(const float2*)(sbase + kt * 4);
        r.s0 = sm.x;
        r.s1 = sm.y;
    } else {
        r.q0 = *(const u32x4*)(qbase + kt * 64);
        r.q1 = *(const u32x4*)(qbase + kt * 64 + 16);
        if constexpr (WQ == WF_Q8_0) {
            r.s0 = sbase[kt * 2];
            r.s1 = r.s0;
        } else {
            const float2 sc = *(const float2*)(sbase + kt * 4);
            r.s0 = sc.x;
            r.s1 = sc.y;
        }
    }
    return r;
}

// signed bytes of w (k order b0..b3) * s, via the unsigned-byte converts: (u - 128) * s = fma(u, s, -128 s)
__device__ __forceinline__ void deq_i8x4(uint32_t w, float s, float c, uint32_t& o0, uint32_t& o1) {
    const uint32_t u = w ^ 0x80808080u;
    const float f0 = fmaf((float)(u & 0xffu), s, c);
    const float f1 = fmaf((float)((u >> 8) & 0xffu), s, c);
    const float f2 = fmaf((float)((u >> 16) & 0xffu), s, c);
    const float f3 = fmaf((float)(u >> 24), s, c);
    o0 = pk_bf16(f0, f1);
    o1 = pk_bf16(f2, f3);
}
// unsigned nibble bytes (0..15) of w * d - m
__device__ __forceinline__ void deq_u4x4(uint32_t w, float d, float nm, uint32_t& o0, uint32_t& o1) {
    const float f0 = fmaf((float)(w & 0xffu), d, nm);
    const float f1 = fmaf((float)((w >> 8) & 0xffu), d, nm);
    const float f2 = fmaf((float)((w >> 16) & 0xffu), d, nm);
    const float f3 = fmaf((float)(w >> 24), d, nm);
    o0 = pk_bf16(f0, f1);
    o1 = pk_bf16(f2, f3);
}

// dequantize one 32-value block to 16 packed bf16 pairs in k order (ggml's dequant arithmetic, one f32
// rounding, then RNE to bf16)
template <int WQ>
__device__ __forceinline__ void dequant_block(const WRaw& r, uint32_t (&o)[16]) {
    if constexpr (WQ == WF_Q4_K) {
        const float d = r.s0, nm = -r.s1;
        const uint32_t w[4] = {r.q0[0], r.q0[1], r.q0[2], r.q0[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // dword i: k = 8i..8i+3 in low nibbles, 8i+4..8i+7 in high nibbles
            deq_u4x4(w[i] & 0x0f0f0f0fu, d, nm, o[4 * i + 0], o[4 * i + 1]);
            deq_u4x4((w[i] >> 4) & 0x0f0f0f0fu, d, nm, o[4 * i + 2], o[4 * i + 3]);
        }
    } else {
        const uint32_t w[8] = {r.q0[0], r.q0[1], r.q0[2], r.q0[3], r.q1[0], r.q1[1], r.q1[2], r.q1[3]};
        const float c0 = -128.0f * r.s0, c1 = -128.0f * r.s1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float s = i < 4 ? r.s0 : r.s1;
            const float c = i < 4 ? c0 : c1;
            deq_i8x4(w[i], s, c, o[2 * i], o[2 * i + 1]);
        }
    }
}

// dequantize one 32-value block and store it as 4 swizzled 16-byte chunks of an LDS row
template <int WQ>
__device__ __forceinline__ void dequant_store(const WRaw& r, uint32_t row_addr, int wh, int sw) {
    uint32_t o[16];
    dequant_block<WQ>(r, o);
#pragma unroll
    for (int c = 0; c < 4; ++c)
        ds_write_b128_v(row_addr + (((wh * 4 + c) ^ sw) * 16), o[4 * c], o[4 * c + 1], o[4 * c + 2], o[4 * c + 3]);
}

// Staged dequant: the bf16 image of a quantized [N][K] weight (the exact values the dequant-fused GEMM
// writes to LDS: the same deq_* arithmetic), one thread per 8 consecutive weights, so a wave reads 512
// (Q8_0, Q6_K) or 256 (Q4_K) contiguous bytes and writes 1 KiB contiguous.  HBM-bound: 1.0625 (Q8_0),
// 0.5625 (Q4_K), 1.125 (Q6_K) bytes read + 2 bytes written per weight.
struct DequantBatch {  // up to 8 same-format matrices expanded by one launch
    const char* q[8];
    const float* s[8];
    uint16_t* out[8];
    int64_t end[8];  // exclusive prefix sums of the 8-weight chunk counts
    int n;
};

template <int WQ>
__device__ __forceinline__ void dequant_chunk(const DequantBatch& b, int64_t c, uint4& o, uint16_t*& dst) {
    int mi = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) mi += (i + 1 < b.n && c >= b.end[i]) ? 1 : 0;
    if (mi > 0) c -= b.end[mi - 1];
    const char* __restrict__ q = b.q[mi];
    const float* __restrict__ sc = b.s[mi];
    const int64_t g = c >> 2;  // 8-weight chunk c: block g = c / 4, part j = c % 4
    const int j = (int)(c & 3);
    if constexpr (WQ == WF_Q4_K) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(q + g * 16 + j * 4);  // k 8j..8j+3 low, +4..7 high
        const float2 dm = *reinterpret_cast<const float2*>(sc + 2 * g);
        deq_u4x4(w & 0x0f0f0f0fu, dm.x, -dm.y, o.x, o.y);
        deq_u4x4((w >> 4) & 0x0f0f0f0fu, dm.x, -dm.y, o.z, o.w);
    } else {
        const uint2 w = *reinterpret_cast<const uint2*>(q + g * 32 + j * 8);
        const float d = WQ == WF_Q8_0 ? sc[g] : sc[2 * g + (j >> 1)];  // Q6_K: one scale per 16 values
        deq_i8x4(w.x, d, -128.0f * d, o.x, o.y);
        deq_i8x4(w.y, d, -128.0f * d, o.z, o.w);
    }
    dst = b.out[mi] + c * 8;
}

// CPT chunks per thread, strided by the grid so each wave instruction stays coalesced; all loads of a
// thread are issued before its first store
template <int WQ, int CPT>
__global__ void __launch_bounds__(256) dequant_bf16_kernel(DequantBatch b) {
    const int64_t tot = b.end[b.n - 1];
    const int64_t stride = (int64_t)gridDim.x * 256;
    const int64_t c0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    uint4 o[CPT];
    uint16_t* dst[CPT];
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        if (c0 + k * stride < tot) dequant_chunk<WQ>(b, c0 + k * stride, o[k], dst[k]);
#pragma unroll
    for (int k = 0; k < CPT; ++k)
        if (c0 + k * stride < tot) *reinterpret_cast<uint4*>(dst[k]) = o[k];
}

template <int BM, int BN, int WM, int WN, int EPI, int WQ>
__global__ void __launch_bounds__(WM * WN * 64) gemm_q_kernel(GemmParams p) {
    constexpr int NW = WM * WN;
    constexpr int WTM = BM / WM;
    constexpr int WTN = BN / WN;
    constexpr int TM = WTM / 16;
    constexpr int TN = WTN / 16;
    constexpr int BK = 64;
    constexpr int ROWB = BK * 2;
    constexpr int STAGE = (BM + BN) * ROWB;
    constexpr int G_A = BM / 8 / NW;
    static_assert(BM % (8 * NW) == 0, "A staging split");
    static_assert(BN * 2 == NW * 64, "one 32-value weight block per thread");
    static_assert(EPI != EPI_SWIGLU || (TN % 2 == 0), "swiglu needs column pairs");

    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;
    int m0, n0;
    block_tile<BM, BN>(p, m0, n0);
    const int wm0 = (wid / WN) * WTM;
    const int wn0 = (wid % WN) * WTN;
    const int M = p.M, K = p.K;

    // A staging sources (LDS-DMA, swizzled source chunk)
    const uint16_t* src[G_A];
#pragma unroll
    for (int j = 0; j < G_A; ++j) {
        const int row = (wid + NW * j) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swz(row);
        src[j] = p.A + (int64_t)min(m0 + row, M - 1) * p.lda + c * 8;
    }
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    auto stage_a = [&](int buf, int kt) {
        char* base = smem + buf * STAGE;
#pragma unroll
        for (int j = 0; j < G_A; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(src[j] + kt * BK), (lds_void*)(base + (wid + NW * j) * 1024),
                                             16, 0, 0);
    };

    // W block owned by this thread: row wr of the tile, K half wh of each 64-wide k-tile
    const int wr = tid >> 1, wh = tid & 1;
    const int64_t grow = n0 + wr;
    const char* qbase;
    const float* sbase;
    if constexpr (WQ == WF_Q4_K) {
        qbase = (const char*)p.Wq + grow * (K / 2) + wh * 16;
        sbase = p.Ws + (grow * (K / 32) + wh) * 2;
    } else if constexpr (WQ == WF_Q8_0) {
        qbase = (const char*)p.Wq + grow * K + wh * 32;
        sbase = p.Ws + grow * (K / 32) + wh;
    } else {
        qbase = (const char*)p.Wq + grow * K + wh * 32;
        sbase = p.Ws + grow * (K / 16) + wh * 2;
    }
    const int wsw = swz(wr);
    const uint32_t wrow_off = BM * ROWB + wr * ROWB;

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = K / BK;
    const int lrow = lane & 15;
    const int lchunk = lane >> 4;
    auto read_frags_asm = [&](int buf, uint4 (&a)[TM][2], uint4 (&b)[TN][2]) {
        const uint32_t sb = lds0 + buf * STAGE;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = (kk * 4 + lchunk) ^ ((lrow >> 1) & 7);
            const uint32_t bb = sb + BM * ROWB + (wn0 + lrow) * ROWB + ch * 16;
            const uint32_t ab = sb + (wm0 + lrow) * ROWB + ch * 16;
            ReadRows<0, TN, 16 * ROWB>::run(bb, b, kk);
            ReadRows<0, TM, 16 * ROWB>::run(ab, a, kk);
        }
        lds_wait_all();
    };

    // prologue: tiles 0 and 1 complete in LDS, W(min(2, nk-1)) requested
    WRaw wnext = load_wq<WQ>(qbase, sbase, 0);
    stage_a(0, 0);
    dequant_store<WQ>(wnext, lds0 + wrow_off, wh, wsw);
    if (nk > 1) {
        wnext = load_wq<WQ>(qbase, sbase, 1);
        stage_a(1, 1);
        dequant_store<WQ>(wnext, lds0 + STAGE + wrow_off, wh, wsw);
    }
    wnext = load_wq<WQ>(qbase, sbase, min(2, nk - 1));
    wait_vmcnt<0>();
    lds_wait_all();
    __builtin_amdgcn_s_barrier();

    auto mfma_all = [&](const uint4 (&a)[TM][2], const uint4 (&b)[TN][2]) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<false>(a[i][kk], b[j][kk], acc[i][j]);
    };

    // One branch-free body for every tile: past the end, the tile indices clamp to nk-1, so the last
    // two iterations re-stage the final tile into a buffer nobody reads again (harmless, and it keeps
    // the accumulators in one loop so they stay put in AGPRs).
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        uint4 a[TM][2], b[TN][2];
        read_frags_asm(cur, a, b);
        // Every MFMA of the tile issues after this barrier (the dequant VALU work interleaves with them).
        __builtin_amdgcn_s_barrier();  // every wave holds its fragments of tile kt: buffer `cur` is free
        asm volatile("" ::: "memory");  // the LDS stores below stay after the barrier
        // W(kt+2): waiting for its bytes also retires the older A(kt+1) DMA
        dequant_store<WQ>(wnext, lds0 + cur * STAGE + wrow_off, wh, wsw);
        // Every wave's ds_writes retire before any wave issues its LDS-DMA: measured on gfx950, an LDS
        // DMA issued while ds_write_b128s of the workgroup are still in flight corrupts lanes 48-63 of
        // those writes (random W elements of rows 24-31 of every 32, on some launches).  A per-wave
        // lgkmcnt(0) cleared the 4-wave tiles but not the 8-wave 256x256 one; lgkmcnt(0) + barrier
        // cleared all (tools/diag_gemm_q.py stress: 0 bad launches of 20 per variant and format).
        lds_wait_all();
        __builtin_amdgcn_s_barrier();
        stage_a(cur, min(kt + 2, nk - 1));
        // keep the W(kt+3) loads behind the A(kt+2) DMA in issue order: the vmcnt the compiler
        // places before the next iteration's dequant (waiting for those bytes) then also retires
        // A(kt+2) before the barrier that ends that iteration publishes buffer `cur` again
        asm volatile("" ::: "memory");
        wnext = load_wq<WQ>(qbase, sbase, min(kt + 3, nk - 1));
        mfma_all(a, b);
        // retire this wave's LDS traffic before the barrier that hands buffer `cur` to the other waves
        // (gfx950 does not wait at s_barrier)
        lds_wait_all();
        __builtin_amdgcn_s_barrier();
    }
    wait_vmcnt<0>();

    if constexpr (EPI == EPI_QKV_PREP)
        qkv_prep_tile<BM, NW, TM, TN, 2 * STAGE>(p, acc, m0, n0, wm0, wn0, tid, smem);
    else
        gemm_epilogue<TM, TN, false, EPI, NW >= 8 ? 64 : 1024>(p, acc, m0 + wm0, n0 + wn0, lane);
}

// split-K workspace of one stream: partial tiles + per-tile ticket / ready counters (zeroed once; each
// launch leaves them zero, see splitk_join).  Launches on one stream are ordered, so one set per
// stream suffices; it only grows (a grow waits for the stream before freeing the old buffers).
struct SplitKWs {
    void* ws = nullptr;
    size_t ws_bytes = 0;
    unsigned* cnt = nullptr;  // [2][tiles]: tickets, ready counts
    size_t tiles = 0;
};
std::mutex g_sk_mu;
std::unordered_map<hipStream_t, SplitKWs> g_sk;

void splitk_setup(GemmParams& p, int ntiles, int S, size_t tile_bytes, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_sk_mu);
    SplitKWs& w = g_sk[s];
    const size_t need = (size_t)ntiles * S * tile_bytes;
    if (w.ws_bytes < need || w.tiles < (size_t)ntiles) ACEMI_HIP(hipStreamSynchronize(s));
    if (w.ws_bytes < need) {
        if (w.ws) ACEMI_HIP(hipFree(w.ws));
        w.ws = nullptr;
        w.ws_bytes = 0;
        ACEMI_HIP(hipMalloc(&w.ws, need));
        w.ws_bytes = need;
    }
    if (w.tiles < (size_t)ntiles) {
        if (w.cnt) ACEMI_HIP(hipFree(w.cnt));
        w.cnt = nullptr;
        w.tiles = 0;
        const size_t t = std::max<size_t>((size_t)ntiles, 4096);
        ACEMI_HIP(hipMalloc(&w.cnt, 2 * t * sizeof(unsigned)));
        ACEMI_HIP(hipMemsetAsync(w.cnt, 0, 2 * t * sizeof(unsigned), s));
        w.tiles = t;
    }
    p.ksplit = S;
    p.sk_ws = static_cast<f32x4*>(w.ws);
    p.sk_cnt = w.cnt;
    p.sk_ready = w.cnt + w.tiles;
}

template <int BM, int BN, int WM, int WN, bool F16, int EPI, int PIPE>
void launch_cfg(GemmParams p, int S, hipStream_t s) {
    const int nbm = (p.M + BM - 1) / BM;
    const int nbn = p.N / BN;
    if (S > 1) {
        if (p.K / 64 < 2 * S) throw std::runtime_error("gemm: split-K needs at least two K-tiles per part");
        if (S > SplitKMax<BM, BN>::value) throw std::runtime_error("gemm: split-K factor too large for this tile");
        splitk_setup(p, nbm * nbn, S, (size_t)BM * BN * 4, s);
    }
    const dim3 grid(nbm * nbn * (S > 1 ? S : 1));
    const dim3 block(WM * WN * 64);
    if constexpr (EPI == EPI_QKV_PREP && BN != 128) {
        throw std::runtime_error("gemm: the fused attention prep needs 128-wide column tiles");
    } else if constexpr (WM * WN == 4 && PIPE == 1) {  // split-K instances: the 4-wave pipelined tiles
        if (S > 1)
            hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, F16, EPI, PIPE, true>), grid, block, 0, s, p);
        else
            hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, F16, EPI, PIPE>), grid, block, 0, s, p);
    } else {
        if (S > 1) throw std::runtime_error("gemm: split-K is for the 4-wave pipelined tiles");
        hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, F16, EPI, PIPE>), grid, block, 0, s, p);
    }
}

template <int BM, bool F16, int EPI>
void launch_cfg8(const GemmParams& p, hipStream_t s) {
    if (p.N % 256 != 0) throw std::runtime_error("gemm: the 8-wave tiles need N % 256 == 0");
    const int nbm = (p.M + BM - 1) / BM;
    hipLaunchKernelGGL((gemm8_kernel<BM, F16, EPI>), dim3(nbm * (p.N / 256)), dim3(512), 0, s, p);
}

// variant: 0 = 128x128 PIPE0, 1 = 128x128 PIPE1, 2 = 256x256 PIPE1 (8 waves 2x4), 3 = 256x128 PIPE1,
// 4 = 192x128 PIPE1, 5 = 192x256 PIPE1 (8 waves 2x4), 6 = 192x64 PIPE1 (dense only), 7 = 96x128 PIPE1,
// 8 = 64x128 PIPE1, 9 = 64x64 PIPE1 (8, 9 dense only: short sequences), 10 = 256x256 / 11 = 192x256 8-wave
// ping-pong (dense only, N % 256 == 0)
// variant + 100 * S (S = 2..4): the 4-wave tiles with split-K over S blocks per tile (splitk_join)
template <bool F16, int EPI>
void launch_variant(int variant, const GemmParams& p, hipStream_t s) {
    const int S = variant / 100;
    if (S > 1 && variant % 100 >= 10) throw std::runtime_error("gemm: split-K is for the 4-wave tiles");
    switch (variant % 100) {
        case 0: launch_cfg<128, 128, 2, 2, F16, EPI, 0>(p, S, s); break;
        case 1: launch_cfg<128, 128, 2, 2, F16, EPI, 1>(p, S, s); break;
        case 2: launch_cfg<256, 256, 2, 4, F16, EPI, 1>(p, S, s); break;
        case 3: launch_cfg<256, 128, 2, 2, F16, EPI, 1>(p, S, s); break;
        case 4: launch_cfg<192, 128, 2, 2, F16, EPI, 1>(p, S, s); break;
        case 5: launch_cfg<192, 256, 2, 4, F16, EPI, 1>(p, S, s); break;
        case 6: launch_cfg<192, 64, 2, 2, F16, EPI, 1>(p, S, s); break;
        case 7: launch_cfg<96, 128, 2, 2, F16, EPI, 1>(p, S, s); break;
        case 8: launch_cfg<64, 128, 2, 2, F16, EPI, 1>(p, S, s); break;
        case 9: launch_cfg<64, 64, 2, 2, F16, EPI, 1>(p, S, s); break;
        case 10: launch_cfg8<256, F16, EPI>(p, s); break;
        case 11: launch_cfg8<192, F16, EPI>(p, s); break;
        default: throw std::runtime_error("gemm: bad variant");
    }
}

template <bool F16>
void dispatch_epi(int variant, const GemmParams& p, hipStream_t s) {
    switch (p.e.kind) {
        case EPI_STORE_F32: launch_variant<F16, EPI_STORE_F32>(variant, p, s); break;
        case EPI_STORE_ACT: launch_variant<F16, EPI_STORE_ACT>(variant, p, s); break;
        case EPI_RESID_GATED: launch_variant<F16, EPI_RESID_GATED>(variant, p, s); break;
        case EPI_RESID: launch_variant<F16, EPI_RESID>(variant, p, s); break;
        case EPI_SWIGLU: launch_variant<F16, EPI_SWIGLU>(variant, p, s); break;
        case EPI_PROJ_OUT: launch_variant<F16, EPI_PROJ_OUT>(variant, p, s); break;
        case EPI_QKV_PREP: launch_variant<F16, EPI_QKV_PREP>(variant, p, s); break;
        default: throw std::runtime_error("gemm: bad epilogue kind");
    }
}

template <int BM, int BN, int WM, int WN, int EPI, int WQ>
void launch_q_cfg(const GemmParams& p, hipStream_t s) {
    const int nbm = (p.M + BM - 1) / BM;
    const int nbn = p.N / BN;
    if constexpr (EPI == EPI_QKV_PREP && BN != 128)
        throw std::runtime_error("gemm: the fused attention prep needs 128-wide column tiles");
    else
        hipLaunchKernelGGL((gemm_q_kernel<BM, BN, WM, WN, EPI, WQ>), dim3(nbm * nbn), dim3(WM * WN * 64), 0, s, p);
}

template <int EPI, int WQ>
void launch_q_variant(int variant, const GemmParams& p, hipStream_t s) {
    switch (variant) {
        case 0:
        case 1: launch_q_cfg<128, 128, 2, 2, EPI, WQ>(p, s); break;
        case 2: launch_q_cfg<256, 256, 2, 4, EPI, WQ>(p, s); break;
        case 3: launch_q_cfg<256, 128, 2, 2, EPI, WQ>(p, s); break;
        case 4: launch_q_cfg<192, 128, 2, 2, EPI, WQ>(p, s); break;
        case 5: launch_q_cfg<192, 256, 2, 4, EPI, WQ>(p, s); break;
        case 7: launch_q_cfg<96, 128, 2, 2, EPI, WQ>(p, s); break;
        default: throw std::runtime_error("gemm: bad variant");
    }
}

template <int WQ>
void dispatch_q_epi(int variant, const GemmParams& p, hipStream_t s) {
    switch (p.e.kind) {
        case EPI_STORE_F32: launch_q_variant<EPI_STORE_F32, WQ>(variant, p, s); break;
        case EPI_STORE_ACT: launch_q_variant<EPI_STORE_ACT, WQ>(variant, p, s); break;
        case EPI_RESID_GATED: launch_q_variant<EPI_RESID_GATED, WQ>(variant, p, s); break;
        case EPI_RESID: launch_q_variant<EPI_RESID, WQ>(variant, p, s); break;
        case EPI_SWIGLU: launch_q_variant<EPI_SWIGLU, WQ>(variant, p, s); break;
        case EPI_PROJ_OUT: launch_q_variant<EPI_PROJ_OUT, WQ>(variant, p, s); break;
        case EPI_QKV_PREP: launch_q_variant<EPI_QKV_PREP, WQ>(variant, p, s); break;
        default: throw std::runtime_error("gemm: bad epilogue kind");
    }
}

int g_forced_variant = -1;

// Tile choice: measured kernel ceiling (random bf16 operands, MI355X: v1 ~950, v2 ~1120 TFLOP/s at
// large shapes) times the wave-quantization efficiency of the grid over 256 CUs (v1: 2 blocks/CU,
// 64 KiB LDS each; v2: 1 block/CU, 128 KiB) and the M-edge utilisation.
// Tile choice from the measured table (tools/gemm_bench.py on MI355X, profiles/r01_gemm_bench.log): at
// M = 3000 the 192-row tiles make 16 exact M blocks, so 192x128 fills the chip in whole rounds where
// 128x128 leaves a half round (qkv: 512 vs 768 tiles, 1036 vs 854 TFLOP/s; gate|up 1536 tiles, 900 vs
// 827); with only N = 2048 (256 tiles) the 128x128 tile's two blocks per CU win (down 779 vs 684).
// Dequant-fused: 192x256 (one block per CU, the dequant VALU spread over 8 waves) leads where it
// gives at least one tile per CU (gate|up 655 vs 525, qkv 709 vs 502), else 192x128 (down 506 vs 437).
// Dense N = 2048 at M = 3000: 96x128 makes 512 tiles, exactly two blocks per CU (down 857 vs 775,
// o / cross 662 vs 569).
double m_edge(int M, int bm) { return (double)M / (double)(((M + bm - 1) / bm) * bm); }

int pick_variant(int M, int N, int K, bool quant) {
    if (g_forced_variant >= 0) {  // forced (tests / micro-benchmarks), where that tile supports the shape
        const int f = g_forced_variant % 100, S = g_forced_variant / 100;
        const bool wide = f == 2 || f == 5 || f == 10 || f == 11;
        const bool dense_only = f == 6 || f >= 8 || S > 1;
        const bool sk_ok = S <= 1 || ((f == 1 || f == 3 || f == 4 ? S <= 2 : (f >= 6 && f <= 9 && S <= 4)) &&
                                      K / 64 >= 2 * S);
        if (!(wide && N % 256 != 0) && !(quant && dense_only) && sk_ok) return g_forced_variant;
    }
    const int64_t mb192 = (M + 191) / 192;
    const bool edge_ok = m_edge(M, 192) >= m_edge(M, 128) - 0.02;
    if (quant) {
        if (N % 256 == 0 && edge_ok && mb192 * (N / 256) >= 256) return 5;
        if (m_edge(M, 96) >= m_edge(M, 128) - 0.02) return 7;  // down 590 vs 493, o / cross 474 vs 396
        return 1;
    }
    // 8-wave ping-pong tiles for batched sequences (tools/gemm_msweep.py on MI355X, TFLOP/s): M = 12000 gate|up
    // 1011 (256x256) vs 941 (v2), qkv 933 vs 902, down 922 (192x256) vs 818, o 814 vs 786; M = 24000 gate|up
    // 1089 vs 1016, qkv 941 vs 897, down 955 vs 915, o 767 (v2) vs 724; M = 6000 down 921 (192x256) vs 853.
    // At M = 3000 the 4-wave tiles stay ahead (their second block per CU hides prologue and epilogue).
    if (N % 256 == 0 && M >= 8192) {
        if (N >= 4096) return 10;
        if (M >= 20000) return K >= 4096 ? 10 : 2;
        return 11;
    }
    if (N % 256 == 0 && M >= 4500 && N <= 2048 && K >= 4096) return 11;
    if (edge_ok && mb192 * (N / 128) >= 384) return 4;
    // short sequences (60 s: M = 750): too few 96-row tiles to cover the CUs -> 64-row tiles, and
    // 64x64 when even those leave CUs idle (M = 750: N = 2048 projections 273-337 -> 364-453 TFLOP/s,
    // qkv 519 -> 567, tools/gemm_small_m.py)
    // split-K (tools/gemm_msweep.py, MI355X): only the K = 6144 down projection between the short and the
    // full-length tiles gains (M = 1500: 96x128 over 2 parts 722 vs 637 TFLOP/s for 64x128); elsewhere the
    // join's device-coherent partial round trip (~3-4 us after the main loop) costs more than the fuller grid
    if (N <= 2048 && K >= 4096 && M >= 1000 && M < 2000) return 207;
    const int64_t mb96 = (M + 95) / 96, mb64 = (M + 63) / 64;
    if (mb96 * (N / 128) <= 256) return mb64 * (N / 128) >= 256 ? 8 : 9;
    if (m_edge(M, 96) >= m_edge(M, 128) - 0.02) return 7;  // N = 2048: 512 tiles, two per CU
    return 1;
}

}  // namespace

void launch_gemm(const uint16_t* A, int lda, const WeightView& W, int M, int N, int K, const GemmEpilogue& epi,
                 hipStream_t s) {
    ACEMI_CHECK(M >= 1 && N % 128 == 0 && K % 64 == 0 && K >= 64, "gemm: unsupported shape");
    ACEMI_CHECK(lda % 8 == 0, "gemm: leading dims must be multiples of 8");
    ACEMI_CHECK(W.q != nullptr, "gemm: null weight");
    GemmParams p{A, (const uint16_t*)W.q, W.q, W.s, lda, W.ld, M, N, K, epi};
    int v = pick_variant(M, N, K, weight_quantized(W.fmt));
    if (epi.kind == EPI_QKV_PREP) {  // 128-wide column tiles: one head per tile
        ACEMI_CHECK(epi.bias == nullptr && epi.prep.n_tok > 0 && M % epi.prep.n_tok == 0,
                    "gemm: fused attention prep needs no bias and whole items");
        ACEMI_CHECK(N == 128 * ((epi.prep.q_col >= 0 ? epi.prep.hq : 0) + (epi.prep.k_col >= 0 ? epi.prep.hkv : 0) +
                                (epi.prep.v_col >= 0 ? epi.prep.hkv : 0)),
                    "gemm: fused attention prep column count");
        const int nqc = epi.prep.q_col >= 0 ? epi.prep.hq : 0, nkc = epi.prep.k_col >= 0 ? epi.prep.hkv : 0;
        ACEMI_CHECK(epi.prep.q_col <= 0 && (epi.prep.k_col < 0 || epi.prep.k_col == 128 * nqc) &&
                        (epi.prep.v_col < 0 || epi.prep.v_col == 128 * (nqc + nkc)),
                    "gemm: fused attention prep expects the [q | k | v] head order");
        v = v == 2 ? 3 : v == 5 ? 4 : v == 6 ? 1 : v == 9 ? 8 : v;
    }
    switch (W.fmt) {
        case WF_BF16:
        case WF_F16:
            ACEMI_CHECK(W.ld % 8 == 0, "gemm: leading dims must be multiples of 8");
            if (W.fmt == WF_F16)
                dispatch_epi<true>(v, p, s);
            else
                dispatch_epi<false>(v, p, s);
            break;
        case WF_Q8_0:
            ACEMI_CHECK(W.s != nullptr, "gemm: null scales");
            dispatch_q_epi<WF_Q8_0>(v, p, s);
            break;
        case WF_Q4_K:
            ACEMI_CHECK(W.s != nullptr, "gemm: null scales");
            dispatch_q_epi<WF_Q4_K>(v, p, s);
            break;
        case WF_Q6_K:
            ACEMI_CHECK(W.s != nullptr, "gemm: null scales");
            dispatch_q_epi<WF_Q6_K>(v, p, s);
            break;
        default: throw std::runtime_error("gemm: bad weight format");
    }
    ACEMI_HIP(hipGetLastError());
}

void launch_gemm(ActType t, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                 const GemmEpilogue& epi, hipStream_t s) {
    WeightView w;
    w.fmt = t == ActType::F16 ? WF_F16 : WF_BF16;
    w.q = W;
    w.ld = ldw;
    launch_gemm(A, lda, w, M, N, K, epi, s);
}

void gemm_force_variant(int v) { g_forced_variant = v; }

void launch_dequant_bf16_batch(const DequantJob* jobs, int n, hipStream_t s) {
    ACEMI_CHECK(n >= 1 && n <= 8, "dequant: 1..8 matrices per launch");
    DequantBatch b{};
    int64_t tot = 0;
    for (int i = 0; i < n; ++i) {
        const DequantJob& jb = jobs[i];
        ACEMI_CHECK(weight_quantized(jb.w.fmt) && jb.w.fmt == jobs[0].w.fmt && jb.w.q && jb.w.s && jb.K % 32 == 0 &&
                        jb.N > 0 && jb.out,
                    "dequant: same-format quantized [N][K] weights");
        b.q[i] = static_cast<const char*>(jb.w.q);
        b.s[i] = jb.w.s;
        b.out[i] = jb.out;
        tot += (int64_t)jb.N * (jb.K / 8);  // 8-weight chunks
        b.end[i] = tot;
    }
    b.n = n;
    static const int cpt = [] {  // chunks per thread (A/B knob; 2 by default: 46 vs 47.5 / 49 us for 1 / 4)
        const char* e = std::getenv("ACE_MI_DEQ_CPT");
        const int v = e ? std::atoi(e) : 2;
        return v == 1 || v == 4 || v == 8 ? v : 2;
    }();
    const dim3 grid((unsigned)((tot + 256 * cpt - 1) / (256 * cpt)));
#define ACEMI_DEQ(WQ)                                                                         \
    switch (cpt) {                                                                            \
        case 1: hipLaunchKernelGGL((dequant_bf16_kernel<WQ, 1>), grid, dim3(256), 0, s, b); break; \
        case 4: hipLaunchKernelGGL((dequant_bf16_kernel<WQ, 4>), grid, dim3(256), 0, s, b); break; \
        case 8: hipLaunchKernelGGL((dequant_bf16_kernel<WQ, 8>), grid, dim3(256), 0, s, b); break; \
        default: hipLaunchKernelGGL((dequant_bf16_kernel<WQ, 2>), grid, dim3(256), 0, s, b); break; \
    }
    switch (jobs[0].w.fmt) {
        case WF_Q8_0: ACEMI_DEQ(WF_Q8_0); break;
        case WF_Q4_K: ACEMI_DEQ(WF_Q4_K); break;
        case WF_Q6_K: ACEMI_DEQ(WF_Q6_K); break;
        default: throw std::runtime_error("dequant: bad weight format");
    }
#undef ACEMI_DEQ
    ACEMI_HIP(hipGetLastError());
}

void launch_dequant_bf16(const WeightView& W, int N, int K, uint16_t* out, hipStream_t s) {
    const DequantJob j{W, N, K, out};
    launch_dequant_bf16_batch(&j, 1, s);
}

}  // namespace acemi
