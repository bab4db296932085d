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
#include <array>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <map>
#include <vector>
#include <type_traits>
#include <utility>

#include "gemm_common.h"

namespace acemi {
namespace gemm_detail {

// Diagnostic ablations (A/B builds only, tools/build_ab.sh; results are wrong by design): bit 0 drops the main loop's
// LDS-DMA staging (every k-tile reuses the prologue's tiles), bit 1 its LDS fragment reads (registers of the first
// k-tile reused), bit 2 stages k-tile 0 again and again (the DMA issue kept, its bytes L2-hot) -- what the loop costs
// without that traffic.
#ifndef ACEMI_GEMM_ABLATE
#define ACEMI_GEMM_ABLATE 0
#endif
constexpr int kAblate = ACEMI_GEMM_ABLATE;


// PIPE 0: stage(t+1) ; compute(t) ; vmcnt(0) ; __syncthreads        (2 LDS buffers)
// PIPE 1: compute first half of tile t from registers read up front, release the LDS buffer with
//         a raw s_barrier, stage tile t+2 into it, compute the second half, then a COUNTED
//         vmcnt(G) retires tile t+1 while t+2 stays in flight across the next barrier.
// SK: split-K instance, held to 256 VGPRs (two blocks per CU where their LDS fits) with a chunked residual preload
// (the residual-prefetch instances, XPF below, are held to 256 VGPRs too: two blocks per CU)
template <int TBM, int TBN, int TWM, int TWN, int TEPI, int TPIPE, bool TSK>
struct GemmTwoPerCU {
    static constexpr bool value =
        (TSK || ((TEPI == EPI_RESID || TEPI == EPI_RESID_GATED) && TPIPE >= 1 && TWM * TWN == 4 &&
                 (TBM / TWM / 16) * 4 * (TBN / TWN / 16) + (TEPI == EPI_RESID_GATED ? 2 * (TBN / TWN / 16) : 0) <= 63)) &&
        (TBM + TBN) * 256 * (TPIPE >= 3 ? TPIPE : 2) <= 160 * 1024;
};

template <int BM, int BN, int WM, int WN, bool F16, int EPI, int PIPE, bool SK = false>
__global__ void __launch_bounds__(WM * WN * 64, (GemmTwoPerCU<BM, BN, WM, WN, EPI, PIPE, SK>::value ? 2 : 1))
    gemm_kernel(GemmParams p) {
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
    // residual prefetch for the 4-wave pipelined tiles whose x (+ gate) loads fit one counted vmcnt
    constexpr int NX = TM * 4 * TN + (EPI == EPI_RESID_GATED ? 2 * TN : 0);
    constexpr bool XPF = (EPI == EPI_RESID || EPI == EPI_RESID_GATED) && PIPE >= 1 && !SK && NW == 4 && NX <= 63;
    constexpr int XW = NX;

    // LDS stages: PIPE 0 / 1 double-buffer; PIPE 3 / 4 keep 3 / 4 k-tiles in the ring (short-sequence tiles, whose
    // few MFMAs per k-tile cannot cover an L2 / Infinity Cache round trip with one tile in flight)
    constexpr int NS = PIPE >= 3 ? PIPE : 2;
    __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

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
            __builtin_amdgcn_global_load_lds((const void*)(src[j] + ((kAblate & 4) ? 0 : kt) * BK),
                                             (lds_void*)(base + g * 1024), 16, 0, 0);
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
    // wait until at most `younger` k-tiles' LDS-DMA (G_PER_WAVE instructions each) of this wave are in flight
    auto wait_retire = [&](int younger) {
        if (NS >= 4 && younger >= 3)
            wait_vmcnt<(NS >= 4 ? 3 : 0) * G_PER_WAVE>();
        else if (NS >= 3 && younger >= 2)
            wait_vmcnt<(NS >= 3 ? 2 : 0) * G_PER_WAVE>();
        else if (younger >= 1)
            wait_vmcnt<G_PER_WAVE>();
        else
            wait_vmcnt<0>();
    };

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
            mfma_war_retire(a, b);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    } else {
        // prologue: k-tiles 0 .. NS-1 requested, tile 0 retired
#pragma unroll
        for (int t = 0; t < NS; ++t)
            if (t < nk) stage(t, t);
        wait_retire(min(nk, NS) - 1);
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
        // Residual prefetch (XPF, the o / cross-o / down projections): the old x (and gate) values of the tile
        // are requested right after the barrier of k-tile nk-2 -- no staging happens from there on, so the
        // counted vmcnt(XW) at its end retires tile nk-1's LDS-DMA while the x loads stay in flight -- and land
        // during the last two k-tiles' MFMAs.  The epilogue then only adds and stores: its read-modify-write of
        // the f32 residual (96 x 128 x 4 B read + written per block, all blocks at once) no longer waits for
        // HBM after the main loop.  The two peeled calls keep the prefetched registers out of any loop.
        float xo[TM][4][TN];  // (dead unless XPF)
        float g0[TN], g1[TN];
        uint4 a_keep[TM][2], b_keep[TN][2];  // (ablation builds only)
        auto body = [&](int kt, auto pf_tag) {
            constexpr bool PF = decltype(pf_tag)::value;
            const int cur = kt % NS;
            uint4 a[TM][2], b[TN][2];
            if constexpr (kAblate & 2) {
                if (kt == 0) read_frags_asm(cur, a_keep, b_keep);
#pragma unroll
                for (int i = 0; i < TM; ++i) a[i][0] = a_keep[i][0], a[i][1] = a_keep[i][1];
#pragma unroll
                for (int j = 0; j < TN; ++j) b[j][0] = b_keep[j][0], b[j][1] = b_keep[j][1];
            } else {
                read_frags_asm(cur, a, b);
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = 0; i < I_EARLY; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<F16>(a[i][kk], b[j][kk], acc[i][j]);
            if constexpr (I_EARLY > 0) mfma_war_retire(a, b);
            __builtin_amdgcn_s_barrier();  // every wave has its fragments of tile kt: buffer `cur` is free
            const bool more = kt + NS < nk && !(kAblate & 1);
            if (more) stage(cur, kt + NS);
            if constexpr (PF) resid_prefetch<TM, TN, EPI>(p, m0 + wm0, n0 + wn0, lane, BM / WM, xo, g0, g1);
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
#pragma unroll
                for (int i = I_EARLY; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<F16>(a[i][kk], b[j][kk], acc[i][j]);
            mfma_war_retire(a, b);
            if (kt + 1 < nk) {
                if constexpr (PF)
                    wait_vmcnt<XW>();  // tile kt+1 (the last) landed, the residual prefetch still in flight
                else
                    wait_retire(min(kt + NS, nk - 1) - (kt + 1));  // tile kt+1 landed, the younger ones in flight
                __builtin_amdgcn_s_barrier();
            }
        };
        if constexpr (XPF) {
            const int kp = nk >= 2 ? nk - 2 : 0;  // no staging from here on (kp + NS >= nk)
            for (int kt = 0; kt < kp; ++kt) body(kt, std::false_type{});
            body(kp, std::true_type{});
            if (kp + 1 < nk) body(kp + 1, std::false_type{});
            resid_apply<TM, TN, EPI>(p, acc, m0 + wm0, n0 + wn0, lane, BM / WM, xo, g0, g1);
            return;
        } else {
            for (int kt = 0; kt < nk; ++kt) body(kt, std::false_type{});
        }
    }

    if constexpr (SK)
        if (!splitk_join<TM, TN, NW, SplitKMax<BM, BN>::value, NS * STAGE>(p, acc, S, sk_tile, sk_part, tid, smem,
                                                                                ticket0))
            return;
    if constexpr (EPI == EPI_QKV_PREP)
        qkv_prep_tile<BM, NW, TM, TN, NS * STAGE>(p, acc, m0, n0, wm0, wn0, tid, smem);
    else
        // residual preload chunk: whole tile for the 4-wave tiles; the 8-wave (2x4) tiles keep the round-1
        // one-row-group chunks (a whole-tile preload spilled 796 B per lane in the 256x256 gated residual)
        gemm_epilogue<TM, TN, F16, EPI, (SK ? 32 : (NW > 4 ? NW : 1024))>(p, acc, m0 + wm0, n0 + wn0, lane);
}


// ---------------------------------------------------------------------------------------------
// Warp-specialized GEMM (variant 18): BM x BN tile, 512 threads = 4 MFMA waves (2 x 2, one per SIMD) + 4
// loader waves (one per SIMD) that issue every LDS-DMA piece.  Measured on the single-role tiles (tools/build_ab.sh
// ablations, profiles/r04/gemm_ablation.md): dropping the main loop's LDS-DMA took the 192x128 tile from 930 to 1127
// TFLOP/s at gate|up and the 96x128 one from 784 to 1051 at the N = 2048 projections, and re-staging L2-hot bytes
// (the DMA issue kept) recovered only 5 % of that -- a wave that issues LDS-DMA pieces stalls its own MFMA stream
// (≈60 cycles per 1 KiB piece, MI355X_MICROARCH.md), whatever the bytes cost.  Here the MFMA waves only read LDS
// and issue MFMAs; the pieces come from waves that have nothing else to issue.
//   ring: NS k-tile slots; the loaders keep tiles t+1 .. t+NS-1 in flight and publish tile t+1 at barrier B(t+1);
//   MFMA waves, k-tile t: half 0 (k 0..31) from registers while the half-1 fragments are read, lgkmcnt(0), B(t+1)
//   (slot t fully read -> the loaders refill it with tile t+NS), half 1 while tile t+1's half-0 fragments are read.
// One barrier per k-tile; a loader waits (counted vmcnt) for tile t+1 just before B(t+1), so tile t+1 has had the
// NS-2 iterations since its issue to land.  Same operands, swizzled LDS image, MFMA and per-element k order as
// gemm_kernel: results are bit-identical to the other dense tiles.
template <int BM, int BN, bool F16, int EPI, int NS>
__global__ void __launch_bounds__(512, 1) gemm_ws_kernel(GemmParams p) {
    constexpr int NC = 4, WN = 2;  // MFMA waves (2 x 2)
    constexpr int WTM = BM / 2, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int BK = 64, ROWB = BK * 2;
    constexpr int STAGE = (BM + BN) * ROWB;
    constexpr int G = (BM + BN) / 8 / 4;  // 1 KiB pieces per loader wave per k-tile
    static_assert((BM + BN) % 32 == 0 && NS >= 3, "ws tile");
    static_assert(EPI != EPI_SWIGLU || (TN % 2 == 0), "swiglu needs column pairs");
    __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int m0, n0;
    block_tile<BM, BN>(p, m0, n0);
    const int nk = p.K / BK;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

    if (wid >= NC) {  // ---- loader wave ----
        const int lw = wid - NC;
        const uint16_t* src[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int row = (lw + 4 * j) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ swz(row);
            src[j] = row < BM ? p.A + (int64_t)min(m0 + row, p.M - 1) * p.lda + c * 8
                              : p.W + (int64_t)(n0 + row - BM) * p.ldw + c * 8;
        }
        auto stage = [&](int slot, int kt) {
#pragma unroll
            for (int j = 0; j < G; ++j)
                __builtin_amdgcn_global_load_lds((const void*)(src[j] + kt * BK),
                                                 (lds_void*)(smem + slot * STAGE + (lw + 4 * j) * 1024), 16, 0, 0);
        };
        // wait until at most n (0 .. NS-1) younger k-tiles of this wave are in flight
        auto wait_tiles = [&](int n) {
            if (NS >= 4 && n >= 3) wait_vmcnt<(NS >= 4 ? 3 : 0) * G>();
            else if (n == 2) wait_vmcnt<2 * G>();
            else if (n == 1) wait_vmcnt<G>();
            else wait_vmcnt<0>();
        };
#pragma unroll
        for (int t = 0; t < NS; ++t)
            if (t < nk) stage(t, t);
        wait_tiles(min(NS, nk) - 1);  // tile 0
        __builtin_amdgcn_s_barrier();  // B(0)
        for (int j = 1; j < nk; ++j) {
            wait_tiles(min(nk - 1, j - 2 + NS) - j);  // tile j landed (tiles up to j-2+NS issued)
            __builtin_amdgcn_s_barrier();              // B(j): slot (j-1) % NS read by every MFMA wave
            if (j - 1 + NS < nk) stage((j - 1) % NS, j - 1 + NS);
        }
        wait_vmcnt<0>();
        if constexpr (EPI == EPI_QKV_PREP)
            qkv_prep_head<BM, 8, NS * STAGE>(p, m0, n0 >> 7, tid, smem, [](float*, int, int) {});
        return;
    }

    // ---- MFMA wave ----
    const int wm0 = (wid / WN) * WTM, wn0 = (wid % WN) * WTN;
    const int lrow = lane & 15, lchunk = lane >> 4;
    const int rsw = (lrow >> 1) & 7;
    const uint32_t ch[2] = {(uint32_t)((lchunk ^ rsw) * 16), (uint32_t)(((4 + lchunk) ^ rsw) * 16)};
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    uint4 a[TM][2], b[TN][2];
    // fragment r of half h of the k-tile in `slot`: r < TN -> B fragment r, else A fragment r - TN
    auto rd = [&](auto r_c, int slot, auto h_c) {
        constexpr int r = decltype(r_c)::value, h = decltype(h_c)::value;
        const uint32_t sb = lds0 + slot * STAGE + ch[h];
        if constexpr (r < TN)
            b[r][h] = ds_read_b128_off<r * 16 * ROWB>(sb + (BM + wn0 + lrow) * ROWB);
        else
            a[r - TN][h] = ds_read_b128_off<(r - TN) * 16 * ROWB>(sb + (wm0 + lrow) * ROWB);
    };
    // the TM x TN MFMAs of half h, the fragment reads of half hr (k-tile in `slot`) one after each of the first
    // TM + TN MFMAs
    auto half = [&](auto h_c, int slot, auto hr_c, auto reads_c) {
        constexpr int h = decltype(h_c)::value;
        static_for<0, TM * TN>([&](auto s_c) {
            constexpr int st = decltype(s_c)::value;
            acc[st / TN][st % TN] = mfma16<F16>(a[st / TN][h], b[st % TN][h], acc[st / TN][st % TN]);
            if constexpr (decltype(reads_c)::value && st < TM + TN) rd(s_c, slot, hr_c);
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    __builtin_amdgcn_s_barrier();  // B(0): tile 0 landed
    static_for<0, TM + TN>([&](auto r_c) { rd(r_c, 0, H0{}); });
    lds_wait_all();
    using RD = std::true_type;
    for (int kt = 0; kt < nk - 1; ++kt) {
        half(H0{}, kt % NS, H1{}, RD{});
        lds_wait_all();
        __builtin_amdgcn_s_barrier();  // B(kt+1): tile kt+1 landed; slot kt is read
        half(H1{}, (kt + 1) % NS, H0{}, RD{});
        lds_wait_all();
    }
    half(H0{}, (nk - 1) % NS, H1{}, RD{});  // the last k-tile (no B(nk))
    lds_wait_all();
    half(H1{}, 0, H0{}, std::false_type{});
    if constexpr (EPI == EPI_QKV_PREP)
        qkv_prep_head<BM, 8, NS * STAGE>(p, m0, n0 >> 7, tid, smem, [&](float* tile, int c0, int CH) {
            const int ccol = lane & 15, crow = (lane >> 4) * 4;
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
    else
        gemm_epilogue<TM, TN, F16, EPI, 64>(p, acc, m0 + wm0, n0 + wn0, lane);
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
// SK: split-K instance (variants 210 / 211: p.ksplit = 2 blocks per tile over the two halves of K, splitk_join).  Built
// for the N = 2048 projections at M = 3000 (16 x 8 tiles of 192 x 256 = one round of 256 blocks with two K parts) and
// measured slower there (tools/sk8_bench.py, profiles/r05/sk8/: o 577 against 834 TFLOP/s for the 96x128 pick, down 838
// against 947): with one block per CU and 16 k-tiles per part the prologue, the join and the epilogue are exposed.
// Forced-only.
template <int BM, bool F16, int EPI, bool SK = false>
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
    int m0, n0, sk_tile = 0, sk_part = 0;
    unsigned ticket0 = 0;  // thread 0's split-K ticket
    const int S = SK ? p.ksplit : 1;
    if constexpr (SK) {
        int ntiles;
        splitk_block(S, sk_tile, sk_part, ntiles);
        block_tile<BM, BN>(p, m0, n0, sk_tile, ntiles);
        if (tid == 0) ticket0 = __hip_atomic_fetch_add(p.sk_cnt + sk_tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        block_tile<BM, BN>(p, m0, n0);
    }
    const int M = p.M;
    const int nk_all = p.K / BK;
    const int kt_begin = sk_part * nk_all / S;  // this block's K-tiles [kt_begin, kt_end)
    const int nk = (sk_part + 1) * nk_all / S - kt_begin;

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
            srcA[h][j] = p.A + (int64_t)ra * p.lda + pch * 8 + kt_begin * BK;
            srcB[h][j] = p.W + (int64_t)(n0 + h * 128 + j * 64 + prow) * p.ldw + pch * 8 + kt_begin * BK;
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
        mfma_war_retire(a, b);
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
        if (!(kAblate & 2) || kt == 0) {
            read_a(buf, 0, a);
            read_b(buf, 0, b0);
        }
        if (!(kAblate & 1)) stage_b(1, kt + 1);
        wait_stages();
        seg();
        lds_wait_all();
        mma(a, b0, acc[0][0]);
        seg();
        // ph2
        if (!(kAblate & 2) || kt == 0) read_b(buf, 1, b1);
        if (!(kAblate & 1)) stage_a(1, kt + 1);
        wait_stages();
        seg();
        lds_wait_all();
        mma(a, b1, acc[0][1]);
        seg();
        // ph3: ph4 reads nothing, so no stage has to retire here (a wait here measured neutral)
        if (!(kAblate & 2) || kt == 0) read_a(buf, 1, a);
        if (!(kAblate & 1)) stage_a(0, kt + 2);
        seg();
        lds_wait_all();
        mma(a, b1, acc[1][1]);
        seg();
        // ph4
        if (!(kAblate & 1)) stage_b(0, kt + 2);
        wait_stages();
        seg();
        __builtin_amdgcn_sched_barrier(0);
        mma(a, b0, acc[1][0]);
        seg();
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // both groups now at the same barrier count
    wait_vmcnt<0>();                            // the scratch-region stages of the last tiles
    if constexpr (SK) {
        // acc[2][2][QM][QN] is the 4 QM x QN accumulator grid the join moves in the MFMA register layout
        auto& acc2 = reinterpret_cast<f32x4 (&)[4 * QM][QN]>(acc);
        if (!splitk_join<4 * QM, QN, 8, SplitKMax<BM, BN>::value, 2 * STAGE + 16 * 1024>(p, acc2, S, sk_tile, sk_part, tid,
                                                                                        smem, ticket0))
            return;
    }

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

// split-K workspace of one (device, stream): partial tiles + per-tile ticket / ready counters (zeroed once;
// each launch leaves them zero, see splitk_join).  Launches on one stream are ordered, so one set per stream
// suffices; keyed by the device too, since the null stream has the same handle on every device.  It only grows
// (a grow waits for the stream before freeing the old buffers) and is freed by gemm_splitk_release when the
// owning context destroys its stream.  The join's timeout error word is per device, in pinned host memory:
// gemm_splitk_check reads it without touching any stream (no sync of another context's, possibly destroyed,
// stream) and clears it once reported.
struct SplitKWs {
    void* ws = nullptr;
    size_t ws_bytes = 0;
    unsigned* cnt = nullptr;  // [2][tiles] tickets, ready counts
    size_t tiles = 0;
};
std::mutex g_sk_mu;
std::map<std::pair<int, hipStream_t>, SplitKWs> g_sk;
std::map<int, unsigned*> g_sk_err;  // per device: host-pinned, device-mapped error word

unsigned* splitk_err_word(int dev) {  // (g_sk_mu held)
    unsigned*& e = g_sk_err[dev];
    if (!e) {
        ACEMI_HIP(hipHostMalloc(reinterpret_cast<void**>(&e), sizeof(unsigned), hipHostMallocMapped));
        *reinterpret_cast<volatile unsigned*>(e) = 0u;
    }
    return e;
}

void splitk_setup(GemmParams& p, int ntiles, int S, size_t tile_bytes, hipStream_t s) {
    int dev = 0;
    ACEMI_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_sk_mu);
    SplitKWs& w = g_sk[std::make_pair(dev, s)];
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
    unsigned* err = splitk_err_word(dev);
    unsigned* err_dev = nullptr;
    ACEMI_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev), err, 0));
    p.ksplit = S;
    p.sk_ws = static_cast<f32x4*>(w.ws);
    p.sk_cnt = w.cnt;
    p.sk_ready = w.cnt + w.tiles;
    p.sk_err = err_dev;
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
    } else if constexpr (WM * WN == 4 && PIPE >= 1) {  // split-K instances: the 4-wave pipelined tiles
        if (S > 1)
            hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, F16, EPI, PIPE, true>), grid, block, 0, s, p);
        else
            hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, F16, EPI, PIPE>), grid, block, 0, s, p);
    } else {
        if (S > 1) throw std::runtime_error("gemm: split-K is for the 4-wave pipelined tiles");
        hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, F16, EPI, PIPE>), grid, block, 0, s, p);
    }
}

template <int BM, int BN, bool F16, int EPI, int NS>
void launch_ws(const GemmParams& p, hipStream_t s) {
    if (p.N % BN != 0) throw std::runtime_error("gemm: the warp-specialized tile needs N % BN == 0");
    if constexpr (EPI == EPI_QKV_PREP && BN != 128) {
        throw std::runtime_error("gemm: the fused attention prep needs 128-wide column tiles");
    } else {
        const int nbm = (p.M + BM - 1) / BM;
        hipLaunchKernelGGL((gemm_ws_kernel<BM, BN, F16, EPI, NS>), dim3(nbm * (p.N / BN)), dim3(512), 0, s, p);
    }
}

template <int BM, bool F16, int EPI>
void launch_cfg8(GemmParams p, int S, hipStream_t s) {
    if (p.N % 256 != 0) throw std::runtime_error("gemm: the 8-wave tiles need N % 256 == 0");
    const int nbm = (p.M + BM - 1) / BM;
    if (S > 1) {
        if (S != 2) throw std::runtime_error("gemm: the ping-pong tiles split K over two parts only");
        if (p.K / 64 < 2 * S) throw std::runtime_error("gemm: split-K needs at least two K-tiles per part");
        splitk_setup(p, nbm * (p.N / 256), S, (size_t)BM * 256 * 4, s);
        hipLaunchKernelGGL((gemm8_kernel<BM, F16, EPI, true>), dim3(nbm * (p.N / 256) * S), dim3(512), 0, s, p);
        return;
    }
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
    if (S > 1 && variant % 100 == 18) throw std::runtime_error("gemm: split-K is not built for the warp-specialized tile");
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
        case 10: launch_cfg8<256, F16, EPI>(p, S, s); break;
        case 11: launch_cfg8<192, F16, EPI>(p, S, s); break;
        case 12: launch_cfg<64, 64, 2, 2, F16, EPI, 4>(p, S, s); break;
        case 13: launch_cfg<64, 128, 2, 2, F16, EPI, 3>(p, S, s); break;
        case 14: launch_cfg<96, 128, 2, 2, F16, EPI, 3>(p, S, s); break;
        case 15: launch_cfg<128, 128, 2, 2, F16, EPI, 3>(p, S, s); break;
        // 8 waves (4 x 2) on a 192x128 tile: one tile per CU at M = 3000, N = 2048 (256 tiles), two waves per SIMD
        case 16: launch_cfg<192, 128, 4, 2, F16, EPI, 1>(p, S, s); break;
        // warp-specialized (4 MFMA + 4 loader waves) 192x128, three k-tiles in the ring (forced only: +18 % isolated at
        // the K = 6144 down projection, neutral in the sampling loop; a 3-stage single-role 192x128 tile (0.7x) and a
        // 4-slot ring (equal or slower) measured in round 4 are not built)
        case 18: launch_ws<192, 128, F16, EPI, 3>(p, s); break;
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


}  // namespace gemm_detail

namespace {
using namespace gemm_detail;

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

// Quantized weights: the LDS-staged dequant kernel (gemm_qr_kernel, variants 20-24 [+ 100 S]); the round-1
// ds_write dequant kernel (gemm_q_kernel, 0-7) only when forced.  Long sequences: 192-row tiles (8 waves where
// N % 256 == 0 leaves a full round of 256-column tiles); short ones: 128 / 64-row tiles, split over K until
// the grid covers the 256 CUs.
int pick_variant_q(int M, int N, int K, int fmt) {
    const int64_t mb192 = (M + 191) / 192;
    (void)fmt;
    if (M > 1024) {
        // M = 3000 (tools/wsq_bench.py, profiles/r05/wsq/): gate|up / qkv on the 8-wave register-dequant tile (21),
        // the N = 2048 projections on the warp-specialized tile (25: the expansion on loader waves; down 662 vs 539,
        // o 560 vs 451 TFLOP/s for the 4-wave register-dequant tile)
        if (N > 2048 && N % 256 == 0 && mb192 * (N / 256) >= 256) return 21;
        return 25;
    }
    // Short sequences: round 1's LDS-dequant kernel (96 x 128).  Whole forwards through the 64 / 128-row
    // register-dequant tiles (22, 23, split or not) were not run-to-run identical (tools/diag_det.py, round 3;
    // every kernel-level test of them passes, the attention-prep epilogue is the one path those tests do not
    // reach) -- forced only.
    (void)K;
    return 7;
}

// Per-shape overrides for in-loop A/B runs (ACE_MI_GEMM_OVERRIDE, read by the self-test library only:
// runtime/test_hooks.cpp): the isolated-GEMM sweeps mispredicted the sampling loop at some shapes (cold weights,
// fresh activations), so tile picks are confirmed with whole bench lines.
static int gemm_override(int N, int K) { return gemm_override_from_env(N, K); }

int pick_variant(int M, int N, int K, bool quant, int fmt) {
    auto supports = [&](int v) {  // the tile / split-K factor handles this shape (and weight format)
        const int f = v % 100, S = v / 100;
        const bool wide = f == 2 || f == 5 || f == 10 || f == 11 || f == 21;  // (12-15: multi-stage rings)
        const bool qr = f >= 20 && f <= 25;
        const bool dense_only = (f == 6 || (f >= 8 && f < 20) || S > 1) && !qr;
        const bool sk_ok = S <= 1 || (qr ? (f == 22 || f == 23) && S <= 4 && K / 64 >= 2 * S
                                         : ((f == 1 || f == 3 || f == 4 || f == 10 || f == 11
                                                 ? S <= 2
                                                 : (((f >= 6 && f <= 9) || (f >= 12 && f <= 15)) && S <= 4)) &&
                                            K / 64 >= 2 * S));
        (void)fmt;
        return !(wide && N % 256 != 0) && !(quant && dense_only) && !(!quant && qr) && sk_ok;
    };
    if (g_forced_variant >= 0x10000) return g_forced_variant & 0xffff;  // diagnostics (selftest): no support check
    if (g_forced_variant >= 0 && supports(g_forced_variant)) return g_forced_variant;  // tests / micro-benchmarks
    if (!quant) {
        const int ov = gemm_override(N, K);
        if (ov >= 0 && supports(ov)) return ov;
    }
    const int64_t mb192 = (M + 191) / 192;
    const bool edge_ok = m_edge(M, 192) >= m_edge(M, 128) - 0.02;
    if (quant) return pick_variant_q(M, N, K, fmt);
    // (a skinny weight-stream kernel for M <= 128 ran the 10 s block linears 2x slower than the tiles below --
    // every 16-column workgroup re-read all of A with 16-byte row-scattered loads -- and was removed in round 4)
    // 8-wave ping-pong tiles for batched sequences (tools/gemm_msweep.py on MI355X, TFLOP/s): M = 12000 gate|up
    // 1011 (256x256) vs 941 (v2), qkv 933 vs 902, down 922 (192x256) vs 818, o 814 vs 786; M = 24000 gate|up
    // 1089 vs 1016, qkv 941 vs 897, down 955 vs 915, o 767 (v2) vs 724; M = 6000 down 921 (192x256) vs 853.
    // At M = 3000 the 4-wave tiles stay ahead (their second block per CU hides prologue and epilogue).
    // narrow outputs (proj_out: N = 128 at M = 3000 -- 16 tiles of 192 rows on a 256-CU chip, 28 TFLOP/s):
    // 64x64 tiles (94 workgroups).  Not split over K: the summation order then stays the one every other tile
    // (and the dequant-fused kernels) uses, which the staged == fused test relies on
    if (N <= 128 && M >= 512) return 9;
    // 600 s single sequences (M = 7500) and similar, 6800 <= M < 8192: the 256x256 ping-pong tiles (one round of
    // 240 tiles for the N = 2048 projections) and the 8-wave 192x128 tiles for qkv.  Measured in the sampling loop
    // (bench.py --seconds 600, same-box A/B against the previous picks, profiles/r03_pick_ab_600s/): 29.75 -> 33.25
    // steps/s.  The isolated-GEMM sweep (profiles/r03_msweep_v16_*.jsonl) also favoured the 192x128 8-wave tiles at
    // M = 4500..12000, but inside the loop (cold weights, fresh activations) they were neutral at M = 6000 and 2 %
    // slower at M = 12000 (profiles/r03_bs_ab/), so the picks below 6800 and from 8192 stay as they were.
    if (M >= 6800 && M < 8192) {
        if (N <= 2048 && N % 256 == 0) return 10;
        // qkv (N = 4096) on the 192x256 ping-pong tile with the fused prep: 26.94 steps/s at 600 s against 26.43-26.59
        // for the 8-wave 192x128 tile (profiles/r05/pick_inloop_600s/); o / down / gate|up stay (192x256: 25.2 / 25.3 / 26.2)
        if (N == 4096 && N % 256 == 0) return 11;
        if (N <= 4096) return 16;
        if (N % 256 == 0) return 10;
    }
    if (N % 256 == 0 && M >= 8192) {
        if (N >= 4096) return 10;
        // (M = 24000, eight 240 s items: o / cross q / cross o on the ping-pong 256x256 tile 83.7 item-steps/s against
        //  80.9-81.0 for the 4-wave-family 256x256 and 82.9 for 192x256, profiles/r05/pick_inloop_bs8/)
        if (M >= 20000) return 10;
        return 11;
    }
    // two 240 s items (M = 6000): the ping-pong tiles, measured as whole bs = 2 lines through ACE_MI_GEMM_OVERRIDE
    // (profiles/r05/pick_inloop_bs2/, item-steps/s): gate|up on 256x256 (1152 tiles, 4.5 rounds) 76.1 against 72.2-72.5
    // for the 192x128 4-wave pick (192x256 75.3, 256x256 4-wave-family 73.8); then, with that pick, o / cross q / cross o
    // (N = K = 2048, 256 tiles: one round) on 192x256 78.8 against 76.0-76.5 (256x256 76.9, 256x128 72.1) and qkv on
    // 192x256 77.5 (256x256 75.9); the K = 6144 down projection stays on 192x256 (256x256 71.8, 8-wave 192x128 72.3)
    if (N % 256 == 0 && M >= 5000 && M < 6800) return N >= 8192 ? 10 : 11;
    if (N % 256 == 0 && M >= 4500 && N <= 2048 && K >= 4096) return 11;
    if (edge_ok && mb192 * (N / 128) >= 384) return 4;
    // short sequences (60 s: M = 750): too few 96-row tiles to cover the CUs -> 64-row tiles, and
    // 64x64 when even those leave CUs idle (M = 750: N = 2048 projections 273-337 -> 364-453 TFLOP/s,
    // qkv 519 -> 567, tools/gemm_small_m.py)
    // split-K (tools/gemm_msweep.py, MI355X): only the K = 6144 down projection between the short and the
    // full-length tiles gains (M = 1500: 96x128 over 2 parts 722 vs 637 TFLOP/s for 64x128); elsewhere the
    // join's device-coherent partial round trip (~3-4 us after the main loop) costs more than the fuller grid
    // (and at 60 s, M = 750: 163.4 steps/s against 158.5-159.4 for the 64x128 3-stage split-K pick,
    //  profiles/r05/pick_inloop_60s/)
    if (N <= 2048 && K >= 4096 && M >= 600 && M < 2000) return 207;
    const int64_t mb96 = (M + 95) / 96, mb64 = (M + 63) / 64;
    // Short sequences read every weight cold (each layer's weights were last touched one step earlier), so the
    // picks below follow the cold-weight sweep (ACE_MI_BENCH_COLD=24, profiles/r03_msweep_cold_ns.jsonl), where
    // the multi-stage rings keep more weight tiles in flight:
    //  10 s (M = 125): gate|up 64x128 3-stage (296 vs 267 TFLOP/s for 64x64), qkv / o 64x64 4-stage (146 vs 114,
    //  76 vs 74), the K = 6144 down 64x64 4-stage over 2 K parts (126 vs 69);
    //  60 s (M = 750): qkv 96x128 (495 vs 433 for 64x128), down 64x128 3-stage over 2 K parts (387 vs 349)
    if (M <= 256) {
        if (K >= 4096) return 212;
        return N >= 8192 ? 13 : 12;
    }
    if (K >= 4096 && mb96 * (N / 128) <= 256 && mb64 * (N / 128) < 256) return 213;
    if (mb96 * (N / 128) <= 256) {
        if (mb96 * (N / 128) == 256) return 7;  // one full round of 96-row tiles (60 s qkv)
        return mb64 * (N / 128) >= 256 ? 8 : 9;
    }
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
    int v = pick_variant(M, N, K, weight_quantized(W.fmt), W.fmt);
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
        if (v >= 100 && g_forced_variant < 0) v %= 100;  // (the narrow-output split-K pick is not for the prep)
        v = v == 2 ? 3 : v == 5 ? 4 : v == 6 ? 1 : v == 9 ? 8 : v == 12 ? 13 : v;
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
            dispatch_quant(WF_Q8_0, v, p, s);
            break;
        case WF_Q4_K:
            ACEMI_CHECK(W.s != nullptr, "gemm: null scales");
            dispatch_quant(WF_Q4_K, v, p, s);
            break;
        case WF_Q6_K:
            ACEMI_CHECK(W.s != nullptr, "gemm: null scales");
            dispatch_quant(WF_Q6_K, v, p, s);
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

void gemm_splitk_check() {
    std::lock_guard<std::mutex> lk(g_sk_mu);
    int cur = 0;
    ACEMI_HIP(hipGetDevice(&cur));
    auto it = g_sk_err.find(cur);
    if (it == g_sk_err.end() || !it->second) return;
    volatile unsigned* e = it->second;
    if (*e) {
        *e = 0u;  // reported once: later calls start clean
        throw std::runtime_error("gemm: a split-K join timed out waiting for its partial tiles (results invalid)");
    }
}

void gemm_splitk_release(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_sk_mu);
    int cur = 0;
    ACEMI_HIP(hipGetDevice(&cur));
    auto it = g_sk.find(std::make_pair(cur, s));
    if (it == g_sk.end()) {
        g_sk[std::make_pair(cur, s)] = SplitKWs{};
        it = g_sk.find(std::make_pair(cur, s));
    }
    (void)hipStreamSynchronize(s);  // the stream is still alive here: its last joins are done with the buffers
    if (it->second.ws) (void)hipFree(it->second.ws);
    if (it->second.cnt) (void)hipFree(it->second.cnt);
    g_sk.erase(it);
}

}  // namespace acemi
