// Quantized-weight GEMMs for the DiT block linears (gfx950): the register-dequant kernel (the default for
// Q8_0 / Q4_K / Q6_K weights), round 1's LDS-dequant kernel (forced variants only) and the staged dequant
// (the bf16 image of a quantized matrix, ACE_MI_QUANT_STAGED=1).  Weight planes: runtime/quant.h; the
// dequant arithmetic is ggml's (dequantize_row_q8_0 / _q4_K / _q6_K: one f32 product, RNE to bf16).
#include "gemm_common.h"

namespace acemi {
namespace gemm_detail {

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
        mfma_war_retire(a, b);
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

// ---------------------------------------------------------------------------------------------
// Quantized-weight GEMM with both operands staged through LDS by LDS-DMA (the quantized default): the
// BM x 64 activation k-tile (bf16, the dense kernels' swizzled image) AND the BN x 64 weight k-tile as its raw
// ggml-format bytes + f32 scale planes (runtime/quant.h: 1.0625 B per Q8_0 weight, 0.5625 B Q4_K, 1.125 B
// Q6_K) land in a 3-slot LDS ring; NW waves side by side along N, each owning 32 columns (two 16-wide MFMA
// column tiles) and ALL BM rows, read their B fragments' bytes from LDS and form the bf16 fragments in
// registers with the staged dequant's arithmetic (deq_i8x4 / deq_u4x4: one f32 product, RNE to bf16) -- so the
// MFMA operands and the per-element k order equal the staged dequant + dense GEMM bit for bit, no bf16 image
// exists, and each weight is expanded once per block and reused by TM = BM / 16 MFMAs.  Every LDS write is an
// LDS-DMA (no ds_write: the DMA / ds_write hazard of DESIGN.md §10 cannot arise) and the per-wave DMA count per
// k-tile is a compile-time constant, so one counted vmcnt per k-tile retires exactly the tile being consumed
// while the next stays in flight (a register-held weight prefetch made hipcc drain every load, vmcnt(0), at
// each k-tile: 0.62 of the dense kernel's rate).
// Pipeline (RS ring slots, RS = 4 where the LDS fits them, else 3): a tile is READ one barrier after the counted
// vmcnt that retires it, never right behind that wait.  Per k-tile t: vmcnt retires tile t+1 [tiles up to t+RS-2 stay
// in flight], barrier, stage tile t+RS-1 into the slot last read at t-1, then read tile t (retired by the previous
// iteration's wait, so at least one barrier and a whole MFMA phase lie between its retiring wait and these reads):
// B bytes -> registers -> bf16 fragments, then per kk: A fragments from LDS, TM x 2 MFMAs.
// Why not read right behind the wait (rounds 2-4's schedule): on gfx950 a wave's counted vmcnt can be satisfied
// before its own LDS-DMA bytes are visible to ds_read -- the wave that arrives last at the barrier and then reads a
// piece it staged itself saw the slot's previous contents (variant 21 x Q4_K, whose q rows are the only ones a wave
// both stages and reads: whole 16-column groups of waves 4-7 wrong on some launches; the 64-row tiles, whose MFMA
// phase is the shortest, not run-to-run identical in whole forwards; DESIGN.md §10, the guide's "read a staged buffer
// one phase AFTER the wait that retires it").
template <int WQ>
struct QTile {  // bytes of one weight row per 64-wide k-tile (q plane, scale plane)
    static constexpr int QB = WQ == WF_Q4_K ? 32 : 64;
    static constexpr int SB = WQ == WF_Q8_0 ? 8 : 16;
};

template <int OFF>
__device__ __forceinline__ uint2 ds_read_b64_off(uint32_t addr) {
    uint2 v;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return v;
}
template <int OFF>
__device__ __forceinline__ uint32_t ds_read_b32_off(uint32_t addr) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
    return v;
}

// this lane's B fragment bytes (columns wn0 + j*16 + (lane & 15), k group g = lane >> 4) of the k-tile in the slot at
// LDS byte address wq (q rows) / ws (scale rows): qd_read issues the LDS reads (the caller waits), qd_dequant forms
// the bf16 fragments of one k half kk
struct QRaw {
    uint32_t q[2][2][2];  // [j][kk] 8 bytes (Q8_0 / Q6_K) or 4 bytes in [..][0] (Q4_K)
    uint4 sc[2];          // [j] scales: Q8_0 (s_kk0, s_kk1, -, -); Q4_K (d0, m0, d1, m1); Q6_K (4 x d*sc per 16)
};

template <int WQ>
__device__ __forceinline__ void qd_read(uint32_t wq, uint32_t ws, int row, int g, QRaw& r) {
    constexpr int QB = QTile<WQ>::QB, SB = QTile<WQ>::SB;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t qa = wq + (row + j * 16) * QB, sa = ws + (row + j * 16) * SB;
        if constexpr (WQ == WF_Q4_K) {
            r.q[j][0][0] = ds_read_b32_off<0>(qa + g * 4);
            r.q[j][1][0] = ds_read_b32_off<16>(qa + g * 4);
            r.sc[j] = ds_read_b128_off<0>(sa);
        } else {
            const uint2 q0 = ds_read_b64_off<0>(qa + g * 8), q1 = ds_read_b64_off<32>(qa + g * 8);
            r.q[j][0][0] = q0.x;
            r.q[j][0][1] = q0.y;
            r.q[j][1][0] = q1.x;
            r.q[j][1][1] = q1.y;
            if constexpr (WQ == WF_Q8_0) {
                const uint2 s2 = ds_read_b64_off<0>(sa);
                r.sc[j] = make_uint4(s2.x, s2.y, 0u, 0u);
            } else {
                r.sc[j] = ds_read_b128_off<0>(sa);
            }
        }
    }
}

template <int WQ>
__device__ __forceinline__ void qd_dequant(const QRaw& r, int g, int kk, uint4 (&b)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const float s[4] = {__uint_as_float(r.sc[j].x), __uint_as_float(r.sc[j].y), __uint_as_float(r.sc[j].z),
                            __uint_as_float(r.sc[j].w)};
        uint32_t o[4];
        if constexpr (WQ == WF_Q4_K) {
            const uint32_t w = r.q[j][kk][0];
            const float d = s[2 * kk], nm = -s[2 * kk + 1];
            deq_u4x4(w & 0x0f0f0f0fu, d, nm, o[0], o[1]);
            deq_u4x4((w >> 4) & 0x0f0f0f0fu, d, nm, o[2], o[3]);
        } else {
            // Q8_0: one scale per 32 (block kk); Q6_K: one per 16 (k group g covers 16-half g >> 1)
            const float d = WQ == WF_Q8_0 ? s[kk] : s[2 * kk + (g >> 1)];
            deq_i8x4(r.q[j][kk][0], d, -128.0f * d, o[0], o[1]);
            deq_i8x4(r.q[j][kk][1], d, -128.0f * d, o[2], o[3]);
        }
        b[j][kk] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

#ifdef ACEMI_QR_DIAG
// Diagnostic build only (tools/build_ab.sh ... -DACEMI_QR_DIAG): every lane's raw LDS reads of every k-tile (q words and
// scales as first read, then the same LDS words re-read after the tile's MFMAs), to tell a late-landing DMA from a wrong one.
__device__ uint32_t g_qr_dbg[1 << 22];
#endif

template <int BM, int NW, int WQ>
struct QRing {
    static constexpr int SLOT = BM * 128 + 32 * NW * (QTile<WQ>::QB + QTile<WQ>::SB);
#ifdef ACEMI_QR_RING3  // A/B build: the 3-slot ring everywhere
    static constexpr int RS = 3;
#else
    static constexpr int RS = 4 * SLOT <= 160 * 1024 ? 4 : 3;  // ring slots
#endif
    static constexpr int BYTES = RS * SLOT;
};

// two workgroups per CU where the ring allows it (not for split-K: its join needs the registers)
template <int BM, int NW, int EPI, int WQ, bool SK = false>
__global__ void __launch_bounds__(NW * 64, (!SK && (NW == 8 || 2 * QRing<BM, NW, WQ>::BYTES <= 160 * 1024)) ? 2 : 1)
    gemm_qr_kernel(GemmParams p) {
    constexpr int BN = 32 * NW;
    constexpr int TM = BM / 16;
    constexpr int TN = 2;
    constexpr int BK = 64;
    constexpr int ROWB = BK * 2;
    constexpr int QB = QTile<WQ>::QB, SB = QTile<WQ>::SB;
    constexpr int A_BYTES = BM * ROWB, WQ_BYTES = BN * QB, WS_BYTES = BN * SB;
    constexpr int SLOT = A_BYTES + WQ_BYTES + WS_BYTES;
    constexpr int RS = QRing<BM, NW, WQ>::RS;
    static_assert(SLOT == QRing<BM, NW, WQ>::SLOT, "ring slot size");
    constexpr int PA = BM / 8;             // 1 KiB pieces (8 rows x 128 B)
    constexpr int PQ = WQ_BYTES / 1024;    // 1 KiB pieces (64 lanes x 16 B)
    constexpr int PS = WS_BYTES / 256;     // 256 B pieces (64 lanes x one f32)
    static_assert(PA % NW == 0 && PQ % NW == 0 && PS % NW == 0, "LDS-DMA pieces must split evenly over the waves");
    constexpr int G = (PA + PQ + PS) / NW;  // LDS-DMA instructions per wave per k-tile
    static_assert(EPI != EPI_SWIGLU || (TN % 2 == 0), "swiglu needs column pairs");

    __shared__ __attribute__((aligned(16))) char smem[RS * SLOT];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;

    const int S = SK ? p.ksplit : 1;
    int m0, n0, sk_tile = 0, sk_part = 0;
    unsigned ticket0 = 0;
    if constexpr (SK) {
        int ntiles;
        splitk_block(S, sk_tile, sk_part, ntiles);
        block_tile<BM, BN>(p, m0, n0, sk_tile, ntiles);
        if (tid == 0) ticket0 = __hip_atomic_fetch_add(p.sk_cnt + sk_tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        block_tile<BM, BN>(p, m0, n0);
    }
    const int wn0 = wid * 32;
    const int M = p.M, K = p.K;
    const int nk_all = K / BK;
    const int kt_begin = sk_part * nk_all / S;
    const int nk = (sk_part + 1) * nk_all / S - kt_begin;

    // LDS-DMA sources, fixed over k (+ kt * k-tile stride): A pieces (swizzled chunk as the dense kernel), W q
    // pieces (QB / 16 lanes per row), W scale pieces (one f32 per lane, SB / 4 per row)
    const uint16_t* srcA[PA / NW];
#pragma unroll
    for (int j = 0; j < PA / NW; ++j) {
        const int row = (wid + NW * j) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ swz(row);
        srcA[j] = p.A + (int64_t)min(m0 + row, M - 1) * p.lda + (int64_t)kt_begin * BK + c * 8;
    }
    const int qrow_bytes = WQ == WF_Q4_K ? K / 2 : K;
    const int srow_floats = WQ == WF_Q8_0 ? K / 32 : K / 16;
    const char* srcQ[PQ / NW];
#pragma unroll
    for (int j = 0; j < PQ / NW; ++j) {
        constexpr int LPR = QB / 16;  // lanes per row
        const int e = (wid + NW * j) * 64 + lane;
        srcQ[j] = static_cast<const char*>(p.Wq) + (int64_t)(n0 + e / LPR) * qrow_bytes + (int64_t)kt_begin * QB +
                  (e % LPR) * 16;
    }
    const float* srcS[PS / NW];
#pragma unroll
    for (int j = 0; j < PS / NW; ++j) {
        constexpr int FPR = SB / 4;  // floats per row
        const int e = (wid + NW * j) * 64 + lane;
        srcS[j] = p.Ws + (int64_t)(n0 + e / FPR) * srow_floats + (int64_t)kt_begin * FPR + (e % FPR);
    }
    auto stage = [&](int kt, int slot) {  // k-tile kt (relative) into ring slot `slot`
        char* base = smem + slot * SLOT;
#pragma unroll
        for (int j = 0; j < PA / NW; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + kt * BK), (lds_void*)(base + (wid + NW * j) * 1024),
                                             16, 0, 0);
#pragma unroll
        for (int j = 0; j < PQ / NW; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(srcQ[j] + (int64_t)kt * QB),
                                             (lds_void*)(base + A_BYTES + (wid + NW * j) * 1024), 16, 0, 0);
#pragma unroll
        for (int j = 0; j < PS / NW; ++j)
            __builtin_amdgcn_global_load_lds((const void*)(srcS[j] + kt * (SB / 4)),
                                             (lds_void*)(base + A_BYTES + WQ_BYTES + (wid + NW * j) * 256), 4, 0, 0);
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
    const int lrow = lane & 15, lchunk = lane >> 4;
    const int rsw = (lrow >> 1) & 7;

    // prologue: k-tiles 0 .. RS-2 requested, tile 0 retired + published.  The body is branch-free: past the last k-tile
    // it re-stages the final one into the slot nobody reads again, so every iteration issues the same G DMA
    // instructions per wave and the counted vmcnt at its top always retires exactly tile kt+1.
#pragma unroll
    for (int s = 0; s < RS - 1; ++s) stage(min(s, nk - 1), s);
    wait_vmcnt<G*(RS - 2)>();
    __builtin_amdgcn_s_barrier();
    for (int kt = 0; kt < nk; ++kt) {
        wait_vmcnt<G*(RS - 3)>();      // this wave's pieces of tile kt+1 landed (read next iteration)
        __builtin_amdgcn_s_barrier();  // every wave: tile kt+1 retired, reads of tile kt-1 done -> its slot is free
        stage(min(kt + RS - 1, nk - 1), (kt + RS - 1) % RS);
        // W bytes and the kk = 0 A fragments in one LDS wait; the kk = 1 A reads are issued before the kk = 0
        // MFMAs, and the kk = 1 dequant VALU sits between those MFMAs (no scheduling barrier in between), so the
        // dequant of the second k half overlaps matrix work
        const uint32_t sbase = lds0 + (kt % RS) * SLOT;
        const uint32_t abase = sbase + lrow * ROWB;
        QRaw raw;
        qd_read<WQ>(sbase + A_BYTES, sbase + A_BYTES + WQ_BYTES, wn0 + lrow, lchunk, raw);
        uint4 a0[TM][2], a1[TM][2], b[TN][2];
        ReadRows<0, TM, 16 * ROWB>::run(abase + (((0 * 4 + lchunk) ^ rsw) * 16), a0, 0);
        lds_wait_all();
        qd_dequant<WQ>(raw, lchunk, 0, b);
        mfma_war_guard();  // (read side: the kk = 0 MFMAs read B fragments just written by this VALU)
        ReadRows<0, TM, 16 * ROWB>::run(abase + (((1 * 4 + lchunk) ^ rsw) * 16), a1, 1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<false>(a0[i][0], b[j][0], acc[i][j]);
        mfma_war_guard();  // the kk = 1 dequant below overwrites A / B registers of the MFMAs just issued
        qd_dequant<WQ>(raw, lchunk, 1, b);
        lds_wait_all();
        mfma_war_guard();
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<false>(a1[i][1], b[j][1], acc[i][j]);
        mfma_war_guard();  // the next k-tile's address VALU and LDS reads reuse this tile's operand registers
#ifdef ACEMI_QR_DIAG
        if constexpr (!SK) {
            QRaw raw2;
            qd_read<WQ>(sbase + A_BYTES, sbase + A_BYTES + WQ_BYTES, wn0 + lrow, lchunk, raw2);
            lds_wait_all();
            uint32_t* d = g_qr_dbg + ((size_t)(blockIdx.x * nk + kt) * (NW * 64) + tid) * 24;
            if ((size_t)(blockIdx.x * nk + kt + 1) * (NW * 64) * 24 <= (1u << 22)) {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    d[j * 12 + 0] = raw.q[j][0][0]; d[j * 12 + 1] = raw.q[j][0][1];
                    d[j * 12 + 2] = raw.q[j][1][0]; d[j * 12 + 3] = raw.q[j][1][1];
                    d[j * 12 + 4] = raw.sc[j].x; d[j * 12 + 5] = raw.sc[j].y; d[j * 12 + 6] = raw.sc[j].z; d[j * 12 + 7] = raw.sc[j].w;
                    d[j * 12 + 8] = raw2.q[j][0][0]; d[j * 12 + 9] = raw2.q[j][1][0];
                    d[j * 12 + 10] = raw2.sc[j].x; d[j * 12 + 11] = raw2.sc[j].z;
                }
            }
        }
#endif
    }
    wait_vmcnt<0>();  // the dummy stages past the end land before the epilogue reuses the ring
    __syncthreads();  // LDS reads done before the epilogue reuses the ring

    if constexpr (SK)
        if (!splitk_join<TM, TN, NW, 4, RS * SLOT>(p, acc, S, sk_tile, sk_part, tid, smem, ticket0)) return;
    if constexpr (EPI == EPI_QKV_PREP) {
        // one head per 128 columns: waves [4 hb, 4 hb + 4) hold head (n0 >> 7) + hb
        const int ccol = lane & 15, crow = (lane >> 4) * 4;
#pragma unroll
        for (int hb = 0; hb < BN / 128; ++hb)
            qkv_prep_head<BM, NW, RS * SLOT>(p, m0, (n0 >> 7) + hb, tid, smem, [&](float* tile, int c0, int CH) {
                if ((wn0 >> 7) != hb) return;
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int rb = i * 16 - c0;
                    if (rb < 0 || rb >= CH) continue;
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int j = 0; j < TN; ++j)
                            tile[(rb + crow + r) * PREP_LD + (wn0 & 127) + j * 16 + ccol] = acc[i][j][r];
                }
            });
    } else {
        gemm_epilogue<TM, TN, false, EPI, (SK ? 32 : 64)>(p, acc, m0, n0 + wn0, lane);
    }
}

// ---------------------------------------------------------------------------------------------
// Warp-specialized dequant-fused GEMM (variant 25): the dense warp-specialized tile (gemm.hip gemm_ws_kernel,
// variant 18) with the dequantization moved onto its loader waves.  512 threads: 4 MFMA waves (2 x 2, 96 x 64 each,
// one per SIMD) that only read bf16 fragments from LDS and issue MFMAs -- the same instruction stream as the dense
// tile -- and 4 loader waves that, per k-tile t, (1) stage A(t) (bf16 activations) and the raw ggml-format W(t)
// bytes + f32 scale planes by LDS-DMA into ring slot t % NS, (2) once those landed, expand W(t) with the staged
// dequant's arithmetic (dequant_block: one f32 product, RNE to bf16) into the slot's swizzled bf16 B image, and
// (3) publish the slot at barrier B(t).  So each weight is expanded once per block by a wave that issues no MFMA
// (the VALU work runs beside the MFMA wave of its SIMD instead of in its stream), the MFMA operands and the k order
// are those of staged dequant + the dense kernel (bit-identical results), and no bf16 image exists in HBM.
// Ring: NS slots of (A image | B image) plus NS raw-W buffers; the loaders keep tiles t+1 .. t+NS-1 in flight.  The
// loaders' LDS reads / writes are inline asm (a compiler-visible LDS access beside an in-flight LDS-DMA draws a
// vmcnt(0) from hipcc); each group of B writes is retired (lgkmcnt(0)) inside its own statement, so no later VALU can
// overwrite their data registers before the LDS unit has read them.
template <int WQ>
__device__ __forceinline__ void wsq_read_raw(uint32_t q_addr, uint32_t s_addr, WRaw& r) {
    if constexpr (WQ == WF_Q4_K) {
        u32x4 q;
        uint2 sc;
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b64 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(q), "=&v"(sc) : "v"(q_addr), "v"(s_addr) : "memory");
        r.q0 = q;
        r.s0 = __uint_as_float(sc.x);
        r.s1 = __uint_as_float(sc.y);
    } else {
        u32x4 q0, q1;
        if constexpr (WQ == WF_Q8_0) {
            uint32_t sc;
            asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %3 offset:16\n\tds_read_b32 %2, %4\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(q0), "=&v"(q1), "=&v"(sc) : "v"(q_addr), "v"(s_addr) : "memory");
            r.s0 = __uint_as_float(sc);
            r.s1 = r.s0;
        } else {
            uint2 sc;
            asm volatile("ds_read_b128 %0, %3\n\tds_read_b128 %1, %3 offset:16\n\tds_read_b64 %2, %4\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(q0), "=&v"(q1), "=&v"(sc) : "v"(q_addr), "v"(s_addr) : "memory");
            r.s0 = __uint_as_float(sc.x);
            r.s1 = __uint_as_float(sc.y);
        }
        r.q0 = q0;
        r.q1 = q1;
    }
}

template <int BM, int BN, int EPI, int WQ, int NS>
__global__ void __launch_bounds__(512, 1) gemm_wsq_kernel(GemmParams p) {
    constexpr int NC = 4, WN = 2;  // MFMA waves (2 x 2)
    constexpr int WTM = BM / 2, WTN = BN / WN;
    constexpr int TM = WTM / 16, TN = WTN / 16;
    constexpr int BK = 64, ROWB = BK * 2;
    constexpr int STAGE = (BM + BN) * ROWB;
    constexpr int QB = QTile<WQ>::QB, SB = QTile<WQ>::SB;
    constexpr int RAW = BN * (QB + SB);
    constexpr int GA = BM / 8 / 4;            // A pieces (1 KiB) per loader wave per k-tile
    constexpr int GQ = BN * QB / 1024 / 4;    // q pieces (1 KiB) per loader wave
    constexpr int GS = BN * SB / 256 / 4;     // scale pieces (256 B: one f32 per lane) per loader wave
    constexpr int G = GA + GQ + GS;
    static_assert(BM % 32 == 0 && (BN * QB) % 4096 == 0 && (BN * SB) % 1024 == 0 && BN * 2 == 256, "wsq tile");
    static_assert(NS >= 3 && NS * (STAGE + RAW) <= 160 * 1024, "wsq ring");
    static_assert(EPI != EPI_SWIGLU || (TN % 2 == 0), "swiglu needs column pairs");
    __shared__ __attribute__((aligned(16))) char smem[NS * (STAGE + RAW)];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int m0, n0;
    block_tile<BM, BN>(p, m0, n0);
    const int nk = p.K / BK;
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

    if (wid >= NC) {  // ---- loader wave ----
        const int lw = wid - NC, ltid = tid - NC * 64;
        const uint16_t* srcA[GA];
#pragma unroll
        for (int j = 0; j < GA; ++j) {
            const int row = (lw + 4 * j) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ swz(row);
            srcA[j] = p.A + (int64_t)min(m0 + row, p.M - 1) * p.lda + c * 8;
        }
        const int qrow_bytes = WQ == WF_Q4_K ? p.K / 2 : p.K;
        const int srow_floats = WQ == WF_Q8_0 ? p.K / 32 : p.K / 16;
        // raw W pieces: loader wave lw stages exactly the rows its own lanes expand (rows 32 lw .. 32 lw + 31), so its
        // own counted vmcnt orders its LDS reads of them (no workgroup barrier between staging and dequant)
        const char* srcQ[GQ];
#pragma unroll
        for (int j = 0; j < GQ; ++j) {
            constexpr int LPR = QB / 16;  // lanes per row
            const int e = (lw * GQ + j) * 64 + lane;
            srcQ[j] = static_cast<const char*>(p.Wq) + (int64_t)(n0 + e / LPR) * qrow_bytes + (e % LPR) * 16;
        }
        const float* srcS[GS];
#pragma unroll
        for (int j = 0; j < GS; ++j) {
            constexpr int FPR = SB / 4;  // floats per row
            const int e = (lw * GS + j) * 64 + lane;
            srcS[j] = p.Ws + (int64_t)(n0 + e / FPR) * srow_floats + (e % FPR);
        }
        auto stage = [&](int t) {  // raw W(t) pieces first, then A(t): a counted vmcnt can retire W(t+1) with A(t+1) in flight
            const int slot = t % NS;
            char* base = smem + slot * STAGE;
            char* raw = smem + NS * STAGE + slot * RAW;
#pragma unroll
            for (int j = 0; j < GQ; ++j)
                __builtin_amdgcn_global_load_lds((const void*)(srcQ[j] + (int64_t)t * QB),
                                                 (lds_void*)(raw + (lw * GQ + j) * 1024), 16, 0, 0);
#pragma unroll
            for (int j = 0; j < GS; ++j)
                __builtin_amdgcn_global_load_lds((const void*)(srcS[j] + t * (SB / 4)),
                                                 (lds_void*)(raw + BN * QB + (lw * GS + j) * 256), 4, 0, 0);
#pragma unroll
            for (int j = 0; j < GA; ++j)
                __builtin_amdgcn_global_load_lds((const void*)(srcA[j] + t * BK), (lds_void*)(base + (lw + 4 * j) * 1024), 16,
                                                 0, 0);
        };
        // this lane's 32-value block of W(t): row wr of the tile, k half wh
        const int wr = ltid >> 1, wh = ltid & 1;
        const int wsw = swz(wr);
        constexpr int QOFF = WQ == WF_Q4_K ? 16 : 32;  // q bytes of one 32-value block
        constexpr int SOFF = WQ == WF_Q8_0 ? 4 : 8;    // scale bytes of one 32-value block
        auto dequant = [&](int t, auto&& between) {  // (between: work the compiler may interleave with the VALU)
            const int slot = t % NS;
            const uint32_t raw = lds0 + NS * STAGE + slot * RAW;
            WRaw r;
            wsq_read_raw<WQ>(raw + wr * QB + wh * QOFF, raw + BN * QB + wr * SB + wh * SOFF, r);
            between();  // (LDS-DMA issue the compiler may interleave with the dequant VALU below)
            uint32_t o[16];
            dequant_block<WQ>(r, o);
            const uint32_t row = lds0 + slot * STAGE + (BM + wr) * ROWB;
            const uint32_t c0 = row + (((wh * 4 + 0) ^ wsw) * 16), c1 = row + (((wh * 4 + 1) ^ wsw) * 16);
            const uint32_t c2 = row + (((wh * 4 + 2) ^ wsw) * 16), c3 = row + (((wh * 4 + 3) ^ wsw) * 16);
            const u32x4 d0{o[0], o[1], o[2], o[3]}, d1{o[4], o[5], o[6], o[7]};
            const u32x4 d2{o[8], o[9], o[10], o[11]}, d3{o[12], o[13], o[14], o[15]};
            asm volatile(
                "ds_write_b128 %0, %4\n\tds_write_b128 %1, %5\n\tds_write_b128 %2, %6\n\tds_write_b128 %3, %7\n\t"
                "s_waitcnt lgkmcnt(0)"
                :
                : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "v"(d0), "v"(d1), "v"(d2), "v"(d3)
                : "memory");
        };
        // Raw W(t) is read one barrier after the counted wait that retires it (the guide's rule for LDS-DMA data: a
        // read right behind its own wait gave run-to-run differences in whole Q4_K / Q6_K forwards): the wait before
        // B(j) retires A(j) and W(j+1) (A(j+1) stays in flight), the dequant of W(j+1) runs after B(j).
        static_assert(NS == 3, "the counted waits below assume three ring slots");
#pragma unroll
        for (int t = 0; t < NS; ++t)
            if (t < nk) stage(t);
        if (nk > 2) wait_vmcnt<GA + G>();       // W(0) A(0) W(1) retired; A(1) W(2) A(2) in flight
        else if (nk == 2) wait_vmcnt<GA>();    // (K = 128: only tiles 0, 1 staged) W(0) A(0) W(1) retired; A(1) in flight
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();  // P: (a barrier between W(0)'s retiring wait and its reads)
        auto none = [] {};
        dequant(0, none);
        __builtin_amdgcn_s_barrier();  // B(0): A(0) landed, B image of tile 0 written
        for (int j = 1; j < nk; ++j) {
            dequant(j, none);  // W(j) retired before B(j-1)
            if (j + 1 < nk) wait_vmcnt<GA>();  // A(j), W(j+1) retired; A(j+1) in flight
            else wait_vmcnt<0>();
            __builtin_amdgcn_s_barrier();  // B(j): slot (j-1) % NS read by every MFMA wave
            if (j - 1 + NS < nk) stage(j - 1 + NS);
        }
        wait_vmcnt<0>();
        if constexpr (EPI == EPI_QKV_PREP)
            qkv_prep_head<BM, 8, NS * STAGE>(p, m0, n0 >> 7, tid, smem, [](float*, int, int) {});
        return;
    }

    // ---- MFMA wave (gemm_ws_kernel's) ----
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
    auto rd = [&](auto r_c, int slot, auto h_c) {
        constexpr int r = decltype(r_c)::value, h = decltype(h_c)::value;
        const uint32_t sb = lds0 + slot * STAGE + ch[h];
        if constexpr (r < TN)
            b[r][h] = ds_read_b128_off<r * 16 * ROWB>(sb + (BM + wn0 + lrow) * ROWB);
        else
            a[r - TN][h] = ds_read_b128_off<(r - TN) * 16 * ROWB>(sb + (wm0 + lrow) * ROWB);
    };
    auto half = [&](auto h_c, int slot, auto hr_c, auto reads_c) {
        constexpr int h = decltype(h_c)::value;
        static_for<0, TM * TN>([&](auto s_c) {
            constexpr int st = decltype(s_c)::value;
            acc[st / TN][st % TN] = mfma16<false>(a[st / TN][h], b[st % TN][h], acc[st / TN][st % TN]);
            if constexpr (decltype(reads_c)::value && st < TM + TN) rd(s_c, slot, hr_c);
            __builtin_amdgcn_sched_barrier(0);
        });
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    __builtin_amdgcn_s_barrier();  // P
    __builtin_amdgcn_s_barrier();  // B(0): tile 0 published
    static_for<0, TM + TN>([&](auto r_c) { rd(r_c, 0, H0{}); });
    lds_wait_all();
    using RD = std::true_type;
    for (int kt = 0; kt < nk - 1; ++kt) {
        half(H0{}, kt % NS, H1{}, RD{});
        lds_wait_all();
        __builtin_amdgcn_s_barrier();  // B(kt+1): tile kt+1 published; slot kt is read
        half(H1{}, (kt + 1) % NS, H0{}, RD{});
        lds_wait_all();
    }
    half(H0{}, (nk - 1) % NS, H1{}, RD{});  // the last k-tile (no B(nk))
    lds_wait_all();
    half(H1{}, 0, H0{}, std::false_type{});
    mfma_war_guard();
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
        gemm_epilogue<TM, TN, false, EPI, 64>(p, acc, m0 + wm0, n0 + wn0, lane);
}

template <int BM, int BN, int EPI, int WQ, int NS>
void launch_wsq_cfg(const GemmParams& p, hipStream_t s) {
    if (p.N % BN != 0) throw std::runtime_error("gemm: the warp-specialized quantized tile needs N % 128 == 0");
    if constexpr (EPI == EPI_QKV_PREP && BN != 128) {
        throw std::runtime_error("gemm: the fused attention prep needs 128-wide column tiles");
    } else {
        const int nbm = (p.M + BM - 1) / BM;
        hipLaunchKernelGGL((gemm_wsq_kernel<BM, BN, EPI, WQ, NS>), dim3(nbm * (p.N / BN)), dim3(512), 0, s, p);
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

// LDS-dequant kernel (gemm_qr_kernel): BM x (32 NW) tiles, split-K over S blocks per tile for the short ones
template <int BM, int NW, int EPI, int WQ>
void launch_qr_cfg(GemmParams p, int S, hipStream_t s) {
    constexpr int BN = 32 * NW;
    if (p.N % BN != 0) throw std::runtime_error("gemm: quantized tile needs N % (32 * waves) == 0");
    const int nbm = (p.M + BM - 1) / BM;
    const int nbn = p.N / BN;
    if (S > 1) {
        if constexpr (BM <= 128 && NW == 4) {
            if (p.K / 64 < 2 * S || S > 4) throw std::runtime_error("gemm: bad split-K factor");
            splitk_setup(p, nbm * nbn, S, (size_t)BM * BN * 4, s);
            hipLaunchKernelGGL((gemm_qr_kernel<BM, NW, EPI, WQ, true>), dim3(nbm * nbn * S), dim3(NW * 64), 0, s, p);
        } else {
            throw std::runtime_error("gemm: split-K is for the 64 / 128-row quantized tiles");
        }
    } else {
        hipLaunchKernelGGL((gemm_qr_kernel<BM, NW, EPI, WQ>), dim3(nbm * nbn), dim3(NW * 64), 0, s, p);
    }
}

template <int EPI, int WQ>
void launch_q_variant(int variant, const GemmParams& p, hipStream_t s) {
    const int S = variant / 100;
    switch (variant % 100) {
        case 20: launch_qr_cfg<192, 4, EPI, WQ>(p, S, s); return;
        case 21: launch_qr_cfg<192, 8, EPI, WQ>(p, S, s); return;
        case 22: launch_qr_cfg<128, 4, EPI, WQ>(p, S, s); return;
        case 23: launch_qr_cfg<64, 4, EPI, WQ>(p, S, s); return;
        case 24: launch_qr_cfg<256, 4, EPI, WQ>(p, S, s); return;
        case 25:
            if (S > 1) throw std::runtime_error("gemm: no split-K for the warp-specialized quantized tile");
            launch_wsq_cfg<192, 128, EPI, WQ, 3>(p, s);
            return;
        default: break;
    }
    if (S > 1) throw std::runtime_error("gemm: split-K is for the register-dequant tiles");
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


void dispatch_quant(int fmt, int variant, const GemmParams& p, hipStream_t s) {
    switch (fmt) {
        case WF_Q8_0: dispatch_q_epi<WF_Q8_0>(variant, p, s); break;
        case WF_Q4_K: dispatch_q_epi<WF_Q4_K>(variant, p, s); break;
        case WF_Q6_K: dispatch_q_epi<WF_Q6_K>(variant, p, s); break;
        default: throw std::runtime_error("gemm: bad quantized weight format");
    }
}

}  // namespace gemm_detail

using namespace gemm_detail;

#ifdef ACEMI_QR_DIAG
extern "C" __attribute__((visibility("default"))) int ace_mi_qr_diag_read(uint32_t* out, size_t n_words, int clear) {
    if (n_words > (1u << 22)) return 2;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(gemm_detail::g_qr_dbg), n_words * 4, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    if (clear) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(gemm_detail::g_qr_dbg)) != hipSuccess || hipMemset(p, 0xff, (1u << 22) * 4) != hipSuccess)
            return 1;
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
#endif

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
