// Oobleck VAE decoder kernels (gfx950): the conv stack of ace_vae::forward_decode
// (acestep_ggml/cpp/acestep_vae_model.cpp:682-742,957-1002) as implicit-GEMM fp16 MFMA.
//
// ggml runs every decoder conv as F16 x F16 with f32 accumulation (im2col to F16 for
// ggml_conv_1d; the F16 kernel and an F16 copy of the input for ggml_conv_transpose_1d), so
// v_mfma_f32_16x16x32_f16 reproduces its arithmetic: exact products, f32 sums.
//
// Layout: activations time-major [T][C] (channel-contiguous rows).  A conv with taps k and
// dilation d is a GEMM over K = taps*Cin whose A row for output t and tap k is the input row
// t + k*d - pad (a shifted view, or a zero row at the edges), staged into LDS by LDS-DMA exactly
// like the DiT GEMM.  A ConvTranspose1d with kernel 2s, stride s is ONE GEMM too: output time
// u = s*j + r takes input rows j (kernel tap r) and j-1 (tap r+s), so with N = s*Cout columns
// (r, co) the GEMM's row-major output IS the [T_out][Cout] layout, shifted by the center crop.
// Epilogues fuse what follows each conv in the graph: bias, the residual add, the f32 store of
// the running activation, and the NEXT Snake (x + sin^2(e^a x)/e^b, f32) written as the fp16
// operand of the next conv.
#include <cmath>
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "../kernels.h"
#include "lds_asm.h"
#include "prep_math.h"
#include "mfma_guard.h"

namespace acemi {
namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ int swz(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ uint16_t f32_to_f16(float f) {
    _Float16 h = (_Float16)f;
    return __builtin_bit_cast(uint16_t, h);
}

// snake_forward (:682-692) with ea = exp(alpha), eb = exp(beta) precomputed on the host (expf).
// The hardware sine (v_sin_f32) and a reciprocal-multiply divide: the epilogue runs this for every
// output element, and the IEEE sinf / division sequences cost ~50 VALU instructions per element --
// more than the tile's MFMAs at 128 channels.  Their results differ from libm's by ~1e-6 relative,
// far below the fp16 rounding of the next conv's operand that follows.
__device__ __forceinline__ float snake_f(float x, float ea, float rcp_eb) {
    float s = __sinf(rn_mul(ea, x));
    s = rn_mul(s, s);
    s = rn_mul(s, rcp_eb);  // / e^beta as a multiply by the (1-ulp) hardware reciprocal
    return rn_add(x, s);
}

template <int I, int N, int STRIDE>
struct ReadRows {
    __device__ __forceinline__ static void run(uint32_t base, uint4 (&dst)[N][2], int kk) {
        if (kk == 0)
            dst[I][0] = ds_read_b128_at<I * STRIDE>(base);
        else
            dst[I][1] = ds_read_b128_at<I * STRIDE>(base);
        ReadRows<I + 1, N, STRIDE>::run(base, dst, kk);
    }
};
template <int N, int STRIDE>
struct ReadRows<N, N, STRIDE> {
    __device__ __forceinline__ static void run(uint32_t, uint4 (&)[N][2], int) {}
};

// HD > 0: the 128-channel k7 conv of a residual unit with dilation HD (Cin = Cout = 128, pad 3*HD).  Its A
// operand is staged ONCE per tile: the BM + 6*HD input rows the tile's seven taps read (the halo) land in LDS
// as 256-byte rows (16-byte chunks XOR-swizzled by row & 15), and tap k reads its fragments at a shift of
// k*HD rows; only the weights stream through the two-buffer ring (4 instead of 8 LDS-DMA pieces per wave per
// k-tile, A read from HBM / L2 once instead of seven times).  Tiles do not cross sequences (block -> (item,
// tile of that item)).  HD = 0: the generic implicit-GEMM staging (A rows re-gathered per k-tile).
template <bool FUSE2, int HD>
__global__ void __launch_bounds__(256, 2) conv_gemm_kernel(ConvGemmArgs p) {
    constexpr int BM = 128, BN = 128, WM = 2, WN = 2, NW = 4;
    constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
    constexpr int BK = 64, ROWB = BK * 2, STAGE = (BM + BN) * ROWB;
    constexpr int WSTAGE = BN * ROWB;                      // weight k-tile (halo mode)
    constexpr int HR = BM + 6 * HD;                        // halo rows
    constexpr int HP = (HR + 3) / 4;                       // 1 KiB halo pieces (4 rows of 256 B)
    constexpr int HPW = (HP + NW - 1) / NW;                // pieces per wave (the last clamped: duplicates)
    constexpr int HALO = HP * 1024;
    constexpr int G_PER_WAVE = HD ? BN / 8 / NW : (BM + BN) / 8 / NW;  // LDS-DMA pieces per wave per k-tile
    constexpr int SMEM = HD ? HALO + 2 * WSTAGE : 2 * STAGE;
    static_assert(BM * BN * 4 <= SMEM, "epilogue tile must fit the LDS image");

    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;

    // block -> tile: XCD-aware bijective remap (consecutive tiles on one XCD), then M-grouped order
    const int Mi = p.M / p.items;  // rows per sequence
    int bid = blockIdx.x;
    {
        const int nwg = gridDim.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    }
    int m0, n0, mlim;
    if constexpr (HD > 0) {
        const int nt = (Mi + BM - 1) / BM;
        const int item = bid / nt;
        m0 = item * Mi + (bid - item * nt) * BM;
        mlim = item * Mi + Mi;
        n0 = 0;
    } else {
        const int nbm = (p.M + BM - 1) / BM;
        const int nbn = p.N / BN;
        constexpr int GM = 8;
        const int group = bid / (GM * nbn);
        const int first_m = group * GM;
        const int gm = min(nbm - first_m, GM);
        m0 = (first_m + (bid % (GM * nbn)) % gm) * BM;
        n0 = ((bid % (GM * nbn)) / gm) * BN;
        mlim = p.M;
    }
    const int wm0 = (wid / WN) * WTM, wn0 = (wid % WN) * WTN;

    const int cblocks = p.Cin / BK;
    const int nk = p.taps * cblocks;
    const int K = p.taps * p.Cin;

    // per-lane staging rows (fixed) and swizzled 16-byte chunk
    int srow[G_PER_WAVE];
    int schunk[G_PER_WAVE];
    int sml[G_PER_WAVE];           // row within its sequence (A rows)
    int64_t sbase[G_PER_WAVE];     // first input row of its sequence
#pragma unroll
    for (int j = 0; j < G_PER_WAVE; ++j) {
        const int row = (wid + NW * j) * 8 + (lane >> 3) + (HD ? BM : 0);  // halo mode: weight rows only
        srow[j] = row;
        schunk[j] = (lane & 7) ^ swz(row);
        const int m = m0 + row, item = m / Mi;
        sml[j] = m - item * Mi;
        sbase[j] = (int64_t)item * p.T_in;
    }
    auto stage = [&](int buf, int kt) {
        char* base = HD ? smem + HALO + buf * WSTAGE - BM * ROWB : smem + buf * STAGE;
        const int tap = kt / cblocks;
        const int c0 = (kt - tap * cblocks) * BK;
        const int shift = tap * p.dil - p.pad;
        const int istr = p.in_stride;
#pragma unroll
        for (int j = 0; j < G_PER_WAVE; ++j) {
            const int row = srow[j];
            const uint16_t* src;
            if (!HD && row < BM) {
                const int m = m0 + row;
                const int t = sml[j] * istr + shift;
                src = (m < p.M && t >= 0 && t < p.T_in) ? p.S + (sbase[j] + t) * p.Cin + c0 + schunk[j] * 8
                                                        : p.zero + schunk[j] * 8;
            } else {
                src = p.W + (int64_t)(n0 + row - BM) * K + kt * BK + schunk[j] * 8;
            }
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(base + (wid + NW * j + (HD ? BM / 8 : 0)) * 1024),
                                             16, 0, 0);
        }
    };
    // halo mode: input rows t0 - 3*HD .. t0 + BM - 1 + 3*HD of the tile's sequence (zero rows outside it)
    auto stage_halo = [&]() {
        const int item = m0 / Mi, t0 = m0 - item * Mi;
        const int hc = lane & 15;
#pragma unroll
        for (int j = 0; j < HPW; ++j) {
            const int pc = min(wid + NW * j, HP - 1);
            const int hr = pc * 4 + (lane >> 4);
            const int t = t0 - 3 * HD + hr;
            const int cl = hc ^ (hr & 15);
            const uint16_t* src = (hr < HR && t >= 0 && t < p.T_in) ? p.S + ((int64_t)item * p.T_in + t) * 128 + cl * 8
                                                                     : p.zero + hc * 8;
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(smem + pc * 1024), 16, 0, 0);
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const uint32_t lds0 = lds_addr(smem);
    const int lrow = lane & 15, lchunk = lane >> 4;
    auto read_frags = [&](int kt, uint4 (&a)[TM][2], uint4 (&b)[TN][2]) {
        const int buf = kt & 1;
        const uint32_t sbB = HD ? lds0 + HALO + buf * WSTAGE : lds0 + buf * STAGE + BM * ROWB;
        const int tap = kt >> 1, half = kt & 1;                 // (halo mode: Cin = 128, two k-tiles per tap)
        const int hrow = wm0 + lrow + tap * HD;                 // halo row of fragment 0 (+16 per fragment)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            const int ch = (kk * 4 + lchunk) ^ ((lrow >> 1) & 7);
            ReadRows<0, TN, 16 * ROWB>::run(sbB + (wn0 + lrow) * ROWB + ch * 16, b, kk);
            if constexpr (HD > 0) {
                const int hch = (half * 8 + kk * 4 + lchunk) ^ (hrow & 15);
                ReadRows<0, TM, 16 * 256>::run(lds0 + hrow * 256 + hch * 16, a, kk);
            } else {
                ReadRows<0, TM, 16 * ROWB>::run(lds0 + buf * STAGE + (wm0 + lrow) * ROWB + ch * 16, a, kk);
            }
        }
        lds_wait_all();
    };
    auto mma = [&](const uint4 (&a)[TM][2], const uint4 (&b)[TN][2], int i0) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
            for (int i = i0; i < i0 + TM / 2; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a[i][kk]),
                                                                       __builtin_bit_cast(f16x8, b[j][kk]),
                                                                       acc[i][j], 0, 0, 0);
    };

    // PIPE-1 schedule of the DiT GEMM (gemm.hip): fragments read up front, raw barrier frees the
    // buffer, tile kt+2 staged while the MFMAs run, counted vmcnt retires kt+1.
    if constexpr (HD > 0) stage_halo();  // retired together with k-tile 0
    stage(0, 0);
    if (nk > 1) {
        stage(1, 1);
        wait_vmcnt<G_PER_WAVE>();
    } else {
        wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    // every MFMA after the barrier: issuing half of them before it makes the register allocator
    // rotate those accumulators through VGPRs each iteration (48 v_accvgpr copies per 32 MFMAs)
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        uint4 a[TM][2], b[TN][2];
        read_frags(kt, a, b);
        __builtin_amdgcn_s_barrier();
        const bool more = kt + 2 < nk;
        if (more) stage(cur, kt + 2);
        mma(a, b, 0);
        mma(a, b, TM / 2);
        mfma_war_retire(a, b);
        if (kt + 1 < nk) {
            if (more)
                wait_vmcnt<G_PER_WAVE>();
            else
                wait_vmcnt<0>();
            __builtin_amdgcn_s_barrier();
        }
    }

    if constexpr (FUSE2) {
        // k1 conv of the residual unit on this tile (N = Cout = 128: the tile holds every channel).
        // W2 fragments straight from global memory (32 KB, L2-resident), issued before the LDS round trip.
        const int lrow2 = lane & 15, lch2 = lane >> 4;
        uint4 b2f[TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
                b2f[j][ks] = *reinterpret_cast<const uint4*>(p.W2 + (int64_t)(wn0 + j * 16 + lrow2) * 128 + ks * 32 +
                                                            lch2 * 8);
        // y = Snake2(acc + bias) as fp16 into a [128][128] LDS tile, 16-byte chunks XOR-swizzled by row
        __builtin_amdgcn_s_barrier();  // every wave's last fragment reads of the main loop are done
        const int ccol2 = lane & 15, crow2 = (lane >> 4) * 4;
        char* ytile = smem;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = wn0 + j * 16 + ccol2;
            const float b1 = p.bias ? p.bias[col] : 0.f;
            const float ea = p.snake2_ea[col], reb = __builtin_amdgcn_rcpf(p.snake2_eb[col]);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = wm0 + i * 16 + crow2 + r;
                    const float v = rn_add(acc[i][j][r], b1);
                    *reinterpret_cast<uint16_t*>(ytile + row * 256 + (((col >> 3) ^ (row & 15)) << 4) + (col & 7) * 2) =
                        f32_to_f16(snake_f(v, ea, reb));
                }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
        const uint32_t y0 = lds_addr(ytile);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            uint4 a2[TM];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm0 + i * 16 + lrow2;
                a2[i] = *reinterpret_cast<const uint4*>(ytile + row * 256 + (((ks * 4 + lch2) ^ (row & 15)) << 4));
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a2[i]),
                                                                       __builtin_bit_cast(f16x8, b2f[j][ks]),
                                                                       acc[i][j], 0, 0, 0);
            mfma_war_retire(a2, b2f);
        }
        (void)y0;
    }
    const float* bias_e = FUSE2 ? p.bias2 : p.bias;

    // Epilogue through LDS: the bias-added tile goes to LDS as f32 [BM][BN] (64 KB = both stage buffers), then
    // every wave sweeps two whole tile rows per instruction (lane = 4 consecutive columns), so the residual read,
    // the f32 store and the fp16 Snake store are 16 / 16 / 8-byte accesses over 512 contiguous bytes of a row.
    // (From the accumulator layout each wave instruction touched 4 rows x 64 B, with 4-byte accesses; at 128
    // channels the read-modify-write of x cost as much as the MFMAs.)  Same arithmetic per element: acc + bias,
    // then x + that, then the Snake of the sum.
    static_assert(BM * BN * 4 <= 2 * STAGE, "epilogue tile must fit the stage buffers");
    float* zt = reinterpret_cast<float*>(smem);
    const int c4 = (lane & 31) * 4;
    const int n = n0 + c4;
    const int rr = p.up > 1 ? n / p.Cout : 0;
    const int co = n - rr * p.Cout;
    constexpr int RPI = NW * 2;  // tile rows per sweep iteration
    constexpr int NIT = BM / RPI;
    // output offset of sweep iteration `it` (this lane's 4 columns), or -1 outside the sequence / the crop
    // (branch-free: the residual loads below are issued unconditionally from a clamped offset -- behind a branch,
    // hipcc waited for every earlier load before the next one)
    auto out_off = [&](int it) -> int64_t {
        const int m = m0 + it * RPI + wid * 2 + (lane >> 5);
        const int item = m / Mi, ml = m - item * Mi;
        const int u = p.up > 1 ? ml * p.up + rr - p.crop : ml;
        const bool ok = m < mlim && u >= 0 && u < p.T_out;
        return ok ? ((int64_t)item * p.T_out + u) * p.Cout + co : (int64_t)-1;
    };
    // per-column bias and Snake parameters first: a wait for any load issued after the residual loads below would
    // also wait for those (vmcnt retires in issue order)
    const int ccol = lane & 15, crow = (lane >> 4) * 4;
    float bz[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        int cz = n0 + wn0 + j * 16 + ccol;
        if (p.up > 1) cz -= (cz / p.Cout) * p.Cout;
        bz[j] = bias_e ? bias_e[cz] : 0.f;
    }
    float ea[4], reb[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        ea[e] = p.snake_ea ? p.snake_ea[co + e] : 0.f;
        reb[e] = p.snake_eb ? __builtin_amdgcn_rcpf(p.snake_eb[co + e]) : 0.f;
    }
    // the residual's old values for the whole sweep are requested here, before the tile goes through LDS, so one
    // HBM round trip (under the z writes and the barriers) replaces one per group of iterations
    // (no resid: the loads read the zero buffer -- a branch around them made hipcc wait vmcnt(0) at the first use
    // of the bias loads, i.e. for all of them)
    // (the asm uses make hipcc retire the bias / Snake loads here: its wait at their first later use was vmcnt(0),
    // i.e. for every residual load too)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(bz[j]));
#pragma unroll
    for (int e = 0; e < 4; ++e) asm volatile("" ::"v"(ea[e]), "v"(reb[e]));
    __builtin_amdgcn_sched_barrier(0);
    const float* xsrc = p.resid ? p.X : reinterpret_cast<const float*>(p.zero);
    float4 xo[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int64_t o = out_off(it);
        xo[it] = *reinterpret_cast<const float4*>(xsrc + (p.resid && o >= 0 ? o : 0));
    }
    __builtin_amdgcn_sched_barrier(0);
    {
        __builtin_amdgcn_s_barrier();  // every wave is done with the stage buffers / the fused conv's y tile
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = wn0 + j * 16 + ccol;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    zt[(wm0 + i * 16 + crow + r) * BN + col] = bias_e ? rn_add(acc[i][j][r], bz[j]) : acc[i][j][r];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int64_t o = out_off(it);
        if (o < 0) continue;
        const int row = it * RPI + wid * 2 + (lane >> 5);
        float4 v = *reinterpret_cast<const float4*>(zt + row * BN + c4);
        if (p.resid) {
            v.x = rn_add(xo[it].x, v.x);
            v.y = rn_add(xo[it].y, v.y);
            v.z = rn_add(xo[it].z, v.z);
            v.w = rn_add(xo[it].w, v.w);
        }
        if (p.store_x) *reinterpret_cast<float4*>(p.X + o) = v;
        if (p.S_out) {
            const float vv[4] = {v.x, v.y, v.z, v.w};
            uint16_t h[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) h[e] = f32_to_f16(p.snake_ea ? snake_f(vv[e], ea[e], reb[e]) : vv[e]);
            *reinterpret_cast<uint2*>(p.S_out + o) =
                make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
        }
    }
}

// f32 -> fp16 copy (the latents' im2col conversion of decoder.conv1)
__global__ void to_f16_kernel(const float* __restrict__ x, int64_t n, uint16_t* __restrict__ y) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = f32_to_f16(x[i]);
}

__global__ void pack_f16_kernel(const float* __restrict__ x, int64_t rows, int C, int Cpad, uint16_t* __restrict__ y) {
    const int64_t n = rows * Cpad;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / Cpad;
        const int c = (int)(i - r * Cpad);
        y[i] = c < C ? f32_to_f16(x[r * C + c]) : (uint16_t)0;
    }
}

// decoder.conv2: C -> out_ch (2), kernel 7, pad 3, no bias, on the fp16 Snake output.  Too narrow
// for MFMA tiles and HBM-bound (the C = 128-channel input is read once, OUT channels written).  A 16-lane
// group owns a strip of R = 8 consecutive output times of one sequence: each lane holds 8 input channels
// (16-byte loads, a group reads each 256-byte row once and keeps the R + 6 rows it needs in registers) and
// its 7 x 8 x OUT weights as f32 in registers; the exact fp16 products are accumulated in f32 per lane and
// combined over the 16 lanes by xor shuffles.
template <int OUT>
__global__ void __launch_bounds__(256) conv_out_kernel(const uint16_t* __restrict__ S, int T,
                                                       const uint16_t* __restrict__ W, float* __restrict__ out,
                                                       int items) {
    constexpr int C = 128, R = 8;
    const int l16 = threadIdx.x & 15;
    float wr[7][8][OUT];  // this lane's channels 8*l16 .. 8*l16+7
#pragma unroll
    for (int k = 0; k < 7; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c)
#pragma unroll
            for (int o = 0; o < OUT; ++o)
                wr[k][c][o] = (float)__builtin_bit_cast(_Float16, W[((int64_t)o * 7 + k) * C + l16 * 8 + c]);
    const int strips = (T + R - 1) / R;
    const int64_t strip = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
    if (strip >= (int64_t)strips * items) return;  // whole 16-lane groups leave together
    const int item = (int)(strip / strips);
    const int t0 = (int)(strip - (int64_t)item * strips) * R;
    const uint16_t* Si = S + (int64_t)item * T * C + l16 * 8;
    uint4 rows[R + 6];
#pragma unroll
    for (int i = 0; i < R + 6; ++i) {
        const int ti = t0 - 3 + i;
        rows[i] = (ti >= 0 && ti < T) ? *reinterpret_cast<const uint4*>(Si + (int64_t)ti * C) : make_uint4(0, 0, 0, 0);
    }
    float acc[R][OUT];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int o = 0; o < OUT; ++o) acc[r][o] = 0.f;
#pragma unroll
    for (int i = 0; i < R + 6; ++i) {
        const uint32_t w4[4] = {rows[i].x, rows[i].y, rows[i].z, rows[i].w};
        float x[8];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            x[2 * h] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w4[h] & 0xffffu));
            x[2 * h + 1] = (float)__builtin_bit_cast(_Float16, (uint16_t)(w4[h] >> 16));
        }
#pragma unroll
        for (int k = 0; k < 7; ++k) {  // input row t0 - 3 + i feeds output r = i - k through tap k
            const int r = i - k;
            if (r < 0 || r >= R) continue;
#pragma unroll
            for (int c = 0; c < 8; ++c)
#pragma unroll
                for (int o = 0; o < OUT; ++o) acc[r][o] = fmaf(x[c], wr[k][c][o], acc[r][o]);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int o = 0; o < OUT; ++o)
#pragma unroll
            for (int off = 8; off >= 1; off >>= 1) acc[r][o] += __shfl_xor(acc[r][o], off);
    if (l16 < R) {  // lane r writes output row t0 + r
        const int t = t0 + l16;
        if (t < T) {
            float v[OUT];
#pragma unroll
            for (int o = 0; o < OUT; ++o) {
                float a = acc[0][o];
#pragma unroll
                for (int r = 1; r < R; ++r) a = l16 == r ? acc[r][o] : a;
                v[o] = a;
            }
            float* dst = out + ((int64_t)item * T + t) * OUT;
#pragma unroll
            for (int o = 0; o < OUT; ++o) dst[o] = v[o];
        }
    }
}

}  // namespace

// ACE_MI_VAE_HALO=0: the residual units' k7 convs through the generic staging (A/B switch, read per launch)
static bool vae_halo_on() {
    const char* e = std::getenv("ACE_MI_VAE_HALO");
    return !(e && e[0] == '0');
}

void launch_conv_gemm(const ConvGemmArgs& a, hipStream_t s) {
    ACEMI_CHECK(a.Cin % 64 == 0 && a.N % 128 == 0 && a.M >= 1 && a.taps >= 1, "conv_gemm: unsupported shape");
    ACEMI_CHECK(a.S && a.W && a.zero, "conv_gemm: null operand");
    ACEMI_CHECK(a.up <= 1 || a.N == a.up * a.Cout, "conv_gemm: transposed conv needs N = stride * Cout");
    ACEMI_CHECK(a.up > 1 || a.N == a.Cout, "conv_gemm: N must equal Cout");
    ACEMI_CHECK(!(a.resid || a.store_x) || a.X, "conv_gemm: null X");
    ACEMI_CHECK(a.items >= 1 && a.M % a.items == 0, "conv_gemm: rows must split evenly into the sequences");
    ACEMI_CHECK(a.Cout % 4 == 0, "conv_gemm: output channels must be a multiple of 4");
    const int nbm = (a.M + 127) / 128, nbn = a.N / 128;
    if (a.W2)
        ACEMI_CHECK(a.N == 128 && a.Cout == 128 && a.up <= 1 && a.snake2_ea && a.snake2_eb,
                    "conv_gemm: the fused k1 conv needs Cout = N = 128 and a Snake between the convs");
    // the residual unit's dilated k7 conv at 128 channels: halo-staged A (one LDS image per tile)
    const int hd = (a.taps == 7 && a.Cin == 128 && a.N == 128 && a.Cout == 128 && a.up <= 1 &&
                    a.in_stride == 1 && a.T_in * a.items == a.M && a.pad == 3 * a.dil &&
                    (a.dil == 1 || a.dil == 3 || a.dil == 9) && vae_halo_on())
                       ? a.dil
                       : 0;
    const dim3 blk(256);
    const int ntiles = hd ? a.items * ((a.M / a.items + 127) / 128) : nbm * nbn;
    if (hd) {
        const dim3 grid((unsigned)ntiles);
        auto go = [&](auto fuse) {
            constexpr bool F = decltype(fuse)::value;
            if (hd == 1) hipLaunchKernelGGL((conv_gemm_kernel<F, 1>), grid, blk, 0, s, a);
            else if (hd == 3) hipLaunchKernelGGL((conv_gemm_kernel<F, 3>), grid, blk, 0, s, a);
            else hipLaunchKernelGGL((conv_gemm_kernel<F, 9>), grid, blk, 0, s, a);
        };
        if (a.W2) go(std::true_type{});
        else go(std::false_type{});
    } else if (a.W2) {
        hipLaunchKernelGGL((conv_gemm_kernel<true, 0>), dim3(nbm * nbn), blk, 0, s, a);
    } else {
        hipLaunchKernelGGL((conv_gemm_kernel<false, 0>), dim3(nbm * nbn), blk, 0, s, a);
    }
    ACEMI_HIP(hipGetLastError());
}

void launch_to_f16(const float* x, int64_t n, uint16_t* y, hipStream_t s) {
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(to_f16_kernel, dim3(std::max(grid, 1)), dim3(256), 0, s, x, n, y);
    ACEMI_HIP(hipGetLastError());
}

void launch_pack_f16(const float* x, int64_t rows, int C, int Cpad, uint16_t* y, hipStream_t s) {
    const int64_t n = rows * Cpad;
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(pack_f16_kernel, dim3(std::max(grid, 1)), dim3(256), 0, s, x, rows, C, Cpad, y);
    ACEMI_HIP(hipGetLastError());
}

void launch_conv_out(const uint16_t* S, int T, int C, const uint16_t* W, int out_ch, float* out, hipStream_t s,
                     int items) {
    ACEMI_CHECK(C == 128, "conv_out: decoder.conv2 input channels must be 128");
    ACEMI_CHECK(items >= 1 && (int64_t)T * items < (1LL << 31), "conv_out: bad sequence count");
    const int64_t strips = (int64_t)((T + 7) / 8) * items;  // 8 output times per 16-lane group
    const dim3 grid((unsigned)((strips + 15) / 16));
    if (out_ch == 1)
        hipLaunchKernelGGL(conv_out_kernel<1>, grid, dim3(256), 0, s, S, T, W, out, items);
    else if (out_ch == 2)
        hipLaunchKernelGGL(conv_out_kernel<2>, grid, dim3(256), 0, s, S, T, W, out, items);
    else
        throw std::runtime_error("conv_out: audio_channels must be 1 or 2");
    ACEMI_HIP(hipGetLastError());
}

}  // namespace acemi
