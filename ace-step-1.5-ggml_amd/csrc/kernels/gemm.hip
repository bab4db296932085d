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
#include "../kernels.h"

namespace acemi {
namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

typedef __attribute__((address_space(3))) void lds_void;

struct GemmParams {
    const uint16_t* A;
    const uint16_t* W;
    int lda, ldw, M, N, K;
    GemmEpilogue e;
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

template <int BM, int BN, int WM, int WN, bool F16, int EPI>
__global__ void __launch_bounds__(WM * WN * 64) gemm_kernel(GemmParams p) {
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

    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wid = tid >> 6;

    // ---- block -> tile (XCD-aware bijective remap, then M-grouped order)
    const int nbm = (p.M + BM - 1) / BM;
    const int nbn = p.N / BN;
    const int nwg = gridDim.x;
    int bid = blockIdx.x;
    {
        const int xcd = bid & 7;
        const int q = nwg >> 3, r = nwg & 7;
        bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    }
    constexpr int GM = 8;
    const int group = bid / (GM * nbn);
    const int first_m = group * GM;
    const int gm = min(nbm - first_m, GM);
    const int bm = first_m + (bid % (GM * nbn)) % gm;
    const int bn = (bid % (GM * nbn)) / gm;
    const int m0 = bm * BM;
    const int n0 = bn * BN;

    const int wm = wid / WN;
    const int wn = wid % WN;
    const int wm0 = wm * WTM;
    const int wn0 = wn * WTN;

    const uint16_t* __restrict__ A = p.A;
    const uint16_t* __restrict__ W = p.W;
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

    const int nk = p.K / BK;
    stage(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    const int lrow = lane & 15;
    const int lchunk = lane >> 4;

    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        if (kt + 1 < nk) stage(cur ^ 1, kt + 1);
        const char* As = smem + cur * STAGE;
        const char* Bs = As + BM * ROWB;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            uint4 a[TM], b[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm0 + i * 16 + lrow;
                const int ch = (kk * 4 + lchunk) ^ swz(row);
                a[i] = *(const uint4*)(As + row * ROWB + ch * 16);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = wn0 + j * 16 + lrow;
                const int ch = (kk * 4 + lchunk) ^ swz(row);
                b[j] = *(const uint4*)(Bs + row * ROWB + ch * 16);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) acc[i][j] = mfma16<F16>(a[i], b[j], acc[i][j]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }

    // ---- epilogue.  C/D map of 16x16x32: col = lane & 15, row = (lane >> 4) * 4 + r.
    const GemmEpilogue& e = p.e;
    const int ccol = lane & 15;
    const int crow = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm0 + i * 16 + crow + r;
            if (m >= M) continue;
            if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
                for (int j = 0; j < TN; j += 2) {
                    const int n = n0 + wn0 + j * 16;  // multiple of 32
                    const float g = acc[i][j][r];
                    const float u = acc[i][j + 1][r];
                    e.c_act[(int64_t)m * e.ldc + (n >> 1) + ccol] = to_act<F16>(silu_f(g) * u);
                }
            } else {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int n = n0 + wn0 + j * 16 + ccol;
                    float v = acc[i][j][r];
                    if constexpr (EPI == EPI_STORE_F32) {
                        if (e.bias) v = v + e.bias[n];
                        e.c_f32[(int64_t)m * e.ldc + n] = v;
                    } else if constexpr (EPI == EPI_STORE_ACT) {
                        if (e.bias) v = v + e.bias[n];
                        e.c_act[(int64_t)m * e.ldc + n] = to_act<F16>(v);
                    } else if constexpr (EPI == EPI_RESID_GATED) {
                        const int item = m / e.rows_per_item;
                        float* xp = e.c_f32 + (int64_t)m * e.ldc + n;
                        const float gated = __fmul_rn(v, e.gate[(int64_t)item * e.gate_stride + n]);
                        *xp = __fadd_rn(*xp, gated);
                    } else if constexpr (EPI == EPI_RESID) {
                        float* xp = e.c_f32 + (int64_t)m * e.ldc + n;
                        *xp = __fadd_rn(*xp, v);
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

template <int BM, int BN, int WM, int WN, bool F16, int EPI>
void launch_cfg(const GemmParams& p, hipStream_t s) {
    const int nbm = (p.M + BM - 1) / BM;
    const int nbn = p.N / BN;
    const dim3 grid(nbm * nbn);
    const dim3 block(WM * WN * 64);
    const size_t lds = 2 * (BM + BN) * 128;
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, F16, EPI>), grid, block, lds, s, p);
}

template <bool F16>
void dispatch_epi(const GemmParams& p, hipStream_t s) {
    switch (p.e.kind) {
        case EPI_STORE_F32: launch_cfg<128, 128, 2, 2, F16, EPI_STORE_F32>(p, s); break;
        case EPI_STORE_ACT: launch_cfg<128, 128, 2, 2, F16, EPI_STORE_ACT>(p, s); break;
        case EPI_RESID_GATED: launch_cfg<128, 128, 2, 2, F16, EPI_RESID_GATED>(p, s); break;
        case EPI_RESID: launch_cfg<128, 128, 2, 2, F16, EPI_RESID>(p, s); break;
        case EPI_SWIGLU: launch_cfg<128, 128, 2, 2, F16, EPI_SWIGLU>(p, s); break;
        case EPI_PROJ_OUT: launch_cfg<128, 128, 2, 2, F16, EPI_PROJ_OUT>(p, s); break;
        default: throw std::runtime_error("gemm: bad epilogue kind");
    }
}

}  // namespace

void launch_gemm(ActType t, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                 const GemmEpilogue& epi, hipStream_t s) {
    ACEMI_CHECK(M >= 1 && N % 128 == 0 && K % 64 == 0 && K >= 64, "gemm: unsupported shape");
    ACEMI_CHECK(lda % 8 == 0 && ldw % 8 == 0, "gemm: leading dims must be multiples of 8");
    GemmParams p{A, W, lda, ldw, M, N, K, epi};
    if (t == ActType::F16)
        dispatch_epi<true>(p, s);
    else
        dispatch_epi<false>(p, s);
    ACEMI_HIP(hipGetLastError());
}

}  // namespace acemi
