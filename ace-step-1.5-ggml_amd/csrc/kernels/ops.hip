// Memory-bound kernels around the DiT GEMMs and attention (gfx950).
// Each kernel cites the ggml graph nodes of ace_dit::forward_dit it fuses.
#include "../kernels.h"
#include "prep_math.h"

namespace acemi {
namespace {

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 64u);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
__device__ __forceinline__ uint16_t f32_to_f16(float f) {
    _Float16 h = (_Float16)f;
    return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ uint16_t to_act(bool f16, float f) { return f16 ? f32_to_f16(f) : f32_to_bf16_rne(f); }
__device__ __forceinline__ float act_to_f32(bool f16, uint16_t v) {
    if (f16) return (float)__builtin_bit_cast(_Float16, v);
    return __uint_as_float((uint32_t)v << 16);
}
__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ---------------------------------------------------------------- pack
// input pack + patchify (acestep_dit_model.cpp:1350-1380): x0[t] = concat(context[t], hidden[t]),
// zero padded to a multiple of the patch, viewed as [Np][P*Cin] (index k*Cin + c).
__global__ void pack_input_kernel(bool f16, bool x3, const float* __restrict__ hidden, const float* __restrict__ context,
                                  int B, int T, int Np, int P, int audio, int cdim, uint16_t* __restrict__ out) {
    const int cin = audio + cdim;
    const int rowlen = P * cin;
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
        if (x3) {  // f32 operand as fp16 [hi | hi | lo] (WF_F32X3 weights)
            const int64_t row = i / rowlen, col = i - row * rowlen;
            uint16_t* o = out + row * 3 * rowlen + col;
            const uint16_t hi = f32_to_f16(v);
            o[0] = hi;
            o[rowlen] = hi;
            o[2 * rowlen] = f32_to_f16(v - (float)__builtin_bit_cast(_Float16, hi));
        } else {
            out[i] = to_act(f16, v);
        }
    }
}

__global__ void to_act_kernel(bool f16, const float* __restrict__ in, int64_t n, bool silu, uint16_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        float v = in[i];
        if (silu) v = silu_f(v);
        out[i] = to_act(f16, v);
    }
}

// ------------------------------------------------------------ rmsnorm
// rms_norm (:1097-1106) + AdaLN modulate (:1477-1481, :1522-1526, :1545-1549):
// y = ((x * 1/sqrt(mean(x^2)+eps)) * w) * (1 + scale) + shift, written in the act type that the
// following mul_mat converts it to.
template <bool F16, int VPT, bool X3 = false>
__global__ void __launch_bounds__(256) rmsnorm_mod_kernel(const float* __restrict__ x, int H, const float* __restrict__ w,
                                                          const float* __restrict__ scale, const float* __restrict__ shift,
                                                          int64_t mod_stride, int rows_per_item, float eps,
                                                          uint16_t* __restrict__ out) {
    // one row per workgroup, VPT float4 per thread kept in registers (H <= 1024 * VPT)
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
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const float tot = red[0] + red[1] + red[2] + red[3];
    const float sc = 1.0f / sqrtf(tot / (float)H + eps);
    const int item = m / rows_per_item;
    const float* scp = scale ? scale + (int64_t)item * mod_stride : nullptr;
    const float* shp = shift ? shift + (int64_t)item * mod_stride : nullptr;
    uint16_t* orow = out + (int64_t)m * H * (X3 ? 3 : 1);
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const int i = (threadIdx.x + k * 256) * 4;
        if (i >= H) break;
        const float4 wv = *(const float4*)(w + i);
        float y[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
        const float ww[4] = {wv.x, wv.y, wv.z, wv.w};
        float s4[4] = {0.f, 0.f, 0.f, 0.f}, h4[4] = {0.f, 0.f, 0.f, 0.f};
        if (scp) {
            const float4 a4 = *(const float4*)(scp + i);
            const float4 b4 = *(const float4*)(shp + i);
            s4[0] = a4.x; s4[1] = a4.y; s4[2] = a4.z; s4[3] = a4.w;
            h4[0] = b4.x; h4[1] = b4.y; h4[2] = b4.z; h4[3] = b4.w;
        }
        uint16_t o[4], lo[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float t = rn_mul(rn_mul(y[j], sc), ww[j]);
            if (scp) t = rn_add(rn_mul(t, rn_add(s4[j], 1.0f)), h4[j]);
            o[j] = (F16 || X3) ? f32_to_f16(t) : f32_to_bf16_rne(t);
            if (X3) lo[j] = f32_to_f16(t - (float)__builtin_bit_cast(_Float16, o[j]));
        }
        if constexpr (X3) {  // f32 operand as fp16 [hi | hi | lo] (WF_F32X3 weights)
            uint2 ph, pl;
            ph.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
            ph.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
            pl.x = (uint32_t)lo[0] | ((uint32_t)lo[1] << 16);
            pl.y = (uint32_t)lo[2] | ((uint32_t)lo[3] << 16);
            *(uint2*)(orow + i) = ph;
            *(uint2*)(orow + H + i) = ph;
            *(uint2*)(orow + 2 * H + i) = pl;
            continue;
        }
        uint2 pk;
        pk.x = (uint32_t)o[0] | ((uint32_t)o[1] << 16);
        pk.y = (uint32_t)o[2] | ((uint32_t)o[3] << 16);
        *(uint2*)(orow + i) = pk;
    }
}

// Same operator, one 64-lane wave per row (4 rows per workgroup): H = 512 * NC, each lane holds NC runs of 8
// consecutive values (two 16-B loads, one 16-B store per run), the row sum is a wave reduction (no LDS, no
// barrier), and the w / scale / shift loads are issued before it so their latency hides under the shuffles.
template <bool F16, int NC>
__global__ void __launch_bounds__(256) rmsnorm_mod_rows_kernel(const float* __restrict__ x, int M, int H,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift, int64_t mod_stride,
                                                               int rows_per_item, float eps,
                                                               uint16_t* __restrict__ out) {
    const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= M) return;
    const int lane = threadIdx.x & 63;
    const float* xr = x + (int64_t)m * H;
    float4 v[2 * NC], wv[2 * NC];
    float ss = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int i = c * 512 + lane * 8;
        v[2 * c] = *(const float4*)(xr + i);
        v[2 * c + 1] = *(const float4*)(xr + i + 4);
        wv[2 * c] = *(const float4*)(w + i);
        wv[2 * c + 1] = *(const float4*)(w + i + 4);
    }
#pragma unroll
    for (int k = 0; k < 2 * NC; ++k) ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
    const int item = m / rows_per_item;
    const float* scp = scale ? scale + (int64_t)item * mod_stride : nullptr;
    const float* shp = shift ? shift + (int64_t)item * mod_stride : nullptr;
    ss = wave_sum(ss);
    const float sc = 1.0f / sqrtf(ss / (float)H + eps);
    uint16_t* orow = out + (int64_t)m * H;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int i = c * 512 + lane * 8;
        float y[8] = {v[2 * c].x, v[2 * c].y, v[2 * c].z, v[2 * c].w,
                      v[2 * c + 1].x, v[2 * c + 1].y, v[2 * c + 1].z, v[2 * c + 1].w};
        const float ww[8] = {wv[2 * c].x, wv[2 * c].y, wv[2 * c].z, wv[2 * c].w,
                             wv[2 * c + 1].x, wv[2 * c + 1].y, wv[2 * c + 1].z, wv[2 * c + 1].w};
        float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, h8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (scp) {
            const float4 a0 = *(const float4*)(scp + i), a1 = *(const float4*)(scp + i + 4);
            const float4 b0 = *(const float4*)(shp + i), b1 = *(const float4*)(shp + i + 4);
            s8[0] = a0.x; s8[1] = a0.y; s8[2] = a0.z; s8[3] = a0.w; s8[4] = a1.x; s8[5] = a1.y; s8[6] = a1.z; s8[7] = a1.w;
            h8[0] = b0.x; h8[1] = b0.y; h8[2] = b0.z; h8[3] = b0.w; h8[4] = b1.x; h8[5] = b1.y; h8[6] = b1.z; h8[7] = b1.w;
        }
        uint32_t pk[4];
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            float t0 = rn_mul(rn_mul(y[j], sc), ww[j]);
            float t1 = rn_mul(rn_mul(y[j + 1], sc), ww[j + 1]);
            if (scp) {
                t0 = rn_add(rn_mul(t0, rn_add(s8[j], 1.0f)), h8[j]);
                t1 = rn_add(rn_mul(t1, rn_add(s8[j + 1], 1.0f)), h8[j + 1]);
            }
            pk[j / 2] = (uint32_t)to_act(F16, t0) | ((uint32_t)to_act(F16, t1) << 16);
        }
        *(uint4*)(orow + i) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    }
}

// Same operator, persistent: a fixed grid of waves strides over the rows, each wave holding w (and the
// current item's 1 + scale, shift) in registers across its rows and loading the next row while it finishes
// this one.  The one-row-per-wave kernels re-read w / scale / shift from L2 for every row (3x the bytes of
// x itself) and run as one ramp-and-tail round of short-lived waves.
template <bool F16, int NC>
__global__ void __launch_bounds__(256) rmsnorm_mod_persist_kernel(const float* __restrict__ x, int M, int H,
                                                                  const float* __restrict__ w,
                                                                  const float* __restrict__ scale,
                                                                  const float* __restrict__ shift, int64_t mod_stride,
                                                                  int rows_per_item, float eps,
                                                                  uint16_t* __restrict__ out) {
    const int nwaves = gridDim.x * 4;
    int m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= M) return;
    const int lane = threadIdx.x & 63;
    float4 wv[2 * NC], s1[2 * NC], hv[2 * NC], v[2 * NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int i = c * 512 + lane * 8;
        v[2 * c] = *(const float4*)(x + (int64_t)m * H + i);
        v[2 * c + 1] = *(const float4*)(x + (int64_t)m * H + i + 4);
        wv[2 * c] = *(const float4*)(w + i);
        wv[2 * c + 1] = *(const float4*)(w + i + 4);
    }
    int item = -1;
    for (;;) {
        const int nxt = m + nwaves;
        float4 vn[2 * NC];
        if (nxt < M) {  // wave-uniform
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int i = c * 512 + lane * 8;
                vn[2 * c] = *(const float4*)(x + (int64_t)nxt * H + i);
                vn[2 * c + 1] = *(const float4*)(x + (int64_t)nxt * H + i + 4);
            }
        }
        const int it = m / rows_per_item;
        if (scale && it != item) {  // wave-uniform: a new batch item's modulation vectors
            item = it;
            const float* scp = scale + (int64_t)it * mod_stride;
            const float* shp = shift + (int64_t)it * mod_stride;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const int i = c * 512 + lane * 8;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const float4 a = *(const float4*)(scp + i + 4 * h);
                    s1[2 * c + h] = make_float4(rn_add(a.x, 1.0f), rn_add(a.y, 1.0f), rn_add(a.z, 1.0f), rn_add(a.w, 1.0f));
                    hv[2 * c + h] = *(const float4*)(shp + i + 4 * h);
                }
            }
        }
        float ss = 0.f;
#pragma unroll
        for (int k = 0; k < 2 * NC; ++k) ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
        ss = wave_sum(ss);
        const float sc = 1.0f / sqrtf(ss / (float)H + eps);
        uint16_t* orow = out + (int64_t)m * H;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int i = c * 512 + lane * 8;
            const float y[8] = {v[2 * c].x, v[2 * c].y, v[2 * c].z, v[2 * c].w,
                                v[2 * c + 1].x, v[2 * c + 1].y, v[2 * c + 1].z, v[2 * c + 1].w};
            const float ww[8] = {wv[2 * c].x, wv[2 * c].y, wv[2 * c].z, wv[2 * c].w,
                                 wv[2 * c + 1].x, wv[2 * c + 1].y, wv[2 * c + 1].z, wv[2 * c + 1].w};
            const float sp[8] = {s1[2 * c].x, s1[2 * c].y, s1[2 * c].z, s1[2 * c].w,
                                 s1[2 * c + 1].x, s1[2 * c + 1].y, s1[2 * c + 1].z, s1[2 * c + 1].w};
            const float hh[8] = {hv[2 * c].x, hv[2 * c].y, hv[2 * c].z, hv[2 * c].w,
                                 hv[2 * c + 1].x, hv[2 * c + 1].y, hv[2 * c + 1].z, hv[2 * c + 1].w};
            uint32_t pk[4];
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                float t0 = rn_mul(rn_mul(y[j], sc), ww[j]);
                float t1 = rn_mul(rn_mul(y[j + 1], sc), ww[j + 1]);
                if (scale) {
                    t0 = rn_add(rn_mul(t0, sp[j]), hh[j]);
                    t1 = rn_add(rn_mul(t1, sp[j + 1]), hh[j + 1]);
                }
                pk[j / 2] = (uint32_t)to_act(F16, t0) | ((uint32_t)to_act(F16, t1) << 16);
            }
            *(uint4*)(orow + i) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
        if (nxt >= M) break;
        m = nxt;
#pragma unroll
        for (int k = 0; k < 2 * NC; ++k) v[k] = vn[k];
    }
}

// f32 output variant for the condition encoders' final norm: ggml_rms_norm + ggml_mul by w
template <int VPT>
__global__ void __launch_bounds__(256) rmsnorm_f32_kernel(const float* __restrict__ x, int64_t row_step, int H,
                                                          const float* __restrict__ w, float eps,
                                                          float* __restrict__ out) {
    const int m = blockIdx.x;
    const float* xr = x + (int64_t)m * row_step * H;
    __shared__ float red[4];
    float4 v[VPT];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const int i = (threadIdx.x + k * 256) * 4;
        v[k] = i < H ? *(const float4*)(xr + i) : make_float4(0.f, 0.f, 0.f, 0.f);
        ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
    }
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    const float tot = red[0] + red[1] + red[2] + red[3];
    const float sc = 1.0f / sqrtf(tot / (float)H + eps);
    float* orow = out + (int64_t)m * H;
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const int i = (threadIdx.x + k * 256) * 4;
        if (i >= H) break;
        const float4 wv = *(const float4*)(w + i);
        float4 o;
        o.x = rn_mul(rn_mul(v[k].x, sc), wv.x);
        o.y = rn_mul(rn_mul(v[k].y, sc), wv.y);
        o.z = rn_mul(rn_mul(v[k].z, sc), wv.z);
        o.w = rn_mul(rn_mul(v[k].w, sc), wv.w);
        *(float4*)(orow + i) = o;
    }
}

// token-embedding gather: one workgroup per token, 4 values per thread per step
template <int FMT>
__global__ void __launch_bounds__(256) embed_rows_kernel(const void* __restrict__ table, const int32_t* __restrict__ ids,
                                                         int H, float* __restrict__ out) {
    const int t = blockIdx.x;
    const int64_t row = ids[t];
    float* o = out + (int64_t)t * H;
    for (int i = threadIdx.x * 4; i < H; i += 256 * 4) {
        float4 v;
        if constexpr (FMT == 2) {
            v = *(const float4*)((const float*)table + row * H + i);
        } else {
            const uint2 u = *(const uint2*)((const uint16_t*)table + row * H + i);
            const uint16_t h[4] = {(uint16_t)(u.x & 0xffffu), (uint16_t)(u.x >> 16), (uint16_t)(u.y & 0xffffu),
                                   (uint16_t)(u.y >> 16)};
            float f[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                f[j] = FMT == 0 ? __uint_as_float((uint32_t)h[j] << 16) : (float)__builtin_bit_cast(_Float16, h[j]);
            v = make_float4(f[0], f[1], f[2], f[3]);
        }
        *(float4*)(o + i) = v;
    }
}

// ------------------------------------------------------------ attention prep
// QK-RMSNorm over head_dim (:1202-1203), NEOX RoPE (:1205-1210), the permute/cont copies
// (:1212-1231) and the V transpose for the P.V MFMA: writes
//   qh [B][hq][n_pad][128], kh [B][hkv][n_pad][128]  (f16, rows >= n_tok zero)
//   vt [B][hkv][128][n_pad] (f16, key position permuted inside each 16-group: positions
//      4..7 <-> 8..11, the k order of the attention kernel's P^T operand)
// (per-token math and the key order: prep_math.h, shared with the QKV GEMM's fused epilogue)

// grid: (n_pad/64 token tiles, nq + nk + nv head slots, B).  Slot < nq: one q head; < nq+nk: one k
// head; else the V^T transpose of one kv head.  One workgroup = 64 tokens of one head.
__global__ void __launch_bounds__(256) attn_prep_kernel(PrepArgs a) {
    const int layer = blockIdx.z / a.B;
    const int b = blockIdx.z - layer * a.B;
    if (a.layers > 1) {  // PrepArgs::layers: this block's layer
        a.src += layer * a.src_layer;
        a.kh += layer * a.kh_layer;
        a.vt += layer * a.vt_layer;
        a.k_norm = a.k_norm_layers[layer];
    }
    const int n0 = blockIdx.x * 64;
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int nq = a.q_col >= 0 ? a.hq : 0;
    const int nk = a.k_col >= 0 ? a.hkv : 0;
    const int slot = blockIdx.y;
    if (slot < nq + nk) {
        const bool isq = slot < nq;
        const int head = isq ? slot : slot - nq;
        const float* w = isq ? a.q_norm : a.k_norm;
        const int col = (isq ? a.q_col : a.k_col) + head * 128;
        uint16_t* base = isq ? a.qh + ((int64_t)b * a.hq + head) * a.n_pad * 128
                             : a.kh + ((int64_t)b * a.hkv + head) * a.n_pad * 128;
        const int64_t plane = isq ? a.q_plane : a.k_plane;
        // lane: token sub = lane / 16 of the wave's group of 4, dims d..d+3 and d+64..d+67; 16-byte
        // loads, 8-byte f16 stores; rows >= n_tok are written as zeros
        const int sub = lane >> 4;
        const int d = (lane & 15) * 4;
#pragma unroll
        for (int t0 = wid * 4; t0 < 64; t0 += 16) {  // 4 groups of 4 tokens per wave
            const int n = n0 + t0 + sub;
            float4 x0 = make_float4(0.f, 0.f, 0.f, 0.f), x1 = x0;
            if (n < a.n_tok) {
                const float* row = a.src + ((int64_t)b * a.n_tok + n) * a.ld + col;
                x0 = *(const float4*)(row + d);
                x1 = *(const float4*)(row + 64 + d);
            }
            float y[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            const bool rope = a.rope_cos && n < a.n_tok;
            prep::head_row(y, w, d, a.eps, rope ? a.rope_cos + (int64_t)n * 64 + d : nullptr,
                           rope ? a.rope_sin + (int64_t)n * 64 + d : nullptr, base + (int64_t)n * 128, plane,
                           a.f8 ? (isq ? 1 : 2) : 0);
        }
        return;
    }
    if (a.v_col < 0) return;
    // V^T without an LDS round trip: lane = one d, a wave = 64 consecutive d (each token's row is
    // one coalesced 256-B load), 16 tokens per group -> two 16-B f16 stores per plane, in the
    // attention kernel's permuted key order
    const int hk = slot - nq - nk;
    const int d = (wid & 1) * 64 + lane;
    const float* vsrc = a.src + (int64_t)b * a.n_tok * a.ld + a.v_col + hk * 128 + d;
    uint16_t* vdst = a.vt + (((int64_t)b * a.hkv + hk) * 128 + d) * a.n_pad;
#pragma unroll
    for (int grp = 0; grp < 2; ++grp) {
        const int g0 = n0 + (wid >> 1) * 32 + grp * 16;
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const int n = g0 + prep::vperm(k);
            v[k] = n < a.n_tok ? vsrc[(int64_t)n * a.ld] : 0.f;
        }
        uint32_t wv[8], wl[8];
        prep::v_words(v, wv, wl);
        *(uint4*)(vdst + g0) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        *(uint4*)(vdst + g0 + 8) = make_uint4(wv[4], wv[5], wv[6], wv[7]);
        if (a.f8 && a.v_plane > 0) {
            float vn[16];
#pragma unroll
            for (int w = 0; w < 16; ++w) vn[w] = v[prep::vperm(w)];
            prep::v_store8(vn, vdst, a.v_plane, g0, 0xffffu);
        } else if (a.v_plane > 0) {
            *(uint4*)(vdst + a.v_plane + g0) = make_uint4(wl[0], wl[1], wl[2], wl[3]);
            *(uint4*)(vdst + a.v_plane + g0 + 8) = make_uint4(wl[4], wl[5], wl[6], wl[7]);
        }
    }
}

// ------------------------------------------------------------ masks
// patch-pooled key mask (:1433-1449) / encoder key mask, as an additive bias.
__global__ void key_bias_kernel(const int32_t* __restrict__ mask, int B, int frames, int patch, int nk, int nk_pad,
                                float* __restrict__ kbias) {
    const int64_t total = (int64_t)B * nk_pad;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(i / nk_pad);
        const int k = (int)(i % nk_pad);
        bool ok = k < nk;
        if (ok && mask) {
            bool any = false;
            for (int j = 0; j < patch; ++j) {
                const int f = k * patch + j;
                if (f < frames && mask[(int64_t)b * frames + f] != 0) any = true;
            }
            ok = any;
        }
        kbias[i] = ok ? 0.f : -INFINITY;
    }
}

// ------------------------------------------------------------ timestep
// build_timestep_freq (:1261-1284) for t[b] - r[b] (r optional; the second embedder
// takes timestep - timestep_r, :1421).
__global__ void timestep_freq_kernel(const float* __restrict__ t, const float* __restrict__ r, int B, int dim,
                                     float scale, float log_max, float* __restrict__ f) {
    const int b = blockIdx.x;
    const int half = dim / 2;
    float tv = t[b];
    if (r) tv = rn_sub(tv, r[b]);
    const float ts = rn_mul(tv, scale);
    // exp / cos / sin evaluated in double and rounded once: the correctly rounded f32 results, i.e. the values
    // any accurate f32 libm gives.  The sinusoid is the most ill-conditioned spot of the graph: arg reaches
    // ~1000, so one ulp of fr moves arg by ~6e-5 and the feature by as much; a 1-2 ulp device expf / cosf
    // put the timestep features ~1e-4 away from an accurate evaluation.
    for (int i = threadIdx.x; i < half; i += blockDim.x) {
        const float expo = rn_div(rn_mul(-log_max, (float)i), (float)half);
        const float fr = (float)exp((double)expo);
        const float arg = rn_mul(ts, fr);
        f[(int64_t)b * dim + i] = (float)cos((double)arg);
        f[(int64_t)b * dim + i + half] = (float)sin((double)arg);
    }
    if ((dim & 1) && threadIdx.x == 0) f[(int64_t)b * dim + dim - 1] = 0.f;
}

// small-M GEMV: one wave computes 4 output columns for all M rows.
// XF32: x arrives as f32 and is rounded to the act type in the kernel, after silu when silu_in — the values
// to_act_kernel would have written, so the pair (to_act, gemv) is one launch with the same bits.
template <bool F16, bool XF32 = false>
__global__ void __launch_bounds__(256) gemv_kernel(const void* __restrict__ xv_, int M, const uint16_t* __restrict__ W,
                                                   int N, int K, const float* __restrict__ bias, bool silu_out,
                                                   bool accumulate, float* __restrict__ y, bool silu_in = false) {
    const uint16_t* x = static_cast<const uint16_t*>(xv_);
    const float* xf32 = static_cast<const float*>(xv_);
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int n0 = (blockIdx.x * 4 + wid) * 4;
    if (n0 >= N) return;
    float acc[8][4];
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[m][c] = 0.f;
    for (int k = lane * 8; k < K; k += 512) {
        float wf[4][8];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint4 wv = *(const uint4*)(W + (int64_t)(n0 + c) * K + k);
            const uint16_t* ws = (const uint16_t*)&wv;
#pragma unroll
            for (int j = 0; j < 8; ++j) wf[c][j] = act_to_f32(F16, ws[j]);
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            if (m < M) {
                uint16_t xs[8];
                if constexpr (XF32) {
                    const float4 a0 = *(const float4*)(xf32 + (int64_t)m * K + k);
                    const float4 a1 = *(const float4*)(xf32 + (int64_t)m * K + k + 4);
                    const float xr[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
                    for (int j = 0; j < 8; ++j) xs[j] = to_act(F16, silu_in ? silu_f(xr[j]) : xr[j]);
                } else {
                    const uint4 xv = *(const uint4*)(x + (int64_t)m * K + k);
                    const uint16_t* xp = (const uint16_t*)&xv;
#pragma unroll
                    for (int j = 0; j < 8; ++j) xs[j] = xp[j];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float xf = act_to_f32(F16, xs[j]);
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[m][c] = fmaf(xf, wf[c][j], acc[m][c]);
                }
            }
        }
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        if (m < M) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                float v = wave_sum(acc[m][c]);
                if (lane == 0) {
                    if (bias) v = rn_add(v, bias[n0 + c]);
                    if (silu_out) v = silu_f(v);
                    float* yp = y + (int64_t)m * N + n0 + c;
                    *yp = accumulate ? rn_add(*yp, v) : v;
                }
            }
        }
    }
}

// AdaLN tables (:1469-1475): mod = scale_shift_table + timestep proj.
__global__ void layer_mods_kernel(const float* __restrict__ tables, const float* __restrict__ proj, int L, int B, int H,
                                  float* __restrict__ mod) {
    const int64_t total = (int64_t)L * B * 6 * H;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % H);
        int64_t r = i / H;
        const int j = (int)(r % 6);
        r /= 6;
        const int b = (int)(r % B);
        const int l = (int)(r / B);
        mod[i] = rn_add(tables[((int64_t)l * 6 + j) * H + c], proj[((int64_t)b * 6 + j) * H + c]);
    }
}

// output AdaLN (:1537-1543): (shift, scale) = out_table + (temb_t + temb_r).
__global__ void out_mods_kernel(const float* __restrict__ table, const float* __restrict__ tt, const float* __restrict__ tr,
                                int B, int H, float* __restrict__ om) {
    const int64_t total = (int64_t)B * 2 * H;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % H);
        const int j = (int)((i / H) % 2);
        const int b = (int)(i / (2 * H));
        const float temb = rn_add(tt[(int64_t)b * H + c], tr[(int64_t)b * H + c]);
        om[i] = rn_add(table[(int64_t)j * H + c], temb);
    }
}

__global__ void euler_kernel(float* __restrict__ xt, const float* __restrict__ v, int64_t n, float dt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        xt[i] = rn_sub(xt[i], rn_mul(v[i], dt));
}

// SDE step of the reference generation loop (acestep/mlx_dit/generate.py:183-192):
// x0 = xt - v*t ; xt = t_next*noise + (1 - t_next)*x0
__global__ void sde_kernel(float* __restrict__ xt, const float* __restrict__ v, const float* __restrict__ noise,
                           int64_t n, float t, float t_next) {
    const float keep = rn_sub(1.0f, t_next);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float x0 = rn_sub(xt[i], rn_mul(v[i], t));
        xt[i] = rn_add(rn_mul(t_next, noise[i]), rn_mul(keep, x0));
    }
}

// Test-only fault injection (ACE_MI_TEST_FAULT, DitEngine): x[r][c] += amp over one 16-row x 128-column
// tile, i.e. one row group of one GEMM output tile.  Exists to show that the parity checks fail on a
// localised error (tests/test_gpu_parity_strict.py); never launched unless that variable is set.
__global__ void fault_tile_kernel(float* __restrict__ x, int ld, int rows, int row0, int col0, float amp) {
    const int r = row0 + (int)(blockIdx.x * 8 + (threadIdx.x >> 7)), c = col0 + (int)(threadIdx.x & 127);
    if (r < rows) x[(int64_t)r * ld + c] = rn_add(x[(int64_t)r * ld + c], amp);
}

inline dim3 grid_for(int64_t n, int block = 256) {
    int64_t g = (n + block - 1) / block;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    return dim3((unsigned)g);
}

}  // namespace

void launch_pack_input(ActType t, const float* hidden, const float* context, int B, int T, int Np, int P,
                       int audio_dim, int ctx_dim, uint16_t* out, hipStream_t s, bool x3) {
    const int64_t n = (int64_t)B * Np * P * (audio_dim + ctx_dim);
    hipLaunchKernelGGL(pack_input_kernel, grid_for(n), dim3(256), 0, s, t == ActType::F16, x3, hidden, context, B, T,
                       Np, P, audio_dim, ctx_dim, out);
    ACEMI_HIP(hipGetLastError());
}

void launch_to_act(ActType t, const float* in, int64_t n, bool silu, uint16_t* out, hipStream_t s) {
    hipLaunchKernelGGL(to_act_kernel, grid_for(n), dim3(256), 0, s, t == ActType::F16, in, n, silu, out);
    ACEMI_HIP(hipGetLastError());
}

void launch_rmsnorm_mod(ActType t, const float* x, int M, int H, const float* w, const float* scale,
                        const float* shift, int64_t mod_stride, int rows_per_item, float eps, uint16_t* out,
                        hipStream_t s, bool x3) {
    ACEMI_CHECK(H % 4 == 0 && H <= 4096, "rmsnorm: H % 4 == 0 and H <= 4096");
    const bool f16 = t == ActType::F16;
    const int vpt = H <= 1024 ? 1 : (H <= 2048 ? 2 : 4);
#define ACEMI_RMS(F, V, X)                                                                                   \
    hipLaunchKernelGGL((rmsnorm_mod_kernel<F, V, X>), dim3(M), dim3(256), 0, s, x, H, w, scale, shift, mod_stride, \
                       rows_per_item, eps, out)
    // ACE_MI_RMSNORM_ROWS=1: wave-per-row kernel for H = 512 * NC.  Measured equal to the workgroup-per-row
    // kernel at 240 s (rocprof 9.4 vs 9.2 us per launch, 3.9 TB/s: the ~37 MB launch is ramp/tail bound), so
    // not the default.
    static const bool rows = [] {
        const char* e = std::getenv("ACE_MI_RMSNORM_ROWS");
        return e && e[0] == '1';
    }();
    // persistent kernel (default for H = 512 * NC, NC <= 4): ACE_MI_RMSNORM_PERSIST = workgroups per CU
    // (default 2; 0 = off)
    static const int persist = [] {
        const char* e = std::getenv("ACE_MI_RMSNORM_PERSIST");
        const int v = e ? std::atoi(e) : 2;
        return v < 0 ? 0 : std::min(v, 16);
    }();
    if (!x3 && persist > 0 && H % 512 == 0 && H <= 2048) {
        static int n_cu = 0;
        if (n_cu == 0) {
            int dev = 0;
            ACEMI_HIP(hipGetDevice(&dev));
            ACEMI_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
        }
        const dim3 g((unsigned)std::min<int64_t>((M + 3) / 4, (int64_t)n_cu * persist));
#define ACEMI_RMSP(F, NC)                                                                                         \
    hipLaunchKernelGGL((rmsnorm_mod_persist_kernel<F, NC>), g, dim3(256), 0, s, x, M, H, w, scale, shift, mod_stride, \
                       rows_per_item, eps, out)
        switch (H / 512) {
            case 1: if (f16) ACEMI_RMSP(true, 1); else ACEMI_RMSP(false, 1); break;
            case 2: if (f16) ACEMI_RMSP(true, 2); else ACEMI_RMSP(false, 2); break;
            case 3: if (f16) ACEMI_RMSP(true, 3); else ACEMI_RMSP(false, 3); break;
            default: if (f16) ACEMI_RMSP(true, 4); else ACEMI_RMSP(false, 4); break;
        }
#undef ACEMI_RMSP
        ACEMI_HIP(hipGetLastError());
        return;
    }
    if (!x3 && rows && H % 512 == 0 && H <= 4096) {
        const dim3 g((M + 3) / 4);
#define ACEMI_RMSR(F, NC) \
    hipLaunchKernelGGL((rmsnorm_mod_rows_kernel<F, NC>), g, dim3(256), 0, s, x, M, H, w, scale, shift, mod_stride, \
                       rows_per_item, eps, out)
        switch (H / 512) {
            case 1: if (f16) ACEMI_RMSR(true, 1); else ACEMI_RMSR(false, 1); break;
            case 2: if (f16) ACEMI_RMSR(true, 2); else ACEMI_RMSR(false, 2); break;
            case 3: if (f16) ACEMI_RMSR(true, 3); else ACEMI_RMSR(false, 3); break;
            case 4: if (f16) ACEMI_RMSR(true, 4); else ACEMI_RMSR(false, 4); break;
            case 5: if (f16) ACEMI_RMSR(true, 5); else ACEMI_RMSR(false, 5); break;
            case 6: if (f16) ACEMI_RMSR(true, 6); else ACEMI_RMSR(false, 6); break;
            case 7: if (f16) ACEMI_RMSR(true, 7); else ACEMI_RMSR(false, 7); break;
            default: if (f16) ACEMI_RMSR(true, 8); else ACEMI_RMSR(false, 8); break;
        }
#undef ACEMI_RMSR
        ACEMI_HIP(hipGetLastError());
        return;
    }
    if (x3) {
        if (vpt == 1) ACEMI_RMS(true, 1, true);
        else if (vpt == 2) ACEMI_RMS(true, 2, true);
        else ACEMI_RMS(true, 4, true);
    } else if (f16) {
        if (vpt == 1) ACEMI_RMS(true, 1, false);
        else if (vpt == 2) ACEMI_RMS(true, 2, false);
        else ACEMI_RMS(true, 4, false);
    } else {
        if (vpt == 1) ACEMI_RMS(false, 1, false);
        else if (vpt == 2) ACEMI_RMS(false, 2, false);
        else ACEMI_RMS(false, 4, false);
    }
#undef ACEMI_RMS
    ACEMI_HIP(hipGetLastError());
}

void launch_rmsnorm_f32(const float* x, int rows, int64_t row_step, int H, const float* w, float eps, float* out,
                        hipStream_t s) {
    ACEMI_CHECK(H % 4 == 0 && H <= 4096 && rows >= 1 && row_step >= 1, "rmsnorm_f32: bad shape");
    if (H <= 1024)
        hipLaunchKernelGGL(rmsnorm_f32_kernel<1>, dim3(rows), dim3(256), 0, s, x, row_step, H, w, eps, out);
    else if (H <= 2048)
        hipLaunchKernelGGL(rmsnorm_f32_kernel<2>, dim3(rows), dim3(256), 0, s, x, row_step, H, w, eps, out);
    else
        hipLaunchKernelGGL(rmsnorm_f32_kernel<4>, dim3(rows), dim3(256), 0, s, x, row_step, H, w, eps, out);
    ACEMI_HIP(hipGetLastError());
}

void launch_embed_rows(const void* table, int fmt, const int32_t* ids, int n, int H, float* out, hipStream_t s) {
    ACEMI_CHECK(H % 4 == 0 && n >= 1 && table && ids, "embed_rows: bad arguments");
    if (fmt == 0)
        hipLaunchKernelGGL(embed_rows_kernel<0>, dim3(n), dim3(256), 0, s, table, ids, H, out);
    else if (fmt == 1)
        hipLaunchKernelGGL(embed_rows_kernel<1>, dim3(n), dim3(256), 0, s, table, ids, H, out);
    else
        hipLaunchKernelGGL(embed_rows_kernel<2>, dim3(n), dim3(256), 0, s, table, ids, H, out);
    ACEMI_HIP(hipGetLastError());
}

void launch_sde(float* xt, const float* v, const float* noise, int64_t n, float t, float t_next, hipStream_t s) {
    hipLaunchKernelGGL(sde_kernel, grid_for(n), dim3(256), 0, s, xt, v, noise, n, t, t_next);
    ACEMI_HIP(hipGetLastError());
}

void launch_attn_prep(const PrepArgs& a, hipStream_t s) {
    ACEMI_CHECK(a.n_pad % 64 == 0, "attn_prep: n_pad % 64");
    const int slots = (a.q_col >= 0 ? a.hq : 0) + (a.k_col >= 0 ? a.hkv : 0) + (a.v_col >= 0 ? a.hkv : 0);
    ACEMI_CHECK(a.ld % 4 == 0 && (a.v_col < 0 || a.v_col % 4 == 0), "attn_prep: alignment");
    ACEMI_CHECK(a.layers >= 1 && (a.layers == 1 || (a.q_col < 0 && a.k_norm_layers && a.src_layer % 4 == 0)),
                "attn_prep: multi-layer launches are for k / v sections with a k-norm table");
    hipLaunchKernelGGL(attn_prep_kernel, dim3(a.n_pad / 64, slots, a.B * a.layers), dim3(256), 0, s, a);
    ACEMI_HIP(hipGetLastError());
}

void launch_key_bias(const int32_t* mask, int B, int frames, int patch, int nk, int nk_pad, float* kbias,
                     hipStream_t s) {
    const int64_t n = (int64_t)B * nk_pad;
    hipLaunchKernelGGL(key_bias_kernel, grid_for(n), dim3(256), 0, s, mask, B, frames, patch, nk, nk_pad, kbias);
    ACEMI_HIP(hipGetLastError());
}

void launch_timestep_freq(const float* t, const float* r, int B, int dim, float scale, float log_max, float* f,
                          hipStream_t s) {
    hipLaunchKernelGGL(timestep_freq_kernel, dim3(B), dim3(128), 0, s, t, r, B, dim, scale, log_max, f);
    ACEMI_HIP(hipGetLastError());
}

void launch_gemv_f32(ActType t, const float* x, bool silu_in, int M, const uint16_t* W, int N, int K,
                     const float* bias, bool silu_out, bool accumulate, float* y, hipStream_t s) {
    ACEMI_CHECK(M >= 1 && M <= 8, "gemv: M must be 1..8");
    ACEMI_CHECK(N % 16 == 0 && K % 8 == 0, "gemv: N % 16, K % 8");
    const dim3 grid(N / 16);
    if (t == ActType::F16)
        hipLaunchKernelGGL((gemv_kernel<true, true>), grid, dim3(256), 0, s, x, M, W, N, K, bias, silu_out, accumulate,
                           y, silu_in);
    else
        hipLaunchKernelGGL((gemv_kernel<false, true>), grid, dim3(256), 0, s, x, M, W, N, K, bias, silu_out,
                           accumulate, y, silu_in);
    ACEMI_HIP(hipGetLastError());
}

void launch_gemv(ActType t, const uint16_t* x_act, int M, const uint16_t* W, int N, int K, const float* bias,
                 bool silu_out, bool accumulate, float* y, hipStream_t s) {
    ACEMI_CHECK(M >= 1 && M <= 8, "gemv: M must be 1..8");
    ACEMI_CHECK(N % 16 == 0 && K % 8 == 0, "gemv: N % 16, K % 8");
    const dim3 grid(N / 16);
    if (t == ActType::F16)
        hipLaunchKernelGGL(gemv_kernel<true>, grid, dim3(256), 0, s, x_act, M, W, N, K, bias, silu_out, accumulate,
                           y);
    else
        hipLaunchKernelGGL(gemv_kernel<false>, grid, dim3(256), 0, s, x_act, M, W, N, K, bias, silu_out, accumulate,
                           y);
    ACEMI_HIP(hipGetLastError());
}

void launch_layer_mods(const float* tables, const float* proj, int n_layers, int B, int H, float* mod,
                       hipStream_t s) {
    const int64_t n = (int64_t)n_layers * B * 6 * H;
    hipLaunchKernelGGL(layer_mods_kernel, grid_for(n), dim3(256), 0, s, tables, proj, n_layers, B, H, mod);
    ACEMI_HIP(hipGetLastError());
}

void launch_out_mods(const float* out_table, const float* temb_t, const float* temb_r, int B, int H,
                     float* outmod, hipStream_t s) {
    const int64_t n = (int64_t)B * 2 * H;
    hipLaunchKernelGGL(out_mods_kernel, grid_for(n), dim3(256), 0, s, out_table, temb_t, temb_r, B, H, outmod);
    ACEMI_HIP(hipGetLastError());
}

void launch_fault_tile(float* x, int ld, int rows, int row0, int col0, float amp, hipStream_t s) {
    ACEMI_CHECK(row0 >= 0 && col0 >= 0 && col0 + 128 <= ld, "fault_tile: tile outside the matrix");
    hipLaunchKernelGGL(fault_tile_kernel, dim3(2), dim3(8 * 128), 0, s, x, ld, rows, row0, col0, amp);
    ACEMI_HIP(hipGetLastError());
}

struct PrefetchSet {
    const uint4* p[6];
    int64_t n16[6];  // 16-byte words per range
    int n;
};
__global__ void __launch_bounds__(256) prefetch_kernel(PrefetchSet ps, unsigned magic, unsigned* sink) {
    uint32_t acc = 0;
    for (int r = 0; r < ps.n; ++r) {
        const uint4* p = ps.p[r];
        const int64_t n = ps.n16[r];
        for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
            const uint4 v = p[i];
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == magic) sink[threadIdx.x & 63] = acc;  // (almost) never: keeps the loads
}

void launch_prefetch(const void* const* ptrs, const size_t* bytes, int n, int blocks, unsigned* sink, hipStream_t s) {
    ACEMI_CHECK(n >= 1 && n <= 6 && blocks >= 1, "prefetch: 1..6 ranges");
    PrefetchSet ps{};
    for (int i = 0; i < n; ++i) {
        ps.p[i] = static_cast<const uint4*>(ptrs[i]);
        ps.n16[i] = (int64_t)(bytes[i] / 16);
    }
    ps.n = n;
    hipLaunchKernelGGL(prefetch_kernel, dim3(blocks), dim3(256), 0, s, ps, 0x9e3779b9u, sink);
    ACEMI_HIP(hipGetLastError());
}

void launch_euler(float* xt, const float* v, int64_t n, float dt, hipStream_t s) {
    hipLaunchKernelGGL(euler_kernel, grid_for(n), dim3(256), 0, s, xt, v, n, dt);
    ACEMI_HIP(hipGetLastError());
}

}  // namespace acemi
