/* Kernel self-test and micro-benchmark entries of the TEST library libacestep_mi355x_selftest.so (the product
 * library's objects + csrc/runtime/selftest.cpp; Makefile target `selftest`).  Not part of the product
 * library libacestep_mi355x.so: the -m gpu parity tests and tools/ call single gfx950 kernels through these on
 * host buffers (blocking) and compare them with fp64 / fp32 references of the same op. */
#ifndef ACESTEP_MI355X_SELFTEST_H
#define ACESTEP_MI355X_SELFTEST_H

#include "acestep_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- kernel self-test entries (blocking, host buffers; used by the -m gpu parity tests) ----
 * GEMM: C = A[M][K] . W[N][K]^T with A, W raw 16-bit words of act_type (0 bf16, 1 fp16).
 * epi 0: out_f32[M][N] = C (+ bias[N] if bias != NULL);
 * epi 4: SwiGLU on 16-column interleaved gate|up weights, out_u16[M][N/2] raw act words;
 * epi 3 / 2: residual update in place, out_f32[M][N] holds x on entry: x += C (epi 3) or
 * x += C * gate[N] (epi 2, the gate passed in `bias`). */
ACE_GGML_API ace_ggml_status ace_mi_kernel_gemm(int32_t act_type, int32_t epi, int32_t M, int32_t N, int32_t K,
                                                const uint16_t* A, const uint16_t* W, const float* bias,
                                                float* out_f32, uint16_t* out_u16);
/* Attention core only (no norm/RoPE): q [B][nq][Hq*128] f32, kv [B][nk][2*Hkv*128] f32 (K then V),
 * kmask [B][nk] int32 or NULL, window > 0 = sliding |q-k| <= window; `split` is a flag word: bit 0 =
 * hi/lo fp16 operands (default engine mode; clear = single fp16), bit 1 = causal (key k > query q
 * masked); out [B][nq][Hq*128] f32 (the kernel's bf16 output widened). */
ACE_GGML_API ace_ggml_status ace_mi_kernel_attention(int32_t B, int32_t Hq, int32_t Hkv, int32_t nq, int32_t nk,
                                                     int32_t window, float scale, int32_t split, const float* q,
                                                     const float* kv, const int32_t* kmask, float* out);

/* Attention micro-benchmark on pseudo-random device operands (fixed seed): average ms per launch (HIP
 * events) of the engine's attention kernel; flags bit 0 = hi/lo operands, bit 1 = causal, bit 2 = a
 * key-padding mask (every 7th key masked). */
ACE_GGML_API ace_ggml_status ace_mi_bench_attention(int32_t B, int32_t Hq, int32_t Hkv, int32_t nq, int32_t nk,
                                                    int32_t window, int32_t flags, int32_t iters, float* avg_ms);

/* GEMM micro-benchmark on random device operands: average ms per launch (HIP events) of the
 * engine's GEMM for act_type (0 bf16, 1 fp16), epilogue `epi` (0 f32 store, 2 gated residual,
 * 4 SwiGLU), kernel `variant` (-1 automatic, 0..9 forced: 128x128 two pipelines, 256x256, 256x128, 192x128, 192x256, 192x64, 96x128, 64x128, 64x64). */
ACE_GGML_API ace_ggml_status ace_mi_bench_gemm(int32_t act_type, int32_t epi, int32_t variant, int32_t M, int32_t N,
                                               int32_t K, int32_t iters, float* avg_ms);
/* Dequant-fused GEMM on ggml block rows W [N][K]: out = A . bf16(dequant(W))^T (+ bias), A bf16 [M][K];
 * epi 0 (f32 store) or 4 (SwiGLU, bf16 out [M][N/2]); variant -1 automatic, 0..7 forced (round 1's ds_write
 * dequant tiles; 6 and 8..11 are dense-only), 20..24 the LDS-DMA dequant tiles (+ 100 S: split-K). */
ACE_GGML_API ace_ggml_status ace_mi_kernel_gemm_q(int32_t qtype, int32_t epi, int32_t variant, int32_t M, int32_t N,
                                                  int32_t K, const uint16_t* A, const uint8_t* W_blocks,
                                                  const float* bias, float* out_f32, uint16_t* out_u16);
/* Staged dequant kernel (the bf16 weight image the DiT's staged-dequant ring multiplies): out = bf16 bits of
 * bf16(dequant(W)) [N][K] for ggml block rows W [N][K]. */
ACE_GGML_API ace_ggml_status ace_mi_kernel_dequant(int32_t qtype, int32_t N, int32_t K, const uint8_t* W_blocks,
                                                   uint16_t* out);
/* ggml-faithful quantized-activation GEMM (ACE_MI_QUANT_ACT=q8): x f32 [M][K] quantized on the device to Q8_0
 * (Q8_0 weights) or Q8_K (K-quants) blocks -- returned as q_out int8 [M][K], s_out f32 [K/32][M] (block scale d),
 * bsum_out f32 [K/32][M] (sum of q per 32, Q8_K) when non-null -- then ggml's per-block integer dot products against
 * the ggml block rows W [N][K].  epi 0: out [M][N] = acc (+ bias); 3: out += acc (+ bias); 7: out [M][N/2] =
 * silu(g) * u (gate|up interleaved in 16-column groups). */
ACE_GGML_API ace_ggml_status ace_mi_kernel_gemm_a8(int32_t qtype, int32_t epi, int32_t M, int32_t N, int32_t K,
                                                   const float* x, const uint8_t* W_blocks, const float* bias,
                                                   float* out_f32, int8_t* q_out, float* s_out, float* bsum_out);
/* The form ace_mi_kernel_gemm_a8 and the q8 mode of this process run Q8_0 GEMMs in (K % 64 == 0): -1 = the
 * environment (ACE_MI_QACT_GEMM=0: i8) / default (bf16 MFMA over exact integer bf16 operands), 0 = the i8-MFMA kernel,
 * 1 = the bf16-MFMA kernel.  Both give the same bits. */
ACE_GGML_API ace_ggml_status ace_mi_kernel_gemm_a8_mode(int32_t mode);
/* The kernel that runs f8c attention in this process: -1 = the environment (ACE_MI_ATTN_KH=0 / 1) / default policy
 * (the two-waves-per-SIMD kernel for blocks of >= 16 key tiles), 0 = the one-wave-per-SIMD kernel, 1 = the two-wave
 * kernel everywhere.  Same results within the f8c bound. */
ACE_GGML_API ace_ggml_status ace_mi_kernel_attn_kh(int32_t mode);
/* Dequant-fused GEMM micro-benchmark: average ms per launch (HIP events). */
ACE_GGML_API ace_ggml_status ace_mi_bench_gemm_q(int32_t qtype, int32_t epi, int32_t variant, int32_t M, int32_t N,
                                                 int32_t K, int32_t iters, float* avg_ms);

#ifdef __cplusplus
}
#endif

#endif /* ACESTEP_MI355X_SELFTEST_H */
