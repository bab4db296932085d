// Host-side launch wrappers for the gfx950 kernels (all stream-ordered, no
// allocation, no synchronisation: safe to capture into a hipGraph).
#pragma once

#include <cstdlib>
#include <stdexcept>
#include <string>

#include "common.h"

namespace acemi {

// Per-head RMSNorm (+ NEOX RoPE) of the q/k sections and f16 re-layout for attention.
struct PrepArgs {
    const float* src;
    int ld;
    int q_col, k_col, v_col;  // -1: section absent
    int hq, hkv;
    int n_tok, n_pad, B;
    const float* q_norm;
    const float* k_norm;
    const float* rope_cos;  // [n_tok][64] or null
    const float* rope_sin;
    float eps;
    uint16_t* qh;
    uint16_t* kh;
    uint16_t* vt;
    int64_t q_plane = 0, k_plane = 0, v_plane = 0;  // >0: also write lo = f16(x - f16(x)) planes
    int f8 = 0;  // 1: the lo planes hold the fp8 operands of the f8c attention mode instead (prep_math.h)
    // > 1 (k / v sections only): one launch for `layers` consecutive layers, layer l reading src + l*src_layer,
    // writing kh + l*kh_layer / vt + l*vt_layer, normalising by k_norm_layers[l] (a device table)
    int layers = 1;
    int64_t src_layer = 0, kh_layer = 0, vt_layer = 0;
    const float* const* k_norm_layers = nullptr;
};

// ---------------------------------------------------------------- GEMM
// C[M][N] = A[M][K] . W[N][K]^T   (A, W: 16-bit act type, f32 accumulate)
// followed by a fused epilogue.  N % 128 == 0, K % 64 == 0, M >= 1.
enum GemmEpiKind : int {
    EPI_STORE_F32 = 0,      // c_f32[m*ldc+n] = acc (+ bias[n])
    EPI_STORE_ACT = 1,      // c_act[m*ldc+n] = act(acc (+ bias[n]))
    EPI_RESID_GATED = 2,    // c_f32[m*ldc+n] += acc * gate[(m / rows_per_item)*gate_stride + n]
    EPI_RESID = 3,          // c_f32[m*ldc+n] += acc
    EPI_SWIGLU = 4,         // columns interleaved [g0..15,u0..15,g16..]: c_act[m*ldc + n'] = act(silu(g)*u)
    EPI_PROJ_OUT = 5,       // c_f32[b][2p+k][c] = acc[m=(b,p)][n = c + k*out_ch] + bias[c], cropped to T
    EPI_QKV_PREP = 6,       // attn_prep fused: column tile n0/128 = one head of [q heads | k heads | v heads]
                            // (sections present per prep.q_col / k_col / v_col >= 0), written straight into
                            // the attention layouts of `prep` (QK-RMSNorm, RoPE, fp16 hi/lo, V^T); 128-wide
                            // column tiles only, no bias
    EPI_SWIGLU_F32 = 7,     // EPI_SWIGLU with an f32 output c_f32 (the quantized-activation GEMM only)
};

struct GemmEpilogue {
    int kind = EPI_STORE_F32;
    const float* bias = nullptr;
    float* c_f32 = nullptr;
    uint16_t* c_act = nullptr;
    int ldc = 0;
    const float* gate = nullptr;
    int64_t gate_stride = 0;
    int rows_per_item = 1;
    int out_T = 0;        // EPI_PROJ_OUT: frames per item
    int out_ch = 0;       // EPI_PROJ_OUT: channels (64)
    int patch = 2;        // EPI_PROJ_OUT
    PrepArgs prep{};      // EPI_QKV_PREP (src / ld unused)
};

// Weight operand.  Dense: 16-bit [N][ld] in the activation type.  Quantized (ggml block formats
// re-laid out at load, runtime/quant.h): q = int8 / nibble plane, s = f32 scales; the kernel
// dequantizes each 32-value block to bf16 while staging it into LDS and multiplies it with a bf16
// activation (`Q -> bf16 dequant-fused` MFMA GEMM).
// WF_F32X3: an F32 weight as the fp16 triple [hi | lo | hi] along K (ld = 3K), multiplied with an
// activation written as [hi | hi | lo] (Ah.Wh + Ah.Wl + Al.Wh) by the plain fp16 GEMM over 3K.
enum WeightFormat : int { WF_BF16 = 0, WF_F16 = 1, WF_Q8_0 = 2, WF_Q4_K = 3, WF_Q6_K = 4, WF_F32X3 = 5 };
struct WeightView {
    int fmt = WF_BF16;
    const void* q = nullptr;   // dense uint16 [N][ld] | Q8_0/Q6_K int8 [N][K] | Q4_K u8 [N][K/2]
    const float* s = nullptr;  // Q8_0 [N][K/32] | Q4_K [N][K/32][2] (d*sc, dmin*m) | Q6_K [N][K/16]
    int ld = 0;                // dense leading dimension (elements)
};
inline ActType weight_act(int fmt) { return (fmt == WF_F16 || fmt == WF_F32X3) ? ActType::F16 : ActType::BF16; }
inline bool weight_quantized(int fmt) { return fmt >= WF_Q8_0; }

void launch_gemm(const uint16_t* A, int lda, const WeightView& W, int M, int N, int K, const GemmEpilogue& epi,
                 hipStream_t s);
// dense shorthand: W 16-bit of type t
void launch_gemm(ActType t, const uint16_t* A, int lda, const uint16_t* W, int ldw, int M, int N, int K,
                 const GemmEpilogue& epi, hipStream_t s);
// -1 = automatic tile choice; 0..11 force a kernel variant, + 100 * S (S = 2..4) split-K over S blocks per
// tile for the 4-wave tiles (micro-benchmarks / tests)
void gemm_force_variant(int v);
// Throws (once) if a split-K GEMM join on the current device timed out since the last check: reads a per-device
// host-pinned error word, no stream is synchronised (called at the library's synchronisation points and on entry).
void gemm_splitk_check();
// free the split-K workspace of stream s on the current device (before the owner destroys s)
void gemm_splitk_release(hipStream_t s);
// bf16 image [N][K] (ld K) of a quantized weight: bit-identical to what the dequant-fused GEMM feeds its MFMAs
void launch_dequant_bf16(const WeightView& W, int N, int K, uint16_t* out, hipStream_t s);
// the same for 1..8 matrices of one format in one launch
struct DequantJob {
    WeightView w;
    int N = 0, K = 0;
    uint16_t* out = nullptr;
};
void launch_dequant_bf16_batch(const DequantJob* jobs, int n, hipStream_t s);

// ------------------------------------------------- ggml-faithful quantized activations (kernels/gemm_a8.hip)
// ggml's mul_mat against a quantized weight first converts the f32 activation rows to the weight's vec_dot_type
// (Q8_0 blocks for Q8_0 weights, Q8_K for K-quants) and takes integer dot products per block
// (ggml-metal-embed.metal:222-227, 3110-3128; ggml-cpu quantize_row_q8_0 / quantize_row_q8_K_ref / vec_dot_*).
// ACE_MI_QUANT_ACT=q8 runs the DiT that way (DitEngine::forward_qact).
// Activation blocks on the device: q int8 [M][K]; s f32 [K/32][ld_s] per 32-value block (Q8_0: fp16(d);
// Q8_K: the 256-block's d in each of its eight 32-blocks); bsum f32 [K/32][ld_s] = sum of the block's q (Q8_K
// only: the Q4_K min term).  ld_s >= M rounded up to 128 (the GEMM reads whole 128-row tiles of s / bsum).
enum QActKind : int { QACT_Q8_0 = 0, QACT_Q8_K = 1 };
struct QAct {
    int kind = QACT_Q8_0;
    const int8_t* q = nullptr;
    const uint16_t* q16 = nullptr;  // Q8_0: bf16(q) [M][K] (exact integers) for the bf16-MFMA form of the GEMM
    const float* s = nullptr;
    const float* bsum = nullptr;
    int64_t ld_s = 0;
};
inline int qact_kind_for(int weight_fmt) { return weight_fmt == WF_Q8_0 ? QACT_Q8_0 : QACT_Q8_K; }
// x f32 [M][ldx] (silu first when silu_in) -> the blocks of `kind` in q / s / bsum (layout above)
// (q16: Q8_0 only, bf16(q) rows as well / instead -- either output may be null, not both)
void launch_quantize_act(int kind, const float* x, int64_t ldx, int M, int K, bool silu_in, int8_t* q, float* s,
                         float* bsum, int64_t ld_s, hipStream_t st, uint16_t* q16 = nullptr);
// C = dequant(A blocks) . dequant(W)^T with ggml's per-block integer dot products (v_mfma_i32_16x16x32_i8) and an
// f32 sum of d_w * d_a * isum over the blocks; W quantized (WF_Q8_0 with QACT_Q8_0, WF_Q4_K / WF_Q6_K with
// QACT_Q8_K); the epilogues of launch_gemm plus EPI_SWIGLU_F32 (a bias on EPI_RESID adds to the product first).
// N % 128 == 0, K % 32 (Q8_0) / % 256 (K-quants) == 0.
// With a.q16 and w16 (the bf16(q) image of W's int8 plane, launch_q8_image) a Q8_0 GEMM runs on the bf16 MFMA
// (gemm_a8s_kernel: each 32-value block's integer dot is exact there; same bits as the i8 kernel), K % 64 == 0.
void launch_gemm_a8(const QAct& a, const WeightView& W, int M, int N, int K, const GemmEpilogue& epi, hipStream_t s,
                    const uint16_t* w16 = nullptr);
// int8 plane [n] -> bf16 image [n] (exact integers), n % 16 == 0
void launch_q8_image(const int8_t* q, int64_t n, uint16_t* out, hipStream_t s);
// whether the q8 mode runs a GEMM with this weight format / depth on the bf16 MFMA: ACE_MI_QACT_GEMM=0 (or
// gemm_a8_mode(0)) keeps every one on the i8 kernel; gemm_a8_mode(-1) = the environment / default (on)
bool gemm_a8_bf16_path(int fmt, int K);
void gemm_a8_mode(int mode);
// launch_rmsnorm_mod's operator with an f32 output [M][H]
void launch_rmsnorm_mod_f32(const float* x, int M, int H, const float* w, const float* scale, const float* shift,
                            int64_t mod_stride, int rows_per_item, float eps, float* out, hipStream_t s);
// launch_pack_input's packing with f32 output [B*Np][P*Cin]
void launch_pack_input_f32(const float* hidden, const float* context, int B, int T, int Np, int P, int audio_dim,
                           int ctx_dim, float* out, hipStream_t s);

// ------------------------------------------------------------ attention
// Flash-style fp16 attention, f32 softmax/accumulate.  D = 128.
// Qh [B][Hq][nq_pad][128] f16, Kh [B][Hkv][nk_pad][128] f16,
// Vt [B][Hkv][128][nk_pad] f16 (keys permuted within groups of 16, see ops.hip),
// kbias [B][nk_pad] f32 additive (0 / -inf) or null, out act [B*nq][Hq*128].
struct AttnArgs {
    const uint16_t* q;
    const uint16_t* k;
    const uint16_t* vt;
    const float* kbias;
    uint16_t* out;
    int B, Hq, Hkv;
    int nq, nq_pad, nk, nk_pad;
    int window;  // >0: bidirectional sliding window |q-k| <= window
    bool causal = false;  // key k > query q masked (Qwen3 text encoder)
    float scale;
    bool split = true;                 // hi/lo fp16 Q.K operands (see attention.hip)
    bool pv_split = false;             // hi/lo fp16 P.V operands too (needs split)
    int64_t q_plane = 0, k_plane = 0, v_plane = 0;  // element offset of the lo planes
    // Optional f32 workspace of attn_part_floats(): with it, a grid too small to fill the chip in whole rounds
    // splits block key ranges in two or four parts, merged by attn_merge_kernel.
    float* part = nullptr;
    int ksplit = 1;  // set by launch_attention
    int xcd_order = 1;  // set by launch_attention: XCD-aware block order
    int split_from = 0;  // set by launch_attention: > 0 = tail split (blocks [0, split_from) whole, the rest in two
                         // key-range parts; ksplit = 2 gives the partials' layout)
    // f32 output [B*nq][Hq*128] instead of `out` (the ggml-faithful quantized-activation mode, whose next linear
    // quantizes the f32 rows), under the same key-split policy: whole blocks and the merges write f32 rows
    float* out_f32 = nullptr;
    bool f8 = false;  // f8c mode (needs split + pv_split): the lo planes hold fp8 hi / lo operands (prep_math.h), the
                      // correction products Kl.Qh + Kh.Ql and Vl.Ph + Vh.Pl run as block-scaled fp8 MFMAs
};
size_t attn_part_floats(int B, int nq, int Hq);
// Which kernel runs the f8c mode: -1 = ACE_MI_ATTN_KH (0 never, 1 always) / default (attn_kh_kernel, two waves per
// SIMD, for blocks of >= 16 key tiles; attn2 below that), 0 = attn2 always, 1 = attn_kh_kernel always
void attn_kh_mode(int mode);
// Operand precision of the attention MFMAs: FP16 = single fp16 operands (two workgroups per CU),
// SPLIT = hi/lo fp16 Q.K (three MFMAs per product) with fp16 P.V, F32 = hi/lo fp16 for both products
// (~22-bit operands, the f32-faithful mode), F8C = hi/lo for both products with the two correction products as
// block-scaled e4m3 MFMAs (hi x hi in fp16, Kl.Qh + Kh.Ql and Vl.Ph + Vh.Pl at e4m3 precision: ~2^-15 relative
// per product instead of F32's ~2^-22, at 2/3 of F32's matrix-core time).  ACE_MI_ATTN_PRECISION=fp16|split|f32 overrides `dflt`;
// the legacy ACE_MI_ATTN_FAST=1 means fp16.
// PV8 = fp16 Q.K with F8C's hi/lo P.V (the P.V roundings carry most of fp16 attention's excess over the f32 graph;
// measured in tests/test_gpu_parity_strict.py), 3/4 of F8C's matrix-core time.
enum class AttnPrecision { FP16, SPLIT, F32, F8C, PV8 };
inline AttnPrecision attn_precision_from_env(AttnPrecision dflt) {
    const char* f = std::getenv("ACE_MI_ATTN_FAST");
    if (f && f[0] && f[0] != '0') return AttnPrecision::FP16;
    const char* e = std::getenv("ACE_MI_ATTN_PRECISION");
    if (!e || !e[0]) return dflt;
    const std::string v(e);
    if (v == "fp16") return AttnPrecision::FP16;
    if (v == "split") return AttnPrecision::SPLIT;
    if (v == "f32") return AttnPrecision::F32;
    if (v == "f8c") return AttnPrecision::F8C;
    if (v == "pv8") return AttnPrecision::PV8;
    throw std::runtime_error("ACE_MI_ATTN_PRECISION must be fp16, split, f32, f8c or pv8");
}
void launch_attention(ActType out_t, const AttnArgs& a, hipStream_t s);

// ------------------------------------------------------------ elementwise
// Pack [context | hidden] frames into patches: out act [B*Np][P*Cin].
// x3: write the f32 value as the fp16 triple [hi | hi | lo] per row (input of a WF_F32X3 weight).
void launch_pack_input(ActType t, const float* hidden, const float* context, int B, int T, int Np, int P,
                       int audio_dim, int ctx_dim, uint16_t* out, hipStream_t s, bool x3 = false);
// f32 -> act conversion (row-major copy), optionally act(silu(x)).
void launch_to_act(ActType t, const float* in, int64_t n, bool silu, uint16_t* out, hipStream_t s);
// y = act( RMSNorm(x) * w * (1 + scale) + shift ); scale/shift optional, per item
// (item = row / rows_per_item, stride mod_stride floats).
void launch_rmsnorm_mod(ActType t, const float* x, int M, int H, const float* w, const float* scale,
                        const float* shift, int64_t mod_stride, int rows_per_item, float eps, uint16_t* out,
                        hipStream_t s, bool x3 = false);
// out[r] = RMSNorm(x[r * row_step]) * w in f32 for r < rows (the condition encoders' final norm,
// acestep_dit_model.cpp:1642-1644 / :1727-1729; row_step > 1 picks every item's first token).
void launch_rmsnorm_f32(const float* x, int rows, int64_t row_step, int H, const float* w, float eps, float* out,
                        hipStream_t s);
// out[t] = f32(table[ids[t]]) for t < n (ggml_get_rows + cast_f32, qwen_model.cpp:563-564):
// table [rows][H] as bf16 (fmt 0), fp16 (1) or f32 (2) values.
void launch_embed_rows(const void* table, int fmt, const int32_t* ids, int n, int H, float* out, hipStream_t s);
void launch_attn_prep(const PrepArgs& a, hipStream_t s);
// kbias[b][k] = (k < nk && pooled mask) ? 0 : -inf ; mask [B][nk*patch-ish frames] or null.
void launch_key_bias(const int32_t* mask, int B, int frames, int patch, int nk, int nk_pad, float* kbias,
                     hipStream_t s);
// Sinusoidal timestep features f[b][256] of t[b] - (r ? r[b] : 0) (acestep_dit_model.cpp:1261-1284).
// log_max = logf(10000) evaluated on the host exactly as the reference does.
void launch_timestep_freq(const float* t, const float* r, int B, int dim, float scale, float log_max, float* f,
                          hipStream_t s);
// Small-M GEMV (timestep MLPs): v = sum_k x_act[m][k] W[n][k] + bias[n]; v = silu(v) if silu_out;
// y[m][n] = accumulate ? y[m][n] + v : v.  M <= 8, K % 512 == 0.
void launch_gemv(ActType t, const uint16_t* x_act, int M, const uint16_t* W, int N, int K, const float* bias,
                 bool silu_out, bool accumulate, float* y, hipStream_t s);
// Same with f32 x rounded to the act type in the kernel (after silu when silu_in): launch_to_act + launch_gemv
// in one launch, same bits.
void launch_gemv_f32(ActType t, const float* x, bool silu_in, int M, const uint16_t* W, int N, int K,
                     const float* bias, bool silu_out, bool accumulate, float* y, hipStream_t s);
// mod[l][b][j][c] = table[l][j][c] + proj[b][j*H + c]  (j < 6)
void launch_layer_mods(const float* tables, const float* proj, int n_layers, int B, int H, float* mod,
                       hipStream_t s);
// outmod[b][j][c] = out_table[j][c] + (temb_t[b][c] + temb_r[b][c]) (j < 2)
void launch_out_mods(const float* out_table, const float* temb_t, const float* temb_r, int B, int H,
                     float* outmod, hipStream_t s);
// TEST ONLY (fault injection for the parity negative control): x[r][c] += amp for r in [row0, row0 + 16),
// c in [col0, col0 + 128)
void launch_fault_tile(float* x, int ld, int rows, int row0, int col0, float amp, hipStream_t s);
// Test-only hooks (runtime/test_hooks.cpp): read from the environment in the self-test library only; the product
// library's versions return "off"
bool test_fault_from_env(int& layer, int& row, int& col, float& amp);
bool test_vae_fault_from_env(int& block, int& row, int& col, float& amp);
int gemm_override_from_env(int N, int K);
// xt -= v * dt
void launch_euler(float* xt, const float* v, int64_t n, float dt, hipStream_t s);
// Read-only sweep of up to 6 device ranges (weights of the next layer) on a side stream, so they sit in the
// memory-side cache (MALL) when the layer's GEMMs read them; `blocks` workgroups.  Nothing is written except
// one word of `sink` in a case that never occurs (keeps the loads).
void launch_prefetch(const void* const* ptrs, const size_t* bytes, int n, int blocks, unsigned* sink, hipStream_t s);
// SDE re-noise step: xt = t_next * noise + (1 - t_next) * (xt - v * t)
void launch_sde(float* xt, const float* v, const float* noise, int64_t n, float t, float t_next, hipStream_t s);

// ------------------------------------------------------------ VAE decoder (kernels/vae.hip)
// Implicit-GEMM conv on fp16 time-major activations.  A row (m, tap) = S[m + tap*dil - pad]
// (zero row outside [0, T_in)); W [N][taps*Cin] fp16.  up == 1: conv, (m, n) -> (u = m, co = n);
// up = s > 1: transposed conv, n = r*Cout + co -> u = s*m + r - crop.  Epilogue on v = acc + bias:
// resid: v = X[u][co] + v; store_x: X[u][co] = v; S_out: S_out[u][co] = f16(snake(v)) (or f16(v)
// when snake_ea is null).
struct ConvGemmArgs {
    const uint16_t* S = nullptr;
    const uint16_t* zero = nullptr;
    const uint16_t* W = nullptr;
    int T_in = 0, Cin = 0, taps = 1, dil = 1, pad = 0;
    int in_stride = 1;  // strided conv: A row (m, tap) = S[m*in_stride + tap*dil - pad]
    int M = 0, N = 0;
    const float* bias = nullptr;
    int Cout = 0, up = 1, crop = 0, T_out = 0;
    float* X = nullptr;
    int resid = 0, store_x = 0;
    uint16_t* S_out = nullptr;
    const float* snake_ea = nullptr;
    const float* snake_eb = nullptr;
    // independent sequences in one launch (windows of the tiled decode): the M rows split into
    // `items` equal runs; S is [items][T_in][Cin], X / S_out are [items][T_out][Cout]
    int items = 1;
    // Fused second conv of a residual unit (residual_forward, acestep_vae_model.cpp:724-733) when
    // Cout = N = 128: the tile's conv output y = Snake2(acc + bias) goes through LDS as fp16 into
    // z = y . W2^T + bias2 (the k1 conv), and the residual / store / S_out epilogue applies to z.
    const uint16_t* W2 = nullptr;  // [Cout][Cout] fp16
    const float* bias2 = nullptr;
    const float* snake2_ea = nullptr;
    const float* snake2_eb = nullptr;
};
void launch_conv_gemm(const ConvGemmArgs& a, hipStream_t s);
void launch_to_f16(const float* x, int64_t n, uint16_t* y, hipStream_t s);
// x [rows][C] f32 -> y [rows][Cpad] fp16, channels >= C zero
void launch_pack_f16(const float* x, int64_t rows, int C, int Cpad, uint16_t* y, hipStream_t s);
// out[t][o] = sum_k sum_c W[o][k][c] * S[t + k - 3][c]   (kernel 7, pad 3, no bias), f32 out
// (items sequences of T rows each: S [items][T][C], out [items][T][out_ch])
void launch_conv_out(const uint16_t* S, int T, int C, const uint16_t* W, int out_ch, float* out, hipStream_t s,
                     int items = 1);

}  // namespace acemi
