/*
 * MI355X extensions of the ACE-Step DiT C-ABI (libacestep_mi355x.so).
 *
 * These add what the reference ABI cannot express (SURVEY §8b "What the
 * build adds"): a device-pointer, batched, stream-ordered forward that
 * removes the per-step host round trip and the serial per-item loop of
 * scripts/run_non_ggml_real_case.py:502-529, and a device-resident Euler
 * sampler equivalent to the C sampler loop acestep_ggml.cpp:2042-2086.
 * All pointers named d_* are HIP device pointers on the context's device;
 * `stream` is a hipStream_t (NULL = the context's own stream).  Calls are
 * asynchronous with respect to the host unless stated otherwise.
 */
#ifndef ACESTEP_MI355X_H
#define ACESTEP_MI355X_H

#include "acestep_ggml.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ace_mi_dit_info {
    int32_t hidden_size;
    int32_t intermediate_size;
    int32_t num_layers;
    int32_t num_heads;
    int32_t num_kv_heads;
    int32_t head_dim;
    int32_t patch_size;
    int32_t in_channels;
    int32_t audio_dim;
    int32_t sliding_window;
    int32_t act_type;       /* 0 = bf16, 1 = fp16 */
    int32_t device;
    int64_t weight_bytes;
} ace_mi_dit_info;

/* Like ace_ggml_create, bound to HIP device `device`. */
ACE_GGML_API ace_ggml_status ace_mi_create_on_device(const ace_ggml_init_params* params, int32_t device,
                                                     ace_ggml_context** out_ctx);

/* Model dimensions of the loaded DiT (ACE_GGML_ERR "dit not loaded" otherwise). */
ACE_GGML_API ace_ggml_status ace_mi_dit_get_info(ace_ggml_context* ctx, ace_mi_dit_info* out);

/* One denoising step for `batch` samples sharing (seq_len, enc_len).
 * d_hidden [B][T][audio], d_context [B][T][in-audio] (either may be NULL = zeros),
 * d_enc [B][L][hidden] (NULL only if enc_len == 0), d_mask [B][T] / d_enc_mask [B][L] int32
 * (NULL = all valid), d_timestep / d_timestep_r [B] f32, d_out [B][T][audio] f32.
 * Result equals `batch` calls of ace_ggml_dit_forward. */
ACE_GGML_API ace_ggml_status ace_mi_dit_forward_batched(ace_ggml_context* ctx, int32_t batch, const float* d_hidden,
                                                        const float* d_context, const float* d_enc,
                                                        const int32_t* d_mask, const int32_t* d_enc_mask,
                                                        int32_t seq_len, int32_t enc_len, const float* d_timestep,
                                                        const float* d_timestep_r, float* d_out, void* stream);

/* Euler ODE sampling on the device (acestep_ggml.cpp:2056-2086, mlx_dit/generate.py:154-197):
 * for i in steps: v = DiT(xt, t_i, r = t_i); xt -= v * (t_i - t_{i+1}); last step xt -= v * t_i.
 * d_xt [B][T][audio] holds the initial noise on entry and x0 on return.
 * `schedule` is a HOST array of n_steps timesteps. */
ACE_GGML_API ace_ggml_status ace_mi_dit_sample(ace_ggml_context* ctx, int32_t batch, float* d_xt,
                                               const float* d_context, const float* d_enc, const int32_t* d_mask,
                                               const int32_t* d_enc_mask, int32_t seq_len, int32_t enc_len,
                                               const float* schedule, int32_t n_steps, void* stream);
/* The Python/MLX generation loop (acestep/mlx_dit/generate.py:143-199) on the device: ODE (sde = 0)
 * or SDE (sde = 1: x0 = xt - v*t; xt = t_next*noise_i + (1 - t_next)*x0 with caller noise
 * d_noise [n_steps-1][batch][seq_len][audio]); when d_enc_nc is non-NULL, every step i >= cover_steps
 * runs on the non-cover conditions (generate.py:160): d_enc_nc replaces d_enc and d_context_nc (if
 * non-NULL) replaces d_context.  d_enc_nc = NULL or cover_steps >= n_steps: no switch; a negative
 * cover_steps switches at step 0.  cache_cross = 1 reuses the
 * encoder-side tensors (condition embedder + every layer's cross K/V) between steps with the same
 * conditions, as MLXCrossAttentionCache (use_cache=True) does.  Last step: x0 = xt - v*t. */
ACE_GGML_API ace_ggml_status ace_mi_dit_sample_ex(ace_ggml_context* ctx, int32_t batch, float* d_xt,
                                                  const float* d_context, const float* d_enc, const int32_t* d_mask,
                                                  const int32_t* d_enc_mask, int32_t seq_len, int32_t enc_len,
                                                  const float* schedule, int32_t n_steps, int32_t sde,
                                                  const float* d_noise, int32_t cover_steps,
                                                  const float* d_context_nc, const float* d_enc_nc,
                                                  int32_t cache_cross, void* stream);

/* Operand precision of the DiT's attention MFMAs for subsequent forwards (the ACE_MI_ATTN_PRECISION
 * default is read when the DiT is loaded): 0 = fp16 operands, 1 = `split` (hi/lo fp16 Q.K, fp16 P.V),
 * 2 = `f32` (hi/lo fp16 for both products), 3 = `f8c` (hi/lo for both products, the hi x hi product in fp16 and
 * the two correction products as block-scaled e4m3 MFMAs; the default when ACE_MI_ATTN_PRECISION is unset),
 * 4 = `pv8` (fp16 Q.K, P.V as in f8c).  All accumulate in f32. */
ACE_GGML_API ace_ggml_status ace_mi_dit_set_attn_precision(ace_ggml_context* ctx, int32_t mode);

/* Per-kernel-class timing with hipEvents on the launch stream (adds a sync per kernel).
 * ace_mi_profile_get copies up to `cap` entries: names (NUL-separated into `names`, `names_cap`
 * bytes), total milliseconds and launch counts.  Returns the number of classes in *n_out. */
ACE_GGML_API ace_ggml_status ace_mi_profile_enable(ace_ggml_context* ctx, int32_t on);
ACE_GGML_API ace_ggml_status ace_mi_profile_reset(ace_ggml_context* ctx);
ACE_GGML_API ace_ggml_status ace_mi_profile_get(ace_ggml_context* ctx, char* names, size_t names_cap, double* ms,
                                                int32_t* counts, int32_t cap, int32_t* n_out);

/* Launch `iters` copies of one DiT GEMM of layer 0 with M token rows on the context stream
 * (which: 0 = MLP gate|up, 1 = MLP down).  Used by bench.py for the roofline probe. */
ACE_GGML_API ace_ggml_status ace_mi_probe_gemm(ace_ggml_context* ctx, int32_t which, int32_t m_rows,
                                               int32_t iters);

/* Synchronise the context stream. */
ACE_GGML_API ace_ggml_status ace_mi_synchronize(ace_ggml_context* ctx);

/* Force the GEMM kernel variant of all later launches in this process (-1 = automatic; dense 0..11, quantized
 * 20..24, + 100 S for split-K over S blocks per tile; A/B measurements).  The kernel self-test and
 * micro-benchmark entries live in the separate test library (include/acestep_mi355x_selftest.h). */
ACE_GGML_API ace_ggml_status ace_mi_gemm_variant(int32_t variant);

/* VAE decode on device pointers, stream-ordered: latents [n_frames][latent_channels] f32 ->
 * out [out_len][audio_channels] f32 (out_len from ace_mi_vae_out_len: n_frames*hop for even strides). */
ACE_GGML_API ace_ggml_status ace_mi_vae_out_len(ace_ggml_context* ctx, int32_t n_frames, int64_t* out_len);
ACE_GGML_API ace_ggml_status ace_mi_vae_decode_device(ace_ggml_context* ctx, const float* d_latents,
                                                      int32_t n_frames, float* d_out, void* stream);
/* VAE encode on device pointers: audio [n_samples][audio_channels] -> latent mean [enc_out_len][latent]. */
ACE_GGML_API ace_ggml_status ace_mi_vae_enc_out_len(ace_ggml_context* ctx, int32_t n_samples, int64_t* out_len);
ACE_GGML_API ace_ggml_status ace_mi_vae_encode_device(ace_ggml_context* ctx, const float* d_audio,
                                                      int32_t n_samples, float* d_out, void* stream);

/* ggml block quantization (qtype 1 = Q8_0, 2 = Q4_K, 3 = Q6_K) with the encoders the loader uses for
 * ACE_GGML_DIT_WEIGHT_QTYPE (try_quantize_matrix, acestep_dit_model.cpp:156-192): rows x cols f32 ->
 * ggml block bytes.  Returns the byte count written, or -1 (bad type / cols % block / dst too small). */
ACE_GGML_API int64_t ace_mi_quantize(int32_t qtype, const float* src, int64_t rows, int64_t cols, uint8_t* dst,
                                     size_t dst_size);
/* ggml dequantize_row_* of block rows to f32. */
ACE_GGML_API ace_ggml_status ace_mi_dequantize(int32_t qtype, const uint8_t* src, int64_t rows, int64_t cols,
                                               float* dst);
/* ---- condition encoders: the conditioning half of
 * ace_generate_audio_style_lyric_timbre_impl (acestep_ggml.cpp:2324-2556) on the GPU.  Host buffers,
 * blocking, like the reference's internal functions they expose. ---- */
typedef struct ace_mi_cond_info {
    int32_t hidden_size;         /* DiT hidden size = width of every condition state */
    int32_t lyric_in_dim;        /* lyric encoder input width (config text_hidden_dim, else 1024) */
    int32_t timbre_in_dim;       /* timbre encoder input width (timbre_hidden_dim, else audio dim, else 64) */
    int32_t text_projector_in;   /* encoder.text_projector in-features (0 = not loaded) */
    int32_t has_lyric_encoder;   /* lyric embed_tokens (or the text-projector fallback) loaded */
    int32_t lyric_layers;
    int32_t has_timbre_encoder;
    int32_t timbre_layers;
} ace_mi_cond_info;
ACE_GGML_API ace_ggml_status ace_mi_cond_get_info(ace_ggml_context* ctx, ace_mi_cond_info* out);

/* ace_project_tokens_linear with encoder.text_projector (acestep_ggml.cpp:1624-1678):
 * states [n_tokens][in_dim] -> out [n_tokens][hidden_size]. */
ACE_GGML_API ace_ggml_status ace_mi_text_project(ace_ggml_context* ctx, const float* states, int32_t n_tokens,
                                                 int32_t in_dim, float* out, size_t out_size);
/* ace_encode_lyric_condition / forward_lyric_encoder (acestep_ggml.cpp:1680-1727,
 * acestep_dit_model.cpp:1562-1651): lyric token embeddings [n_tokens][lyric_in_dim] ->
 * [n_tokens][hidden_size]; ACE_GGML_LYRIC_MAX_LAYERS honoured. */
ACE_GGML_API ace_ggml_status ace_mi_lyric_encode(ace_ggml_context* ctx, const float* lyric_embeds, int32_t n_tokens,
                                                 float* out, size_t out_size);
/* ace_encode_timbre_condition / forward_timbre_encoder (acestep_ggml.cpp:1803-1899,
 * acestep_dit_model.cpp:1653-1737): refer [n_refer][refer_len][timbre_in_dim] -> one token per
 * reference, out [n_refer][hidden_size]; a non-zero order_mask entry is ACE_GGML_ERR_UNSUPPORTED. */
ACE_GGML_API ace_ggml_status ace_mi_timbre_encode(ace_ggml_context* ctx, const float* refer,
                                                  const int32_t* order_mask, int32_t n_refer, int32_t refer_len,
                                                  float* out, size_t out_size);
/* The encoder_hidden_states assembly of ace_generate_audio_style_lyric_timbre_impl
 * (acestep_ggml.cpp:2414-2556): style states [n_style][text_hidden] (text-encoder output) through the
 * text projector, lyric embeddings [n_lyric][text_hidden] through the lyric encoder (copy fallback),
 * timbre references through the timbre encoder, packed lyric | timbre | style with
 * ace_pack_sequences_single_batch (:1729-1801).  Writes out_enc [len][hidden_size] f32,
 * out_mask [len] int32 and *out_len = len (sizes in bytes). */
ACE_GGML_API ace_ggml_status ace_mi_build_condition(ace_ggml_context* ctx, const float* style_states,
                                                    int32_t n_style, const float* lyric_embeds, int32_t n_lyric,
                                                    int32_t text_hidden, const float* refer,
                                                    const int32_t* refer_order_mask, int32_t n_refer,
                                                    int32_t refer_len, float* out_enc, size_t out_enc_size,
                                                    int32_t* out_mask, size_t out_mask_size, int32_t* out_len);

/* The x_T stream of the reference generator (std::mt19937(seed) + std::normal_distribution<float>,
 * acestep_ggml.cpp:2043-2048) as the generate entries draw it: n values into out (host). */
ACE_GGML_API ace_ggml_status ace_mi_reference_noise(int32_t seed, int64_t n, float* out);

#ifdef __cplusplus
}
#endif

#endif /* ACESTEP_MI355X_H */
