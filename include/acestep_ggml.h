/*
 * Drop-in C-ABI for the ACE-Step 1.5 DiT hot path, implemented on MI355X
 * (gfx950) by libacestep_mi355x.so.
 *
 * Every declaration below has the exact name, argument order, types and
 * status codes of the reference ABI it replaces, so existing callers
 * (ctypes GGMLCAPIBridge, the C sampler, ace_ggml_cli --dit, compare_dit.py)
 * can load this library instead of libacestep_ggml.so:
 *
 *   ace_ggml_status / ace_ggml_init_params   acestep_ggml/cpp/acestep_ggml.h:23-35
 *   ace_ggml_create                          acestep_ggml/cpp/acestep_ggml.h:37
 *   ace_ggml_destroy                         acestep_ggml/cpp/acestep_ggml.h:38
 *   ace_ggml_last_error                      acestep_ggml/cpp/acestep_ggml.h:39
 *   ace_ggml_load_dit                        acestep_ggml/cpp/acestep_ggml.h:43
 *   ace_ggml_dit_forward                     acestep_ggml/cpp/acestep_ggml.h:96-108
 *   ace_ggml_load_vae                        acestep_ggml/cpp/acestep_ggml.h:44
 *   ace_ggml_vae_get_info                    acestep_ggml/cpp/acestep_ggml.h:45-49
 *   ace_ggml_vae_decode                      acestep_ggml/cpp/acestep_ggml.h:50-55
 *   ace_ggml_vae_encode                      acestep_ggml/cpp/acestep_ggml.h:56-61
 *   ace_ggml_load_lm                         acestep_ggml/cpp/acestep_ggml.h:41
 *   ace_ggml_load_text_encoder               acestep_ggml/cpp/acestep_ggml.h:42
 *   ace_ggml_text_encoder_forward            acestep_ggml/cpp/acestep_ggml.h:63-68
 *   ace_ggml_text_encoder_forward_masked     acestep_ggml/cpp/acestep_ggml.h:70-76
 *   ace_ggml_text_encoder_forward_embeddings acestep_ggml/cpp/acestep_ggml.h:78-83
 *   ace_ggml_text_encoder_forward_layers     acestep_ggml/cpp/acestep_ggml.h:86-94
 *   ace_ggml_generate_audio_simple           acestep_ggml/cpp/acestep_ggml.h:110-120
 *   ace_ggml_generate_audio_style_lyric_simple         acestep_ggml/cpp/acestep_ggml.h:122-134
 *   ace_ggml_generate_audio_style_lyric_timbre_simple  acestep_ggml/cpp/acestep_ggml.h:136-152
 *
 * Semantics: host f32 row-major, time-major buffers; one sample
 * per call; the caller owns every buffer; blocking; one context is not
 * thread-safe.  `n_threads` and `use_metal` are accepted and ignored
 * (the compute runs on the GPU); `compute_buffer_bytes` is ignored (the
 * workspace is sized from the shapes).  ace_ggml_load_dit accepts the reference's weight sources:
 * model.safetensors (BF16/F16, optional online ACE_GGML_DIT_WEIGHT_QTYPE=Q8_0/Q6_K/Q4_K) and GGUF
 * (ACE_GGML_DIT_GGUF[_PATH], <dir>.gguf or <dir>/model.gguf; F16/BF16/Q8_0/Q6_K/Q4_K tensors).
 * The device is HIP device 0 unless
 * ACE_MI_DEVICE is set, or ace_mi_create_on_device (acestep_mi355x.h) is used.
 */
#ifndef ACESTEP_GGML_H
#define ACESTEP_GGML_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACE_GGML_API __attribute__((visibility("default")))

typedef struct ace_ggml_context ace_ggml_context;

typedef enum ace_ggml_status {
    ACE_GGML_OK = 0,
    ACE_GGML_ERR = 1,
    ACE_GGML_ERR_INVALID_ARG = 2,
    ACE_GGML_ERR_IO = 3,
    ACE_GGML_ERR_UNSUPPORTED = 4
} ace_ggml_status;

typedef struct ace_ggml_init_params {
    int32_t n_threads;
    int32_t use_metal;
    size_t compute_buffer_bytes;
} ace_ggml_init_params;

ACE_GGML_API ace_ggml_status ace_ggml_create(const ace_ggml_init_params* params, ace_ggml_context** out_ctx);
ACE_GGML_API void ace_ggml_destroy(ace_ggml_context* ctx);
ACE_GGML_API const char* ace_ggml_last_error(const ace_ggml_context* ctx);

ACE_GGML_API ace_ggml_status ace_ggml_load_dit(ace_ggml_context* ctx, const char* model_dir);

ACE_GGML_API ace_ggml_status ace_ggml_dit_forward(ace_ggml_context* ctx, const float* hidden_states,
                                                  const float* context_latents, const float* encoder_hidden_states,
                                                  const int32_t* attention_mask,
                                                  const int32_t* encoder_attention_mask, int32_t seq_len,
                                                  int32_t enc_len, float timestep, float timestep_r, float* out,
                                                  size_t out_size);

/* Oobleck VAE decoder (diffusion_pytorch_model.safetensors + config.json).  Decode: latents
 * [n_frames][latent_channels] f32 -> audio [n_frames*hop][audio_channels] f32 interleaved;
 * INVALID_ARG "output buffer too small" if out_size < n_frames*hop*audio_channels*4. */
ACE_GGML_API ace_ggml_status ace_ggml_load_vae(ace_ggml_context* ctx, const char* model_dir);
ACE_GGML_API ace_ggml_status ace_ggml_vae_get_info(ace_ggml_context* ctx, int32_t* latent_channels,
                                                   int32_t* audio_channels, int32_t* hop_length);
ACE_GGML_API ace_ggml_status ace_ggml_vae_decode(ace_ggml_context* ctx, const float* latents, int32_t n_frames,
                                                 float* out, size_t out_size);
/* Encode: audio [n_samples][audio_channels] f32 -> latent mean [n_samples/hop][latent_channels] f32
 * (needs the encoder.* tensors of the VAE checkpoint). */
ACE_GGML_API ace_ggml_status ace_ggml_vae_encode(ace_ggml_context* ctx, const float* audio, int32_t n_samples,
                                                 float* out, size_t out_size);

/* Qwen3 text encoder.  Both loaders fill the same text-encoder slot
 * (acestep_ggml.cpp:246-258); safetensors (ACE_GGML_QWEN_WEIGHT_QTYPE / ACE_GGML_WEIGHT_QTYPE online
 * quantization) or GGUF (ACE_GGML_QWEN_GGUF, ACE_GGML_TEXT_ENCODER_GGUF, ACE_GGML_LM_GGUF, <dir>.gguf,
 * <dir>/model.gguf).  Forwards are causal; out is [n_tokens][hidden_size] f32. */
ACE_GGML_API ace_ggml_status ace_ggml_load_lm(ace_ggml_context* ctx, const char* model_dir);
ACE_GGML_API ace_ggml_status ace_ggml_load_text_encoder(ace_ggml_context* ctx, const char* model_dir);
ACE_GGML_API ace_ggml_status ace_ggml_text_encoder_forward(ace_ggml_context* ctx, const int32_t* token_ids,
                                                           int32_t n_tokens, float* out, size_t out_size);
ACE_GGML_API ace_ggml_status ace_ggml_text_encoder_forward_masked(ace_ggml_context* ctx, const int32_t* token_ids,
                                                                  const int32_t* attention_mask, int32_t n_tokens,
                                                                  float* out, size_t out_size);
ACE_GGML_API ace_ggml_status ace_ggml_text_encoder_forward_embeddings(ace_ggml_context* ctx,
                                                                      const int32_t* token_ids, int32_t n_tokens,
                                                                      float* out, size_t out_size);
ACE_GGML_API ace_ggml_status ace_ggml_text_encoder_forward_layers(ace_ggml_context* ctx, const int32_t* token_ids,
                                                                  const int32_t* attention_mask, int32_t n_tokens,
                                                                  int32_t n_layers, int32_t apply_final_norm,
                                                                  float* out, size_t out_size);

/* End-to-end text-to-audio (acestep_ggml.cpp:1901-2576): text encoder -> condition -> 8-step Euler
 * sampler (turbo schedule nearest to `shift`, x_T from std::mt19937(seed)) -> VAE decode.  out_audio
 * [samples][audio_channels] f32 with out_size >= seq_len * hop * channels * 4; the silence-latent
 * context and the windowed decode honour the reference's ACE_GGML_* variables. */
ACE_GGML_API ace_ggml_status ace_ggml_generate_audio_simple(ace_ggml_context* ctx, const int32_t* token_ids,
                                                            int32_t n_tokens, int32_t seq_len, float shift,
                                                            int32_t seed, float* out_audio, size_t out_size,
                                                            int32_t* out_audio_samples, int32_t* out_audio_channels);
ACE_GGML_API ace_ggml_status ace_ggml_generate_audio_style_lyric_simple(
    ace_ggml_context* ctx, const int32_t* style_token_ids, int32_t n_style_tokens, const int32_t* lyric_token_ids,
    int32_t n_lyric_tokens, int32_t seq_len, float shift, int32_t seed, float* out_audio, size_t out_size,
    int32_t* out_audio_samples, int32_t* out_audio_channels);
ACE_GGML_API ace_ggml_status ace_ggml_generate_audio_style_lyric_timbre_simple(
    ace_ggml_context* ctx, const int32_t* style_token_ids, int32_t n_style_tokens, const int32_t* lyric_token_ids,
    int32_t n_lyric_tokens, const float* refer_audio_acoustic_hidden_states, const int32_t* refer_audio_order_mask,
    int32_t n_refer_audio, int32_t refer_audio_len, int32_t seq_len, float shift, int32_t seed, float* out_audio,
    size_t out_size, int32_t* out_audio_samples, int32_t* out_audio_channels);

#ifdef __cplusplus
}
#endif

#endif /* ACESTEP_GGML_H */
