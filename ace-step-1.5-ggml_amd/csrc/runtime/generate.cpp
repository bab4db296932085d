// End-to-end generation entries of the reference ABI (include/acestep_ggml.h):
// ace_ggml_generate_audio_simple / _style_lyric_simple / _style_lyric_timbre_simple
// (acestep_ggml.cpp:1901-2576) with every stage on the GPU: Qwen3 text encoder, condition encoders,
// the silence-latent context (VAE encode), the 8-step Euler loop on device-resident x_t
// (ace_mi_dit_sample) and the windowed VAE decode.  Host-side control flow, environment variables,
// status codes and messages follow the reference function by function; the noise is the reference's
// own std::mt19937 / std::normal_distribution<float> stream, so a seed gives the same x_T.
#include <algorithm>
#include <cmath>
#include <fstream>
#include <iterator>
#include <map>
#include <random>
#include <vector>

#include "context.h"

using namespace acemi_abi;

namespace {

// ace_read_nonneg_env_int (acestep_ggml.cpp:1502-1511)
int32_t nonneg_env(const char* key, int32_t fallback) {
    if (const char* v = std::getenv(key)) {
        char* end = nullptr;
        const long long x = std::strtoll(v, &end, 10);
        if (end && end != v && x >= 0) return static_cast<int32_t>(x);
    }
    return fallback;
}

// ace_get_shift_schedule (:1484-1500): the 8-step turbo schedule nearest to `shift`
std::vector<float> shift_schedule(float shift) {
    static const float s1[] = {1.0f, 0.875f, 0.75f, 0.625f, 0.5f, 0.375f, 0.25f, 0.125f};
    static const float s2[] = {1.0f,          0.9333333333f, 0.8571428571f, 0.7692307692f,
                               0.6666666667f, 0.5454545455f, 0.4f,          0.2222222222f};
    static const float s3[] = {1.0f, 0.9545454545f, 0.9f, 0.8333333333f, 0.75f, 0.6428571429f, 0.5f, 0.3f};
    const float d1 = std::fabs(shift - 1.0f), d2 = std::fabs(shift - 2.0f), d3 = std::fabs(shift - 3.0f);
    if (d1 <= d2 && d1 <= d3) return std::vector<float>(std::begin(s1), std::end(s1));
    if (d2 <= d1 && d2 <= d3) return std::vector<float>(std::begin(s2), std::end(s2));
    return std::vector<float>(std::begin(s3), std::end(s3));
}

// ace_load_silence_latent_f32 (:1513-1572): raw f32 [frames][dim], frame t -> min(t, frames - 1)
bool load_silence_latent(const char* path, int32_t seq_len, int32_t dim, std::vector<float>& out) {
    if (!path || !path[0] || seq_len <= 0 || dim <= 0) return false;
    std::ifstream fin(path, std::ios::binary | std::ios::ate);
    if (!fin) return false;
    const std::streamsize size = fin.tellg();
    if (size <= 0 || size % (std::streamsize)sizeof(float) != 0) return false;
    const size_t n_floats = (size_t)size / sizeof(float);
    if (n_floats % (size_t)dim != 0) return false;
    const size_t n_frames = n_floats / (size_t)dim;
    std::vector<float> full(n_floats);
    fin.seekg(0, std::ios::beg);
    fin.read(reinterpret_cast<char*>(full.data()), size);
    if (!fin) return false;
    out.assign((size_t)seq_len * dim, 0.0f);
    for (int32_t t = 0; t < seq_len; ++t) {
        const size_t st = std::min<size_t>((size_t)t, n_frames - 1);
        std::copy(&full[st * dim], &full[st * dim] + dim, &out[(size_t)t * dim]);
    }
    return true;
}

struct DevMem {
    void* p = nullptr;
    explicit DevMem(size_t n) { ACEMI_HIP(hipMalloc(&p, std::max<size_t>(n, 16))); }
    ~DevMem() {
        if (p) (void)hipFree(p);
    }
    template <typename T>
    T* as() const {
        return static_cast<T*>(p);
    }
};

// ace_generate_audio_from_encoder (:1901-2238)
ace_ggml_status generate_from_encoder(ace_ggml_context* ctx, const float* enc, const int32_t* enc_mask, int32_t enc_len,
                                      int32_t seq_len, float shift, int32_t seed, float* out_audio, size_t out_size,
                                      int32_t* out_audio_samples, int32_t* out_audio_channels) {
    if (!ctx || !enc || enc_len <= 0 || seq_len <= 0 || !out_audio) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    const acemi::DitConfig& dc = ctx->dit->model().cfg;
    const int32_t audio_dim = dc.audio_dim, ctx_dim = dc.in_channels - audio_dim, H = dc.hidden;
    if (ctx_dim <= 0) return set_error(ctx, ACE_GGML_ERR, "invalid dit context dimension");
    int32_t latent_channels = 0, audio_channels = 0, hop_length = 0;
    ace_ggml_status st = ace_ggml_vae_get_info(ctx, &latent_channels, &audio_channels, &hop_length);
    if (st != ACE_GGML_OK) return st;
    if (latent_channels != audio_dim)
        return set_error(ctx, ACE_GGML_ERR, "vae latent channels mismatch with dit audio dim");
    const size_t needed_audio = (size_t)seq_len * hop_length * audio_channels * sizeof(float);
    if (out_size < needed_audio) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");

    // context_latents = [src_latents | chunk mask] (:1948-2041): silence latents from a file, else the VAE
    // encoding of silent audio in chunks (identical chunks of equal length are encoded once)
    std::vector<float> context((size_t)seq_len * ctx_dim, 0.0f);
    if (nonneg_env("ACE_GGML_USE_SILENCE_CONTEXT", 1) != 0) {
        const int32_t src_dim = std::min(audio_dim, ctx_dim);
        const float fill = nonneg_env("ACE_GGML_CHUNK_MASK_FILL", 1) != 0 ? 1.0f : 0.0f;
        std::vector<float> src((size_t)seq_len * src_dim, 0.0f);
        if (!load_silence_latent(std::getenv("ACE_GGML_SILENCE_LATENT_F32"), seq_len, src_dim, src)) {
            const int32_t enc_chunk = nonneg_env("ACE_GGML_VAE_ENCODE_CHUNK_FRAMES", 0);
            int32_t chunk = seq_len;
            if (enc_chunk > 0) {
                chunk = std::max(1, std::min(enc_chunk, seq_len));
            } else {
                int32_t autoc = nonneg_env("ACE_GGML_VAE_ENCODE_CHUNK_FRAMES_AUTO", 0);
                if (autoc <= 0) autoc = seq_len > 128 ? 64 : seq_len;
                chunk = std::max(1, std::min(autoc, seq_len));
            }
            bool ok = true;
            std::map<int32_t, std::vector<float>> by_len;
            for (int32_t f0 = 0; f0 < seq_len && ok; f0 += chunk) {
                const int32_t cur = std::min(chunk, seq_len - f0);
                auto it = by_len.find(cur);
                if (it == by_len.end()) {
                    const int32_t n_samples = cur * hop_length;
                    std::vector<float> silence((size_t)n_samples * audio_channels, 0.0f);
                    std::vector<float> lat((size_t)cur * audio_dim, 0.0f);
                    if (ace_ggml_vae_encode(ctx, silence.data(), n_samples, lat.data(), lat.size() * sizeof(float)) !=
                        ACE_GGML_OK) {
                        ok = false;
                        break;
                    }
                    it = by_len.emplace(cur, std::move(lat)).first;
                }
                for (int32_t t = 0; t < cur; ++t)
                    std::copy(&it->second[(size_t)t * audio_dim], &it->second[(size_t)t * audio_dim] + src_dim,
                              &src[(size_t)(f0 + t) * src_dim]);
            }
            if (!ok) ctx->last_error.clear();  // keep what was encoded (zeros after a first-chunk failure)
        }
        for (int32_t t = 0; t < seq_len; ++t) {
            float* row = &context[(size_t)t * ctx_dim];
            std::copy(&src[(size_t)t * src_dim], &src[(size_t)t * src_dim] + src_dim, row);
            for (int32_t c = src_dim; c < ctx_dim; ++c) row[c] = fill;
        }
    }

    // x_T from the reference's generator (:2043-2048)
    std::mt19937 rng(static_cast<uint32_t>(seed));
    std::normal_distribution<float> dist(0.0f, 1.0f);
    std::vector<float> xt((size_t)seq_len * audio_dim);
    for (float& v : xt) v = dist(rng);
    const std::vector<float> schedule = shift_schedule(shift);

    // the Euler loop (:2056-2086) on device-resident x_t; attention_mask is all ones (= no mask)
    try {
        bind_device(ctx);
        hipStream_t s = ctx->stream;
        DevMem d_xt(xt.size() * 4), d_ctx(context.size() * 4), d_enc((size_t)enc_len * H * 4), d_em((size_t)enc_len * 4);
        ACEMI_HIP(hipMemcpyAsync(d_xt.p, xt.data(), xt.size() * 4, hipMemcpyHostToDevice, s));
        ACEMI_HIP(hipMemcpyAsync(d_ctx.p, context.data(), context.size() * 4, hipMemcpyHostToDevice, s));
        ACEMI_HIP(hipMemcpyAsync(d_enc.p, enc, (size_t)enc_len * H * 4, hipMemcpyHostToDevice, s));
        if (enc_mask) ACEMI_HIP(hipMemcpyAsync(d_em.p, enc_mask, (size_t)enc_len * 4, hipMemcpyHostToDevice, s));
        st = ace_mi_dit_sample(ctx, 1, d_xt.as<float>(), d_ctx.as<float>(), d_enc.as<float>(), nullptr,
                               enc_mask ? d_em.as<int32_t>() : nullptr, seq_len, enc_len, schedule.data(),
                               (int32_t)schedule.size(), s);
        if (st != ACE_GGML_OK) return st;
        ACEMI_HIP(hipMemcpyAsync(xt.data(), d_xt.p, xt.size() * 4, hipMemcpyDeviceToHost, s));
        ACEMI_HIP(hipStreamSynchronize(s));
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("dit forward failed: ") + e.what());
    }

    // VAE decode, windowed like the reference (:2114-2223)
    const char* chunk_env = std::getenv("ACE_GGML_VAE_CHUNK_FRAMES");
    int32_t chunk = nonneg_env("ACE_GGML_VAE_CHUNK_FRAMES", -1);
    if (!chunk_env || !chunk_env[0]) {
        const int32_t autof = nonneg_env("ACE_GGML_VAE_CHUNK_FRAMES_AUTO", 0);
        chunk = autof > 0 ? autof : (seq_len > 128 ? 128 : 0);
    } else if (chunk < 0) {
        chunk = 0;
    }
    int32_t produced = seq_len * hop_length;
    if (chunk > 0 && chunk < seq_len) {
        const size_t cs = (size_t)audio_channels;
        const size_t cap_samples = out_size / (sizeof(float) * cs);
        int32_t overlap = nonneg_env("ACE_GGML_VAE_CHUNK_OVERLAP_FRAMES", -1);
        if (overlap < 0) overlap = std::min<int32_t>(64, std::max<int32_t>(1, chunk / 4));
        if (overlap * 2 >= chunk) overlap = std::max<int32_t>(0, chunk / 2 - 1);
        int32_t stride = chunk - 2 * overlap;
        if (stride <= 0) {
            overlap = 0;
            stride = chunk;
        }
        // The windows (reference order) decode in batches: consecutive windows of equal length share
        // every conv launch (VaeEngine::decode items), so the narrow early stages of a 128-frame
        // window fill the chip.  Each window's output is the reference's zero-filled
        // wf * hop_length buffer holding the decoder's out_len(wf) samples, trimmed as there.
        struct Win {
            int32_t core0, core1, w0, w1;
        };
        std::vector<Win> wins;
        for (int32_t core0 = 0; core0 < seq_len; core0 += stride) {
            const int32_t core1 = std::min(core0 + stride, seq_len);
            wins.push_back({core0, core1, std::max(0, core0 - overlap), std::min(seq_len, core1 + overlap)});
        }
        const int32_t max_batch = std::max<int32_t>(1, nonneg_env("ACE_MI_VAE_WINDOW_BATCH", 16));
        double up = -1.0;
        size_t pos = 0;
        try {
            bind_device(ctx);
            hipStream_t s = ctx->stream;
            for (size_t g0 = 0; g0 < wins.size();) {
                const int32_t wf = wins[g0].w1 - wins[g0].w0;
                size_t g1 = g0 + 1;
                while (g1 < wins.size() && (int32_t)(g1 - g0) < max_batch && wins[g1].w1 - wins[g1].w0 == wf) ++g1;
                const int nb = (int)(g1 - g0);
                const int64_t dec_len = ctx->vae->out_len(wf);
                const size_t lat_n = (size_t)wf * audio_dim, aud_n = (size_t)dec_len * cs;
                std::vector<float> lat((size_t)nb * lat_n);
                for (int b = 0; b < nb; ++b)
                    std::copy(&xt[(size_t)wins[g0 + b].w0 * audio_dim], &xt[(size_t)wins[g0 + b].w0 * audio_dim] + lat_n,
                              &lat[(size_t)b * lat_n]);
                DevMem d_lat(lat.size() * 4), d_aud((size_t)nb * aud_n * 4);
                ACEMI_HIP(hipMemcpyAsync(d_lat.p, lat.data(), lat.size() * 4, hipMemcpyHostToDevice, s));
                ctx->vae->decode(d_lat.as<float>(), wf, d_aud.as<float>(), s, nb);
                std::vector<float> dec((size_t)nb * aud_n);
                ACEMI_HIP(hipMemcpyAsync(dec.data(), d_aud.p, dec.size() * 4, hipMemcpyDeviceToHost, s));
                ACEMI_HIP(hipStreamSynchronize(s));
                for (int b = 0; b < nb; ++b) {
                    const Win& w = wins[g0 + b];
                    std::vector<float> audio((size_t)wf * hop_length * cs, 0.0f);
                    std::copy(&dec[(size_t)b * aud_n], &dec[(size_t)b * aud_n] + std::min(aud_n, audio.size()),
                              audio.begin());
                    const size_t decoded = audio.size() / cs;
                    if (up <= 0.0 && wf > 0) up = (double)decoded / (double)wf;
                    const double trim = up > 0.0 ? up : (double)hop_length;
                    int32_t ts = (int32_t)std::llround((double)(w.core0 - w.w0) * trim);
                    int32_t te = (int32_t)std::llround((double)(w.w1 - w.core1) * trim);
                    ts = std::max(0, std::min(ts, (int32_t)decoded));
                    te = std::max(0, std::min(te, (int32_t)decoded));
                    int32_t end = (int32_t)decoded - te;
                    if (end < ts) end = ts;
                    size_t core = (size_t)(end - ts);
                    if (core > 0 && pos < cap_samples) {
                        core = std::min(core, cap_samples - pos);
                        std::copy(&audio[(size_t)ts * cs], &audio[(size_t)ts * cs] + core * cs, out_audio + pos * cs);
                        pos += core;
                    }
                }
                g0 = g1;
            }
        } catch (const std::exception& e) {
            return set_error(ctx, ACE_GGML_ERR, std::string("graph compute failed: ") + e.what());
        }
        produced = (int32_t)pos;
    } else {
        st = ace_ggml_vae_decode(ctx, xt.data(), seq_len, out_audio, out_size);
        if (st != ACE_GGML_OK) return st;
        // the reference reports seq_len * hop samples; with odd decoder strides the decode is shorter
        // (PyTorch ConvTranspose1d lengths) and the tail it leaves untouched is zeroed here
        int64_t n_dec = 0;
        if (ace_mi_vae_out_len(ctx, seq_len, &n_dec) == ACE_GGML_OK && n_dec < produced)
            std::fill(out_audio + n_dec * audio_channels, out_audio + (size_t)produced * audio_channels, 0.0f);
    }
    if (out_audio_samples) *out_audio_samples = produced;
    if (out_audio_channels) *out_audio_channels = audio_channels;
    return ACE_GGML_OK;
}

// style states through the text encoder (ACE_GGML_TEXT_MAX_LAYERS caps it, :2376-2400)
ace_ggml_status encode_text(ace_ggml_context* ctx, const int32_t* ids, int32_t n, std::vector<float>& out) {
    out.assign((size_t)n * ctx->text->model().cfg.hidden, 0.0f);
    const int32_t max_layers = nonneg_env("ACE_GGML_TEXT_MAX_LAYERS", -1);
    if (max_layers >= 0)
        return ace_ggml_text_encoder_forward_layers(ctx, ids, nullptr, n, max_layers, 1, out.data(),
                                                    out.size() * sizeof(float));
    return ace_ggml_text_encoder_forward(ctx, ids, n, out.data(), out.size() * sizeof(float));
}

// ace_generate_audio_style_lyric_timbre_impl (:2324-2556)
ace_ggml_status style_lyric_timbre(ace_ggml_context* ctx, const int32_t* style_ids, int32_t n_style,
                                   const int32_t* lyric_ids, int32_t n_lyric, const float* refer,
                                   const int32_t* refer_order_mask, int32_t n_refer, int32_t refer_len,
                                   int32_t seq_len, float shift, int32_t seed, float* out_audio, size_t out_size,
                                   int32_t* out_samples, int32_t* out_channels) {
    const bool has_style = n_style > 0, has_lyric = n_lyric > 0, has_timbre = n_refer > 0;
    if (!ctx || !out_audio || seq_len <= 0 || (!has_style && !has_lyric && !has_timbre)) return ACE_GGML_ERR_INVALID_ARG;
    if (has_style && !style_ids) return ACE_GGML_ERR_INVALID_ARG;
    if (has_lyric && !lyric_ids) return ACE_GGML_ERR_INVALID_ARG;
    if (has_timbre && (!refer || refer_len <= 0)) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->text) return set_error(ctx, ACE_GGML_ERR, "text encoder not loaded");
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    const int32_t text_hidden = ctx->text->model().cfg.hidden;
    const int32_t H = ctx->dit->model().cfg.hidden;
    std::vector<float> style, lyric;
    ace_ggml_status st = ACE_GGML_OK;
    if (has_style && (st = encode_text(ctx, style_ids, n_style, style)) != ACE_GGML_OK) return st;
    if (has_lyric) {
        lyric.assign((size_t)n_lyric * text_hidden, 0.0f);
        st = ace_ggml_text_encoder_forward_embeddings(ctx, lyric_ids, n_lyric, lyric.data(), lyric.size() * sizeof(float));
        if (st != ACE_GGML_OK) return st;
    }
    const int32_t cap = (has_style ? n_style : 0) + (has_lyric ? n_lyric : 0) + (has_timbre ? n_refer : 0);
    std::vector<float> enc((size_t)cap * H);
    std::vector<int32_t> mask((size_t)cap);
    int32_t len = 0;
    st = ace_mi_build_condition(ctx, has_style ? style.data() : nullptr, n_style, has_lyric ? lyric.data() : nullptr,
                                n_lyric, text_hidden, refer, refer_order_mask, n_refer, refer_len, enc.data(),
                                enc.size() * sizeof(float), mask.data(), mask.size() * sizeof(int32_t), &len);
    if (st != ACE_GGML_OK) return st;
    return generate_from_encoder(ctx, enc.data(), mask.data(), len, seq_len, shift, seed, out_audio, out_size,
                                 out_samples, out_channels);
}

}  // namespace

extern "C" {

ace_ggml_status ace_ggml_generate_audio_simple(ace_ggml_context* ctx, const int32_t* token_ids, int32_t n_tokens,
                                               int32_t seq_len, float shift, int32_t seed, float* out_audio,
                                               size_t out_size, int32_t* out_audio_samples,
                                               int32_t* out_audio_channels) {
    if (!ctx || !token_ids || !out_audio || n_tokens <= 0 || seq_len <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->text) return set_error(ctx, ACE_GGML_ERR, "text encoder not loaded");
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    const int32_t H = ctx->dit->model().cfg.hidden, text_hidden = ctx->text->model().cfg.hidden;
    if (text_hidden != H && std::getenv("ACE_GGML_ALLOW_TEXT_DIM_MISMATCH") == nullptr)
        return set_error(ctx, ACE_GGML_ERR, "text encoder hidden size mismatch with dit");
    std::vector<float> states;
    const ace_ggml_status st = encode_text(ctx, token_ids, n_tokens, states);
    if (st != ACE_GGML_OK) return st;
    // text states straight into encoder_hidden_states, truncated / zero padded to H (:2289-2300)
    std::vector<float> enc((size_t)n_tokens * H, 0.0f);
    const int32_t cpy = std::min(text_hidden, H);
    for (int32_t t = 0; t < n_tokens; ++t)
        std::copy(&states[(size_t)t * text_hidden], &states[(size_t)t * text_hidden] + cpy, &enc[(size_t)t * H]);
    std::vector<int32_t> mask((size_t)n_tokens, 1);
    return generate_from_encoder(ctx, enc.data(), mask.data(), n_tokens, seq_len, shift, seed, out_audio, out_size,
                                 out_audio_samples, out_audio_channels);
}

ace_ggml_status ace_ggml_generate_audio_style_lyric_simple(ace_ggml_context* ctx, const int32_t* style_token_ids,
                                                           int32_t n_style_tokens, const int32_t* lyric_token_ids,
                                                           int32_t n_lyric_tokens, int32_t seq_len, float shift,
                                                           int32_t seed, float* out_audio, size_t out_size,
                                                           int32_t* out_audio_samples, int32_t* out_audio_channels) {
    return style_lyric_timbre(ctx, style_token_ids, n_style_tokens, lyric_token_ids, n_lyric_tokens, nullptr, nullptr,
                              0, 0, seq_len, shift, seed, out_audio, out_size, out_audio_samples, out_audio_channels);
}

ace_ggml_status ace_ggml_generate_audio_style_lyric_timbre_simple(
    ace_ggml_context* ctx, const int32_t* style_token_ids, int32_t n_style_tokens, const int32_t* lyric_token_ids,
    int32_t n_lyric_tokens, const float* refer_audio_acoustic_hidden_states, const int32_t* refer_audio_order_mask,
    int32_t n_refer_audio, int32_t refer_audio_len, int32_t seq_len, float shift, int32_t seed, float* out_audio,
    size_t out_size, int32_t* out_audio_samples, int32_t* out_audio_channels) {
    return style_lyric_timbre(ctx, style_token_ids, n_style_tokens, lyric_token_ids, n_lyric_tokens,
                              refer_audio_acoustic_hidden_states, refer_audio_order_mask, n_refer_audio,
                              refer_audio_len, seq_len, shift, seed, out_audio, out_size, out_audio_samples,
                              out_audio_channels);
}

// the reference generator's x_T (std::mt19937 + std::normal_distribution<float>, :2043-2048), for tests
ace_ggml_status ace_mi_reference_noise(int32_t seed, int64_t n, float* out) {
    if (!out || n < 0) return ACE_GGML_ERR_INVALID_ARG;
    std::mt19937 rng(static_cast<uint32_t>(seed));
    std::normal_distribution<float> dist(0.0f, 1.0f);
    for (int64_t i = 0; i < n; ++i) out[i] = dist(rng);
    return ACE_GGML_OK;
}

}  // extern "C"
