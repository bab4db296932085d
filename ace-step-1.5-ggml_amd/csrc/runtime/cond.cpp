// Condition-encoder entry points (include/acestep_mi355x.h).
//
// The reference builds encoder_hidden_states once per request on the CPU
// (ace_generate_audio_style_lyric_timbre_impl, acestep_ggml.cpp:2324-2556): the style states go
// through encoder.text_projector, the lyric token embeddings through the lyric encoder, every timbre
// reference through the timbre encoder (first token kept), and the three are packed with
// ace_pack_sequences_single_batch.  Here the projections and encoder blocks run on the GPU with the
// DiT's kernels (DitEngine::encode); the packing is host bookkeeping on a few hundred rows.
// Status codes and messages follow the reference functions each entry mirrors.
#include <algorithm>
#include <numeric>
#include <vector>

#include "context.h"

using namespace acemi_abi;

namespace {

// ACE_GGML_{LYRIC,TIMBRE}_MAX_LAYERS (acestep_dit_model.cpp:1605-1612 / :1696-1703): a value >= 0 caps
// the layer count; anything else leaves it alone
int encoder_max_layers(const char* key) {
    const char* v = std::getenv(key);
    if (!v || !v[0]) return -1;
    char* end = nullptr;
    const long long x = std::strtoll(v, &end, 10);
    return (end && end != v && x >= 0) ? static_cast<int>(std::min<long long>(x, 1 << 20)) : -1;
}

// Upload `in` [B][n][proj.cols], run one encoder pass, download [B][n][H] (or [B][H] when first_only).
void encode_host(ace_ggml_context* ctx, const acemi::DevEncoder* enc, const acemi::DevWeight& proj,
                 const float* proj_b, const float* in, int B, int n, bool first_only, float* out, int max_layers) {
    bind_device(ctx);
    hipStream_t s = ctx->stream;
    const int H = ctx->dit->model().cfg.hidden;
    const size_t n_in = (size_t)B * n * proj.cols;
    const size_t n_out = (size_t)(first_only ? B : B * n) * H;
    const size_t o_out = (n_in * 4 + 255) & ~size_t(255);
    ensure_dev(ctx->d_in, ctx->d_in_bytes, o_out + n_out * 4);
    char* base = static_cast<char*>(ctx->d_in);
    ACEMI_HIP(hipMemcpyAsync(base, in, n_in * 4, hipMemcpyHostToDevice, s));
    acemi::EncodeIO io;
    io.enc = enc;
    io.proj = &proj;
    io.proj_b = proj_b;
    io.in = reinterpret_cast<const float*>(base);
    io.B = B;
    io.n = n;
    io.first_only = first_only;
    io.out = reinterpret_cast<float*>(base + o_out);
    io.max_layers = max_layers;
    ctx->dit->encode(io, s);
    ACEMI_HIP(hipMemcpyAsync(out, io.out, n_out * 4, hipMemcpyDeviceToHost, s));
    ACEMI_HIP(hipStreamSynchronize(s));
}

// ace_pack_sequences_single_batch (acestep_ggml.cpp:1729-1801): rows whose mask is set first (stable),
// then the rest; the output mask is 1 for the first n_valid rows.
void pack_sequences(const std::vector<float>& h1, const std::vector<int32_t>& m1, int len1,
                    const std::vector<float>& h2, const std::vector<int32_t>& m2, int len2, int dim,
                    std::vector<float>& out_h, std::vector<int32_t>& out_m) {
    if (len1 <= 0 && len2 <= 0) {
        out_h.clear();
        out_m.clear();
        return;
    }
    if (len2 <= 0) {
        out_h = h1;
        out_m = m1;
        return;
    }
    if (len1 <= 0) {
        out_h = h2;
        out_m = m2;
        return;
    }
    const int len = len1 + len2;
    out_h.assign((size_t)len * dim, 0.0f);
    out_m.assign((size_t)len, 0);
    auto valid = [&](int i) { return i < len1 ? m1[(size_t)i] != 0 : m2[(size_t)(i - len1)] != 0; };
    std::vector<int> idx((size_t)len);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_partition(idx.begin(), idx.end(), valid);
    int n_valid = 0;
    for (int i = 0; i < len; ++i) {
        const int src = idx[(size_t)i];
        const float* p = src < len1 ? &h1[(size_t)src * dim] : &h2[(size_t)(src - len1) * dim];
        std::copy(p, p + dim, &out_h[(size_t)i * dim]);
        if (valid(src)) ++n_valid;
    }
    std::fill(out_m.begin(), out_m.begin() + n_valid, 1);
}

// the lyric encoder's input projection: embed_tokens, else the text projector (no bias)
// (forward_lyric_encoder :1577-1578)
const acemi::DevWeight* lyric_proj(const acemi::DitModel& m, const float** bias) {
    if (m.lyric.has_embed()) {
        *bias = m.lyric.embed_b;
        return &m.lyric.embed;
    }
    *bias = nullptr;
    return m.text_proj.q ? &m.text_proj : nullptr;
}

// ace_encode_lyric_condition without the argument checks; false = forward_lyric_encoder failed
bool lyric_forward(ace_ggml_context* ctx, const float* embeds, int n, float* out) {
    const acemi::DitModel& m = ctx->dit->model();
    const float* bias = nullptr;
    const acemi::DevWeight* w = lyric_proj(m, &bias);
    if (!w || w->cols != m.cfg.lyric_in_dim() || w->rows != m.cfg.hidden) return false;
    encode_host(ctx, &m.lyric, *w, bias, embeds, 1, n, false, out, encoder_max_layers("ACE_GGML_LYRIC_MAX_LAYERS"));
    return true;
}

ace_ggml_status timbre_forward(ace_ggml_context* ctx, const float* refer, const int32_t* order_mask, int n_refer,
                               int refer_len, float* out) {
    const acemi::DitModel& m = ctx->dit->model();
    if (!m.timbre.has_embed()) return set_error(ctx, ACE_GGML_ERR, "timbre encoder weights are not loaded");
    for (int i = 0; i < n_refer; ++i)
        if (order_mask && order_mask[i] != 0)
            return set_error(ctx, ACE_GGML_ERR_UNSUPPORTED, "multi-batch refer_audio_order_mask is not supported");
    const acemi::DevWeight& w = m.timbre.embed;
    if (w.cols != m.cfg.timbre_in_dim() || w.rows != m.cfg.hidden)
        return set_error(ctx, ACE_GGML_ERR, "forward_timbre_encoder failed");
    // the reference encodes the references one by one; they are independent, so one batched pass
    encode_host(ctx, &m.timbre, w, m.timbre.embed_b, refer, n_refer, refer_len, true, out,
                encoder_max_layers("ACE_GGML_TIMBRE_MAX_LAYERS"));
    return ACE_GGML_OK;
}

}  // namespace

extern "C" {

ace_ggml_status ace_mi_cond_get_info(ace_ggml_context* ctx, ace_mi_cond_info* out) {
    if (!ctx || !out) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    const acemi::DitModel& m = ctx->dit->model();
    out->hidden_size = m.cfg.hidden;
    out->lyric_in_dim = m.cfg.lyric_in_dim();
    out->timbre_in_dim = m.cfg.timbre_in_dim();
    out->text_projector_in = m.text_proj.q ? m.text_proj.cols : 0;
    const float* b = nullptr;
    out->has_lyric_encoder = lyric_proj(m, &b) != nullptr;
    out->lyric_layers = (int32_t)m.lyric.layers.size();
    out->has_timbre_encoder = m.timbre.has_embed();
    out->timbre_layers = (int32_t)m.timbre.layers.size();
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_text_project(ace_ggml_context* ctx, const float* states, int32_t n_tokens, int32_t in_dim,
                                    float* out, size_t out_size) {
    if (!ctx) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    const acemi::DitModel& m = ctx->dit->model();
    if (!m.text_proj.q || !states || !out || n_tokens <= 0 || in_dim <= 0)
        return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "invalid linear projection args");
    if (m.text_proj.cols != in_dim) return set_error(ctx, ACE_GGML_ERR, "linear projection weight shape mismatch");
    if (out_size < (size_t)n_tokens * m.cfg.hidden * sizeof(float))
        return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");
    try {
        encode_host(ctx, nullptr, m.text_proj, nullptr, states, 1, n_tokens, false, out, -1);
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("linear projection compute failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_lyric_encode(ace_ggml_context* ctx, const float* lyric_embeds, int32_t n_tokens, float* out,
                                    size_t out_size) {
    if (!ctx || !lyric_embeds || n_tokens <= 0 || !out) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    if (out_size < (size_t)n_tokens * ctx->dit->model().cfg.hidden * sizeof(float))
        return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");
    try {
        if (!lyric_forward(ctx, lyric_embeds, n_tokens, out))
            return set_error(ctx, ACE_GGML_ERR, "forward_lyric_encoder failed");
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("lyric encoder compute failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_timbre_encode(ace_ggml_context* ctx, const float* refer, const int32_t* order_mask,
                                     int32_t n_refer, int32_t refer_len, float* out, size_t out_size) {
    if (!ctx || !refer || n_refer <= 0 || refer_len <= 0 || !out) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    if (out_size < (size_t)n_refer * ctx->dit->model().cfg.hidden * sizeof(float))
        return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");
    try {
        return timbre_forward(ctx, refer, order_mask, n_refer, refer_len, out);
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("timbre encoder compute failed: ") + e.what());
    }
}

ace_ggml_status ace_mi_build_condition(ace_ggml_context* ctx, const float* style_states, int32_t n_style,
                                       const float* lyric_embeds, int32_t n_lyric, int32_t text_hidden,
                                       const float* refer, const int32_t* refer_order_mask, int32_t n_refer,
                                       int32_t refer_len, float* out_enc, size_t out_enc_size, int32_t* out_mask,
                                       size_t out_mask_size, int32_t* out_len) {
    const bool has_style = n_style > 0, has_lyric = n_lyric > 0, has_timbre = n_refer > 0;
    if (!ctx || !out_enc || !out_mask || !out_len || (!has_style && !has_lyric && !has_timbre))
        return ACE_GGML_ERR_INVALID_ARG;
    if ((has_style && !style_states) || (has_lyric && !lyric_embeds)) return ACE_GGML_ERR_INVALID_ARG;
    if (has_timbre && (!refer || refer_len <= 0)) return ACE_GGML_ERR_INVALID_ARG;
    if ((has_style || has_lyric) && text_hidden <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    const acemi::DitModel& m = ctx->dit->model();
    const int H = m.cfg.hidden;
    const bool allow_text_mismatch = std::getenv("ACE_GGML_ALLOW_TEXT_DIM_MISMATCH") != nullptr;
    try {
        std::vector<float> style_cond, lyric_cond, timbre_cond;
        bool style_encoded = false, lyric_encoded = false;
        if (has_style && m.text_proj.q) {  // :2426-2438
            if (m.text_proj.cols != text_hidden)
                return set_error(ctx, ACE_GGML_ERR, "linear projection weight shape mismatch");
            style_cond.resize((size_t)n_style * H);
            encode_host(ctx, nullptr, m.text_proj, nullptr, style_states, 1, n_style, false, style_cond.data(), -1);
            style_encoded = true;
        }
        const float* lb = nullptr;
        if (has_lyric && lyric_proj(m, &lb)) {  // :2440-2452: a failing lyric encoder falls back to a copy
            lyric_cond.resize((size_t)n_lyric * H);
            lyric_encoded = text_hidden == m.cfg.lyric_in_dim() && lyric_forward(ctx, lyric_embeds, n_lyric,
                                                                                  lyric_cond.data());
            ctx->last_error.clear();
        }
        if (has_timbre) {  // :2453-2467
            timbre_cond.resize((size_t)n_refer * H);
            const ace_ggml_status st =
                timbre_forward(ctx, refer, refer_order_mask, n_refer, refer_len, timbre_cond.data());
            if (st != ACE_GGML_OK) return st;
        }
        if (((has_style && !style_encoded) || (has_lyric && !lyric_encoded)) && text_hidden != H &&
            !allow_text_mismatch)
            return set_error(ctx, ACE_GGML_ERR, "text encoder hidden size mismatch with dit");
        const int cpy = std::min(text_hidden, H);
        // un-encoded states are copied into H-wide rows (truncated or zero padded), :2475-2505
        auto widen = [&](const float* src, int n, std::vector<float>& dst) {
            dst.assign((size_t)n * H, 0.0f);
            for (int t = 0; t < n; ++t) std::copy(src + (size_t)t * text_hidden, src + (size_t)t * text_hidden + cpy,
                                                  &dst[(size_t)t * H]);
        };
        std::vector<float> style_hidden, lyric_hidden;
        if (has_style) {
            if (style_encoded)
                style_hidden.swap(style_cond);
            else
                widen(style_states, n_style, style_hidden);
        }
        if (has_lyric) {
            if (lyric_encoded)
                lyric_hidden.swap(lyric_cond);
            else
                widen(lyric_embeds, n_lyric, lyric_hidden);
        }
        // packing order lyric | timbre | style (:2507-2548)
        int cond_len = 0;
        std::vector<float> enc;
        std::vector<int32_t> mask;
        if (has_lyric) {
            enc = lyric_hidden;
            mask.assign((size_t)n_lyric, 1);
            cond_len = n_lyric;
        }
        if (has_timbre) {
            std::vector<float> ph;
            std::vector<int32_t> pm;
            pack_sequences(enc, mask, cond_len, timbre_cond, std::vector<int32_t>((size_t)n_refer, 1), n_refer, H, ph,
                           pm);
            enc.swap(ph);
            mask.swap(pm);
            cond_len += n_refer;
        }
        if (has_style) {
            std::vector<float> ph;
            std::vector<int32_t> pm;
            pack_sequences(enc, mask, cond_len, style_hidden, std::vector<int32_t>((size_t)n_style, 1), n_style, H,
                           ph, pm);
            enc.swap(ph);
            mask.swap(pm);
            cond_len += n_style;
        }
        if (cond_len <= 0) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "empty style/lyric/timbre inputs");
        if (out_enc_size < (size_t)cond_len * H * sizeof(float) || out_mask_size < (size_t)cond_len * sizeof(int32_t))
            return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");
        std::copy(enc.begin(), enc.end(), out_enc);
        std::copy(mask.begin(), mask.end(), out_mask);
        *out_len = cond_len;
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("condition encoder compute failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

}  // extern "C"
