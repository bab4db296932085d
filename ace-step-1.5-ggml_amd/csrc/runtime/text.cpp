// Text-encoder entry points of the reference ABI (include/acestep_ggml.h:41-94), on the GPU.
//
// Same prototypes, status codes and messages as acestep_ggml.cpp:238-258 (load) and :1074-1302
// (ace_ggml_text_encoder_forward / _masked / _embeddings / _layers): INVALID_ARG without a message
// for null pointers or n_tokens <= 0, ERR "text encoder not loaded", INVALID_ARG "output buffer too
// small", ERR_IO with the loader's message.  Token ids outside [0, vocab) are rejected with
// INVALID_ARG "token id out of range" (ggml_get_rows would abort the process).
#include <vector>

#include "context.h"

using namespace acemi_abi;

namespace {

ace_ggml_status load_text(ace_ggml_context* ctx, const char* model_dir) {
    if (!ctx || !model_dir) return ACE_GGML_ERR_INVALID_ARG;
    try {
        bind_device(ctx);
        ACEMI_HIP(hipStreamSynchronize(ctx->stream));
        ctx->text.reset();
        auto eng = std::make_unique<acemi::TextEncoderEngine>();
        acemi::load_text_model(model_dir, eng->model());
        ctx->text = std::move(eng);
    } catch (const acemi::HipError& e) {
        ctx->text.reset();
        return set_error(ctx, ACE_GGML_ERR, e.what());
    } catch (const std::exception& e) {
        ctx->text.reset();
        return set_error(ctx, ACE_GGML_ERR_IO, e.what());
    }
    return ACE_GGML_OK;
}

// mode 0: embeddings only; 1: blocks (n_layers < 0 = all) + final norm when requested
ace_ggml_status run_text(ace_ggml_context* ctx, const int32_t* ids, const int32_t* mask, int32_t n, int mode,
                         int32_t n_layers, bool final_norm, float* out, size_t out_size, const char* fail_msg) {
    if (!ctx || !ids || !out || n <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->text) return set_error(ctx, ACE_GGML_ERR, "text encoder not loaded");
    const acemi::TextConfig& c = ctx->text->model().cfg;
    const size_t needed = (size_t)c.hidden * (size_t)n * sizeof(float);
    if (out_size < needed) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");
    for (int32_t i = 0; i < n; ++i)
        if (ids[i] < 0 || ids[i] >= c.vocab) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "token id out of range");
    try {
        bind_device(ctx);
        hipStream_t s = ctx->stream;
        // staging: ids | mask | out
        const size_t o_mask = ((size_t)n * 4 + 255) & ~size_t(255), o_out = o_mask + o_mask;
        ensure_dev(ctx->d_in, ctx->d_in_bytes, o_out + needed);
        char* base = static_cast<char*>(ctx->d_in);
        ACEMI_HIP(hipMemcpyAsync(base, ids, (size_t)n * 4, hipMemcpyHostToDevice, s));
        const int32_t* d_mask = nullptr;
        if (mask) {
            ACEMI_HIP(hipMemcpyAsync(base + o_mask, mask, (size_t)n * 4, hipMemcpyHostToDevice, s));
            d_mask = reinterpret_cast<const int32_t*>(base + o_mask);
        }
        float* d_out = reinterpret_cast<float*>(base + o_out);
        const int32_t* d_ids = reinterpret_cast<const int32_t*>(base);
        if (mode == 0)
            ctx->text->embeddings(d_ids, n, d_out, s);
        else
            ctx->text->forward(d_ids, d_mask, n, n_layers, final_norm, d_out, s);
        ACEMI_HIP(hipMemcpyAsync(out, d_out, needed, hipMemcpyDeviceToHost, s));
        ACEMI_HIP(hipStreamSynchronize(s));
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string(fail_msg) + ": " + e.what());
    }
    return ACE_GGML_OK;
}

}  // namespace

extern "C" {

// both load the Qwen3 weights into the text-encoder slot (acestep_ggml.cpp:246-258)
ace_ggml_status ace_ggml_load_lm(ace_ggml_context* ctx, const char* model_dir) { return load_text(ctx, model_dir); }

ace_ggml_status ace_ggml_load_text_encoder(ace_ggml_context* ctx, const char* model_dir) {
    return load_text(ctx, model_dir);
}

ace_ggml_status ace_ggml_text_encoder_forward(ace_ggml_context* ctx, const int32_t* token_ids, int32_t n_tokens,
                                              float* out, size_t out_size) {
    return run_text(ctx, token_ids, nullptr, n_tokens, 1, -1, true, out, out_size, "graph compute failed");
}

ace_ggml_status ace_ggml_text_encoder_forward_masked(ace_ggml_context* ctx, const int32_t* token_ids,
                                                     const int32_t* attention_mask, int32_t n_tokens, float* out,
                                                     size_t out_size) {
    return run_text(ctx, token_ids, attention_mask, n_tokens, 1, -1, true, out, out_size, "graph compute failed");
}

ace_ggml_status ace_ggml_text_encoder_forward_embeddings(ace_ggml_context* ctx, const int32_t* token_ids,
                                                         int32_t n_tokens, float* out, size_t out_size) {
    return run_text(ctx, token_ids, nullptr, n_tokens, 0, 0, false, out, out_size, "graph compute failed");
}

ace_ggml_status ace_ggml_text_encoder_forward_layers(ace_ggml_context* ctx, const int32_t* token_ids,
                                                     const int32_t* attention_mask, int32_t n_tokens, int32_t n_layers,
                                                     int32_t apply_final_norm, float* out, size_t out_size) {
    return run_text(ctx, token_ids, attention_mask, n_tokens, 1, n_layers, apply_final_norm != 0, out, out_size,
                    "graph compute failed");
}

}  // extern "C"
