// The ace_ggml_context behind the C-ABI and the helpers every entry-point file shares
// (status/error behaviour of acestep_ggml.cpp:65-70 ace_set_error).
#pragma once

#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "../../../include/acestep_mi355x.h"
#include "engine.h"
#include "text_encoder.h"
#include "vae.h"

struct ace_ggml_context {
    int32_t n_threads = 0;
    bool use_metal = false;
    size_t compute_buffer_bytes = 0;
    std::string last_error;
    int device = -1;
    hipStream_t stream = nullptr;
    std::unique_ptr<acemi::DitEngine> dit;
    std::unique_ptr<acemi::VaeEngine> vae;
    std::unique_ptr<acemi::TextEncoderEngine> text;  // ace_ggml_load_text_encoder / ace_ggml_load_lm
    void* d_vae = nullptr;  // host-ABI staging for ace_ggml_vae_decode
    size_t d_vae_bytes = 0;
    // host-ABI staging (device)
    void* d_in = nullptr;
    size_t d_in_bytes = 0;
    // sampler scratch
    float* d_v = nullptr;
    size_t d_v_bytes = 0;
    float* d_sched = nullptr;
    size_t d_sched_bytes = 0;
};

namespace acemi_abi {

inline ace_ggml_status set_error(ace_ggml_context* ctx, ace_ggml_status code, const std::string& msg) {
    if (ctx) ctx->last_error = msg;
    return code;
}

inline bool env_enabled(const char* key) {
    const char* v = std::getenv(key);
    return v && v[0] && std::strcmp(v, "0") != 0;
}

inline int env_int(const char* key, int fallback) {
    const char* v = std::getenv(key);
    if (!v || !v[0]) return fallback;
    char* end = nullptr;
    const long long x = std::strtoll(v, &end, 10);
    return (end && end != v) ? static_cast<int>(x) : fallback;
}

// ACE_GGML_DIT_MAX_LAYERS (acestep_dit_model.cpp:1457-1464)
inline int max_layers_env() {
    const int v = env_int("ACE_GGML_DIT_MAX_LAYERS", -1);
    return v > 0 ? v : -1;
}

inline void bind_device(ace_ggml_context* ctx) {
    if (ctx->device < 0) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) throw std::runtime_error("no HIP device available");
        ctx->device = env_int("ACE_MI_DEVICE", 0);
        if (ctx->device >= n) throw std::runtime_error("ACE_MI_DEVICE out of range");
    }
    ACEMI_HIP(hipSetDevice(ctx->device));
    if (!ctx->stream) ACEMI_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
}

inline void ensure_dev(void*& p, size_t& have, size_t need) {
    if (have >= need) return;
    if (p) {
        ACEMI_HIP(hipDeviceSynchronize());  // in-flight work may still use the old staging buffer
        ACEMI_HIP(hipFree(p));
    }
    p = nullptr;
    have = 0;
    ACEMI_HIP(hipMalloc(&p, need));
    have = need;
}

}  // namespace acemi_abi
