// extern "C" entry points of libacestep_mi355x.so (include/acestep_ggml.h, include/acestep_mi355x.h).
//
// Status/error behaviour follows the reference implementation
// (acestep_ggml/cpp/acestep_ggml.cpp:65-70 ace_set_error, :108-194 create,
// :230-236 last_error, :260-357 load_dit, :1304-1482 dit_forward).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "context.h"

using namespace acemi_abi;

extern "C" {

ace_ggml_status ace_ggml_create(const ace_ggml_init_params* params, ace_ggml_context** out_ctx) {
    if (!out_ctx) return ACE_GGML_ERR_INVALID_ARG;
    ace_ggml_context* ctx = new (std::nothrow) ace_ggml_context();
    if (!ctx) return ACE_GGML_ERR;
    if (params) {
        ctx->n_threads = params->n_threads;
        ctx->use_metal = params->use_metal != 0;
        ctx->compute_buffer_bytes = params->compute_buffer_bytes;
    }
    if (ctx->compute_buffer_bytes == 0) ctx->compute_buffer_bytes = 512ULL * 1024ULL * 1024ULL;
    *out_ctx = ctx;
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_create_on_device(const ace_ggml_init_params* params, int32_t device,
                                        ace_ggml_context** out_ctx) {
    ace_ggml_status st = ace_ggml_create(params, out_ctx);
    if (st != ACE_GGML_OK) return st;
    if (device < 0) {
        ace_ggml_destroy(*out_ctx);
        *out_ctx = nullptr;
        return ACE_GGML_ERR_INVALID_ARG;
    }
    (*out_ctx)->device = device;
    return ACE_GGML_OK;
}

void ace_ggml_destroy(ace_ggml_context* ctx) {
    if (!ctx) return;
    if (ctx->device >= 0) (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    ctx->dit.reset();
    ctx->vae.reset();
    ctx->text.reset();
    if (ctx->d_vae) (void)hipFree(ctx->d_vae);
    if (ctx->d_in) (void)hipFree(ctx->d_in);
    if (ctx->d_v) (void)hipFree(ctx->d_v);
    if (ctx->d_sched) (void)hipFree(ctx->d_sched);
    if (ctx->stream) {
        try {
            acemi::gemm_splitk_release(ctx->stream);
        } catch (const std::exception&) {
        }
        (void)hipStreamDestroy(ctx->stream);
    }
    delete ctx;
}

const char* ace_ggml_last_error(const ace_ggml_context* ctx) {
    if (!ctx) return "ace_ggml_last_error: null context";
    return ctx->last_error.c_str();
}

ace_ggml_status ace_ggml_load_dit(ace_ggml_context* ctx, const char* model_dir) {
    if (!ctx || !model_dir) return ACE_GGML_ERR_INVALID_ARG;
    int hint = 3;
    try {
        bind_device(ctx);
        ACEMI_HIP(hipStreamSynchronize(ctx->stream));
        ctx->dit.reset();
        auto eng = std::make_unique<acemi::DitEngine>(ctx->device);
        acemi::load_dit_model(model_dir, eng->model(), hint);
        ctx->dit = std::move(eng);
    } catch (const acemi::HipError& e) {
        ctx->dit.reset();
        return set_error(ctx, ACE_GGML_ERR, e.what());
    } catch (const std::exception& e) {
        ctx->dit.reset();
        return set_error(ctx, hint == 4 ? ACE_GGML_ERR_UNSUPPORTED : (hint == 1 ? ACE_GGML_ERR : ACE_GGML_ERR_IO),
                         e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_ggml_dit_forward(ace_ggml_context* ctx, const float* hidden_states, const float* context_latents,
                                     const float* encoder_hidden_states, const int32_t* attention_mask,
                                     const int32_t* encoder_attention_mask, int32_t seq_len, int32_t enc_len,
                                     float timestep, float timestep_r, float* out, size_t out_size) {
    if (!ctx || !out || seq_len <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    const acemi::DitConfig& c = ctx->dit->model().cfg;
    const int audio = c.audio_dim, cdim = c.ctx_dim(), H = c.hidden;
    const size_t needed = (size_t)audio * (size_t)seq_len * sizeof(float);
    if (out_size < needed) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");
    const int L = enc_len > 0 ? enc_len : 0;
    if (L > 0 && !encoder_hidden_states) return set_error(ctx, ACE_GGML_ERR, "dit forward failed");
    const bool profile = env_enabled("ACE_GGML_DIT_PROFILE");
    try {
        const auto t0 = std::chrono::steady_clock::now();
        bind_device(ctx);
        hipStream_t s = ctx->stream;
        // device staging layout: hidden | context | enc | mask | enc_mask | t | r | out
        const size_t n_h = (size_t)seq_len * audio, n_c = (size_t)seq_len * cdim, n_e = (size_t)L * H;
        auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
        const size_t o_h = 0, o_c = o_h + al(n_h * 4), o_e = o_c + al(n_c * 4), o_m = o_e + al(n_e * 4),
                     o_em = o_m + al((size_t)seq_len * 4), o_t = o_em + al((size_t)L * 4 + 4), o_out = o_t + 256,
                     total = o_out + al(n_h * 4);
        ensure_dev(ctx->d_in, ctx->d_in_bytes, total);
        char* base = static_cast<char*>(ctx->d_in);
        acemi::ForwardIO io;
        io.B = 1;
        io.T = seq_len;
        io.L = L;
        if (hidden_states) {
            ACEMI_HIP(hipMemcpyAsync(base + o_h, hidden_states, n_h * 4, hipMemcpyHostToDevice, s));
            io.hidden = reinterpret_cast<const float*>(base + o_h);
        }
        if (context_latents) {
            ACEMI_HIP(hipMemcpyAsync(base + o_c, context_latents, n_c * 4, hipMemcpyHostToDevice, s));
            io.context = reinterpret_cast<const float*>(base + o_c);
        }
        if (L > 0) {
            ACEMI_HIP(hipMemcpyAsync(base + o_e, encoder_hidden_states, n_e * 4, hipMemcpyHostToDevice, s));
            io.enc = reinterpret_cast<const float*>(base + o_e);
        }
        if (attention_mask) {
            ACEMI_HIP(hipMemcpyAsync(base + o_m, attention_mask, (size_t)seq_len * 4, hipMemcpyHostToDevice, s));
            io.mask = reinterpret_cast<const int32_t*>(base + o_m);
        }
        if (encoder_attention_mask && L > 0) {
            ACEMI_HIP(hipMemcpyAsync(base + o_em, encoder_attention_mask, (size_t)L * 4, hipMemcpyHostToDevice, s));
            io.enc_mask = reinterpret_cast<const int32_t*>(base + o_em);
        }
        const float tr[2] = {timestep, timestep_r};
        ACEMI_HIP(hipMemcpyAsync(base + o_t, tr, 8, hipMemcpyHostToDevice, s));
        io.t = reinterpret_cast<const float*>(base + o_t);
        io.r = reinterpret_cast<const float*>(base + o_t + 4);
        io.out = reinterpret_cast<float*>(base + o_out);
        io.max_layers = max_layers_env();
        ACEMI_HIP(hipStreamSynchronize(s));
        const auto t1 = std::chrono::steady_clock::now();
        ctx->dit->forward(io, s);
        ACEMI_HIP(hipStreamSynchronize(s));
        acemi::gemm_splitk_check();
        const auto t2 = std::chrono::steady_clock::now();
        ACEMI_HIP(hipMemcpyAsync(out, io.out, needed, hipMemcpyDeviceToHost, s));
        ACEMI_HIP(hipStreamSynchronize(s));
        const auto t3 = std::chrono::steady_clock::now();
        if (profile) {
            using ms = std::chrono::duration<double, std::milli>;
            std::fprintf(stderr,
                         "ace_ggml_dit_forward profile: backend=mi355x seq=%d enc=%d device=%d upload_ms=%.3f "
                         "compute_ms=%.3f copy_ms=%.3f total_ms=%.3f\n",
                         seq_len, L, ctx->device, ms(t1 - t0).count(), ms(t2 - t1).count(), ms(t3 - t2).count(),
                         ms(t3 - t0).count());
        }
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("dit forward failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_dit_get_info(ace_ggml_context* ctx, ace_mi_dit_info* out) {
    if (!ctx || !out) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    const auto& m = ctx->dit->model();
    const auto& c = m.cfg;
    out->hidden_size = c.hidden;
    out->intermediate_size = c.intermediate;
    out->num_layers = c.layers;
    out->num_heads = c.hq;
    out->num_kv_heads = c.hkv;
    out->head_dim = c.head_dim;
    out->patch_size = c.patch;
    out->in_channels = c.in_channels;
    out->audio_dim = c.audio_dim;
    out->sliding_window = c.sliding_window;
    out->act_type = static_cast<int32_t>(m.act);
    out->device = ctx->device;
    out->weight_bytes = static_cast<int64_t>(m.weight_bytes);
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_dit_forward_batched(ace_ggml_context* ctx, int32_t batch, const float* d_hidden,
                                           const float* d_context, const float* d_enc, const int32_t* d_mask,
                                           const int32_t* d_enc_mask, int32_t seq_len, int32_t enc_len,
                                           const float* d_timestep, const float* d_timestep_r, float* d_out,
                                           void* stream) {
    if (!ctx || !d_out || seq_len <= 0 || batch <= 0 || !d_timestep || !d_timestep_r)
        return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    if (enc_len > 0 && !d_enc) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "encoder_hidden_states is null");
    try {
        bind_device(ctx);
        acemi::gemm_splitk_check();  // a failure of an earlier asynchronous call surfaces here
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
        acemi::ForwardIO io;
        io.B = batch;
        io.T = seq_len;
        io.L = enc_len > 0 ? enc_len : 0;
        io.hidden = d_hidden;
        io.context = d_context;
        io.enc = d_enc;
        io.mask = d_mask;
        io.enc_mask = d_enc_mask;
        io.t = d_timestep;
        io.r = d_timestep_r;
        io.out = d_out;
        io.max_layers = max_layers_env();
        ctx->dit->forward(io, s);
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("dit forward failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

namespace {
// The generation loop shared by ace_mi_dit_sample (the C sampler, acestep_ggml.cpp:2042-2086) and
// ace_mi_dit_sample_ex (the Python/MLX loop, acestep/mlx_dit/generate.py:143-199).
ace_ggml_status run_sampler(ace_ggml_context* ctx, int32_t batch, float* d_xt, const float* d_context,
                            const float* d_enc, const int32_t* d_mask, const int32_t* d_enc_mask, int32_t seq_len,
                            int32_t enc_len, const float* schedule, int32_t n_steps, bool sde, const float* d_noise,
                            int32_t cover_steps, const float* d_context_nc, const float* d_enc_nc, bool cache_cross,
                            void* stream) {
    if (!ctx || !d_xt || seq_len <= 0 || batch <= 0 || !schedule || n_steps <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    if (enc_len > 0 && !d_enc) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "encoder_hidden_states is null");
    if (sde && n_steps > 1 && !d_noise) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "sde needs noise");
    try {
        bind_device(ctx);
        acemi::gemm_splitk_check();  // a failure of an earlier asynchronous call surfaces here
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
        const auto& c = ctx->dit->model().cfg;
        const size_t n = (size_t)batch * seq_len * c.audio_dim;
        void* vp = ctx->d_v;
        ensure_dev(vp, ctx->d_v_bytes, n * 4);
        ctx->d_v = static_cast<float*>(vp);
        std::vector<float> tt((size_t)n_steps * batch);
        for (int i = 0; i < n_steps; ++i)
            for (int b = 0; b < batch; ++b) tt[(size_t)i * batch + b] = schedule[i];
        void* sp = ctx->d_sched;
        // sized generously so a longer loop later does not reallocate (hipFree syncs the device)
        ensure_dev(sp, ctx->d_sched_bytes, std::max<size_t>(tt.size() * 4, 64 * 1024));
        ctx->d_sched = static_cast<float*>(sp);
        ACEMI_HIP(hipMemcpyAsync(ctx->d_sched, tt.data(), tt.size() * 4, hipMemcpyHostToDevice, s));
        ACEMI_HIP(hipStreamSynchronize(s));
        acemi::ForwardIO io;
        io.B = batch;
        io.T = seq_len;
        io.L = enc_len > 0 ? enc_len : 0;
        io.hidden = d_xt;
        io.context = d_context;
        io.enc = d_enc;
        io.mask = d_mask;
        io.enc_mask = d_enc_mask;
        io.out = ctx->d_v;
        io.max_layers = max_layers_env();
        // every step's timestep is known now: the timestep MLPs of all steps in one pass (r = t in the sampler)
        const auto ts = ctx->dit->precompute_timesteps(ctx->d_sched, ctx->d_sched, n_steps * batch, s);
        const int H = c.hidden;
        bool switched = false;
        for (int i = 0; i < n_steps; ++i) {
            bool fresh = (i == 0);
            // generate.py:160: `step_idx >= cover_steps and enc_hs_nc is not None` -> non-cover
            // conditions from that step on (a negative cover_steps switches at step 0, a value
            // >= n_steps or a NULL d_enc_nc never switches); the context follows when given
            if (!switched && d_enc_nc && i >= cover_steps) {
                io.enc = d_enc_nc;
                if (d_context_nc) io.context = d_context_nc;
                switched = true;
                fresh = true;
            }
            io.reuse_cross = cache_cross && !fresh;
            io.reuse_stage = i > 0;  // quantized weights: dequantized once per call (engine.h)
            io.t = ctx->d_sched + (size_t)i * batch;
            io.r = io.t;
            io.ts_proj = ts.proj + (size_t)i * batch * 6 * H;
            io.ts_temb_t = ts.temb_t + (size_t)i * batch * H;
            io.ts_temb_r = ts.temb_r + (size_t)i * batch * H;
            ctx->dit->forward(io, s);
            if (i + 1 == n_steps) {  // final step: x0 = xt - v * t
                acemi::launch_euler(d_xt, ctx->d_v, (int64_t)n, schedule[i], s);
            } else if (sde) {
                acemi::launch_sde(d_xt, ctx->d_v, d_noise + (size_t)i * n, (int64_t)n, schedule[i], schedule[i + 1], s);
            } else {
                acemi::launch_euler(d_xt, ctx->d_v, (int64_t)n, schedule[i] - schedule[i + 1], s);
            }
        }
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("dit sample failed: ") + e.what());
    }
    return ACE_GGML_OK;
}
}  // namespace

ace_ggml_status ace_mi_dit_sample(ace_ggml_context* ctx, int32_t batch, float* d_xt, const float* d_context,
                                  const float* d_enc, const int32_t* d_mask, const int32_t* d_enc_mask,
                                  int32_t seq_len, int32_t enc_len, const float* schedule, int32_t n_steps,
                                  void* stream) {
    return run_sampler(ctx, batch, d_xt, d_context, d_enc, d_mask, d_enc_mask, seq_len, enc_len, schedule, n_steps,
                       false, nullptr, -1, nullptr, nullptr, false, stream);
}

ace_ggml_status ace_mi_dit_sample_ex(ace_ggml_context* ctx, int32_t batch, float* d_xt, const float* d_context,
                                     const float* d_enc, const int32_t* d_mask, const int32_t* d_enc_mask,
                                     int32_t seq_len, int32_t enc_len, const float* schedule, int32_t n_steps,
                                     int32_t sde, const float* d_noise, int32_t cover_steps, const float* d_context_nc,
                                     const float* d_enc_nc, int32_t cache_cross, void* stream) {
    return run_sampler(ctx, batch, d_xt, d_context, d_enc, d_mask, d_enc_mask, seq_len, enc_len, schedule, n_steps,
                       sde != 0, d_noise, cover_steps, d_context_nc, d_enc_nc, cache_cross != 0, stream);
}

ace_ggml_status ace_mi_dit_set_attn_precision(ace_ggml_context* ctx, int32_t mode) {
    if (!ctx || mode < 0 || mode > 4) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    static const acemi::AttnPrecision modes[5] = {acemi::AttnPrecision::FP16, acemi::AttnPrecision::SPLIT,
                                                  acemi::AttnPrecision::F32, acemi::AttnPrecision::F8C,
                                                  acemi::AttnPrecision::PV8};
    ctx->dit->set_attn_precision(modes[mode]);
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_profile_enable(ace_ggml_context* ctx, int32_t on) {
    if (!ctx) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    try {
        bind_device(ctx);
        ctx->dit->set_profiling(on != 0);
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_profile_reset(ace_ggml_context* ctx) {
    if (!ctx) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    ctx->dit->reset_times();
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_profile_get(ace_ggml_context* ctx, char* names, size_t names_cap, double* ms, int32_t* counts,
                                   int32_t cap, int32_t* n_out) {
    if (!ctx || !n_out) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    const auto& t = ctx->dit->times();
    *n_out = static_cast<int32_t>(t.names.size());
    size_t pos = 0;
    for (int i = 0; i < cap && i < (int)t.names.size(); ++i) {
        if (ms) ms[i] = t.ms[i];
        if (counts) counts[i] = t.count[i];
        if (names) {
            const std::string& nm = t.names[i];
            if (pos + nm.size() + 1 <= names_cap) {
                std::memcpy(names + pos, nm.c_str(), nm.size() + 1);
                pos += nm.size() + 1;
            }
        }
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_probe_gemm(ace_ggml_context* ctx, int32_t which, int32_t m_rows, int32_t iters) {
    if (!ctx || m_rows <= 0 || iters <= 0 || which < 0 || which > 1) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->dit) return set_error(ctx, ACE_GGML_ERR, "dit not loaded");
    try {
        bind_device(ctx);
        ctx->dit->probe_gemm(which, m_rows, iters, ctx->stream);
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_synchronize(ace_ggml_context* ctx) {
    if (!ctx) return ACE_GGML_ERR_INVALID_ARG;
    try {
        if (ctx->stream) {
            ACEMI_HIP(hipSetDevice(ctx->device));
            ACEMI_HIP(hipStreamSynchronize(ctx->stream));
            acemi::gemm_splitk_check();
        }
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, e.what());
    }
    return ACE_GGML_OK;
}

}  // extern "C"

extern "C" {

// ------------------------------------------------------------------ VAE decoder
// ace_ggml_load_vae / vae_get_info / vae_decode (acestep_ggml.cpp:545-974, acestep_ggml.h:44-55)
ace_ggml_status ace_ggml_load_vae(ace_ggml_context* ctx, const char* model_dir) {
    if (!ctx || !model_dir) return ACE_GGML_ERR_INVALID_ARG;
    int hint = 3;
    try {
        bind_device(ctx);
        ACEMI_HIP(hipStreamSynchronize(ctx->stream));
        ctx->vae.reset();
        auto eng = std::make_unique<acemi::VaeEngine>(ctx->device);
        acemi::load_vae_model(model_dir, eng->model(), hint);
        ctx->vae = std::move(eng);
    } catch (const acemi::HipError& e) {
        ctx->vae.reset();
        return set_error(ctx, ACE_GGML_ERR, e.what());
    } catch (const std::exception& e) {
        ctx->vae.reset();
        return set_error(ctx, hint == 4 ? ACE_GGML_ERR_UNSUPPORTED : (hint == 1 ? ACE_GGML_ERR : ACE_GGML_ERR_IO),
                         e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_ggml_vae_get_info(ace_ggml_context* ctx, int32_t* latent_channels, int32_t* audio_channels,
                                      int32_t* hop_length) {
    if (!ctx) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    const auto& c = ctx->vae->model().cfg;
    if (latent_channels) *latent_channels = c.decoder_input_channels;
    if (audio_channels) *audio_channels = c.audio_channels;
    if (hop_length) *hop_length = c.hop_length;
    return ACE_GGML_OK;
}

ace_ggml_status ace_ggml_vae_decode(ace_ggml_context* ctx, const float* latents, int32_t n_frames, float* out,
                                    size_t out_size) {
    if (!ctx || !latents || !out || n_frames <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    const auto& c = ctx->vae->model().cfg;
    const size_t expected = (size_t)n_frames * (size_t)c.hop_length * (size_t)c.audio_channels * sizeof(float);
    if (out_size < expected) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");
    const bool profile = env_enabled("ACE_GGML_VAE_PROFILE");
    try {
        const auto t0 = std::chrono::steady_clock::now();
        bind_device(ctx);
        hipStream_t s = ctx->stream;
        const int64_t out_len = ctx->vae->out_len(n_frames);
        const size_t needed = (size_t)out_len * (size_t)c.audio_channels * sizeof(float);
        if (out_size < needed) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small for actual output");
        const size_t n_in = (size_t)n_frames * c.decoder_input_channels * sizeof(float);
        const size_t o_out = (n_in + 255) & ~size_t(255);
        ensure_dev(ctx->d_vae, ctx->d_vae_bytes, o_out + needed);
        char* base = static_cast<char*>(ctx->d_vae);
        ACEMI_HIP(hipMemcpyAsync(base, latents, n_in, hipMemcpyHostToDevice, s));
        ACEMI_HIP(hipStreamSynchronize(s));
        const auto t1 = std::chrono::steady_clock::now();
        ctx->vae->decode(reinterpret_cast<const float*>(base), n_frames, reinterpret_cast<float*>(base + o_out), s);
        ACEMI_HIP(hipStreamSynchronize(s));
        const auto t2 = std::chrono::steady_clock::now();
        ACEMI_HIP(hipMemcpyAsync(out, base + o_out, needed, hipMemcpyDeviceToHost, s));
        ACEMI_HIP(hipStreamSynchronize(s));
        const auto t3 = std::chrono::steady_clock::now();
        if (profile) {
            using ms = std::chrono::duration<double, std::milli>;
            std::fprintf(stderr,
                         "ace_ggml_vae_decode profile: backend=mi355x frames=%d out_len=%lld device=%d upload_ms=%.3f "
                         "compute_ms=%.3f copy_ms=%.3f total_ms=%.3f\n",
                         n_frames, (long long)out_len, ctx->device, ms(t1 - t0).count(), ms(t2 - t1).count(),
                         ms(t3 - t2).count(), ms(t3 - t0).count());
        }
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("graph compute failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

// ace_ggml_vae_encode (acestep_ggml.cpp:975-1072): audio [n_samples][audio_channels] -> latent mean
// [n_samples/hop][latent_channels]
ace_ggml_status ace_ggml_vae_encode(ace_ggml_context* ctx, const float* audio, int32_t n_samples, float* out,
                                    size_t out_size) {
    if (!ctx || !audio || !out || n_samples <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    const auto& c = ctx->vae->model().cfg;
    const size_t expected = (size_t)(n_samples / c.hop_length) * (size_t)c.decoder_input_channels * sizeof(float);
    if (out_size < expected) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small");
    if (!ctx->vae->model().has_encoder) return set_error(ctx, ACE_GGML_ERR, "vae encode failed: encoder weights not loaded");
    try {
        bind_device(ctx);
        hipStream_t s = ctx->stream;
        const int64_t out_len = ctx->vae->enc_out_len(n_samples);
        if (out_len <= 0) return set_error(ctx, ACE_GGML_ERR, "unexpected vae output shape");
        const size_t needed = (size_t)out_len * (size_t)c.decoder_input_channels * sizeof(float);
        if (out_size < needed) return set_error(ctx, ACE_GGML_ERR_INVALID_ARG, "output buffer too small for actual output");
        const size_t n_in = (size_t)n_samples * c.audio_channels * sizeof(float);
        const size_t o_out = (n_in + 255) & ~size_t(255);
        ensure_dev(ctx->d_vae, ctx->d_vae_bytes, o_out + needed);
        char* base = static_cast<char*>(ctx->d_vae);
        ACEMI_HIP(hipMemcpyAsync(base, audio, n_in, hipMemcpyHostToDevice, s));
        ctx->vae->encode(reinterpret_cast<const float*>(base), n_samples, reinterpret_cast<float*>(base + o_out), s);
        ACEMI_HIP(hipMemcpyAsync(out, base + o_out, needed, hipMemcpyDeviceToHost, s));
        ACEMI_HIP(hipStreamSynchronize(s));
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("graph compute failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_vae_enc_out_len(ace_ggml_context* ctx, int32_t n_samples, int64_t* out_len) {
    if (!ctx || !out_len || n_samples <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    if (!ctx->vae->model().has_encoder) return set_error(ctx, ACE_GGML_ERR, "vae encoder weights not loaded");
    *out_len = ctx->vae->enc_out_len(n_samples);
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_vae_encode_device(ace_ggml_context* ctx, const float* d_audio, int32_t n_samples, float* d_out,
                                         void* stream) {
    if (!ctx || !d_audio || !d_out || n_samples <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    try {
        bind_device(ctx);
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
        ctx->vae->encode(d_audio, n_samples, d_out, s);
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("graph compute failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_vae_out_len(ace_ggml_context* ctx, int32_t n_frames, int64_t* out_len) {
    if (!ctx || !out_len || n_frames <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    *out_len = ctx->vae->out_len(n_frames);
    return ACE_GGML_OK;
}

ace_ggml_status ace_mi_vae_decode_device(ace_ggml_context* ctx, const float* d_latents, int32_t n_frames, float* d_out,
                                         void* stream) {
    if (!ctx || !d_latents || !d_out || n_frames <= 0) return ACE_GGML_ERR_INVALID_ARG;
    if (!ctx->vae) return set_error(ctx, ACE_GGML_ERR, "vae not loaded");
    try {
        bind_device(ctx);
        hipStream_t s = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
        ctx->vae->decode(d_latents, n_frames, d_out, s);
    } catch (const std::exception& e) {
        return set_error(ctx, ACE_GGML_ERR, std::string("graph compute failed: ") + e.what());
    }
    return ACE_GGML_OK;
}

}  // extern "C"
