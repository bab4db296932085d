// AddressSanitizer / UBSan driver (TEST INFRASTRUCTURE): the product's runtime/*.cpp linked with the
// host kernel emulation (kernel_emul.cpp), built with -fsanitize=address,undefined and driven through the
// C-ABI over every entry family.  "Device" buffers are host allocations here, so a workspace sized
// smaller than what a launch touches, a loader that reads past a tensor, or a bad offset in the ABI
// staging shows up as a sanitizer report instead of a GPU memory fault.
//
// usage: asan_driver <dit_cond_dir> <vae_dir> <text_dir> <dit_gguf_dir> [<malformed_dit_dir>...]
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../include/acestep_mi355x.h"

static int failures = 0;
#define EXPECT(cond)                                                      \
    do {                                                                  \
        if (!(cond)) {                                                    \
            std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond); \
            ++failures;                                                   \
        }                                                                 \
    } while (0)

static std::vector<float> randn(size_t n, unsigned seed) {
    std::mt19937 g(seed);
    std::normal_distribution<float> d(0.f, 1.f);
    std::vector<float> v(n);
    for (auto& x : v) x = d(g);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 5) return 2;
    const char *dit = argv[1], *vae = argv[2], *text = argv[3], *gguf = argv[4];
    ace_ggml_context* ctx = nullptr;
    EXPECT(ace_ggml_create(nullptr, &ctx) == ACE_GGML_OK);
    EXPECT(ace_ggml_load_dit(ctx, dit) == ACE_GGML_OK);
    ace_mi_dit_info info{};
    EXPECT(ace_mi_dit_get_info(ctx, &info) == ACE_GGML_OK);
    const int H = info.hidden_size, A = info.audio_dim, C = info.in_channels - info.audio_dim;

    // DiT forward: odd T (patch padding), masks, short encoder
    {
        const int T = 37, L = 9;
        auto h = randn((size_t)T * A, 1), c = randn((size_t)T * C, 2), e = randn((size_t)L * H, 3);
        std::vector<int32_t> m(T, 1), em(L, 1);
        m[30] = 0;
        em[8] = 0;
        std::vector<float> out((size_t)T * A);
        EXPECT(ace_ggml_dit_forward(ctx, h.data(), c.data(), e.data(), m.data(), em.data(), T, L, 0.7f, 0.4f,
                                    out.data(), out.size() * 4) == ACE_GGML_OK);
        EXPECT(ace_ggml_dit_forward(ctx, h.data(), c.data(), e.data(), nullptr, nullptr, T, L, 0.7f, 0.4f, out.data(),
                                    out.size() * 4 - 4) == ACE_GGML_ERR_INVALID_ARG);
        // batched + the generation loop with SDE, cover switch and the cross cache ("device" = host)
        const int B = 2;
        auto xb = randn((size_t)B * T * A, 4), cb = randn((size_t)B * T * C, 5), eb = randn((size_t)B * L * H, 6);
        auto cnc = randn((size_t)B * T * C, 7), enc2 = randn((size_t)B * L * H, 8);
        auto noise = randn((size_t)3 * B * T * A, 9);
        std::vector<float> tt = {0.9f, 0.6f}, ob((size_t)B * T * A);
        EXPECT(ace_mi_dit_forward_batched(ctx, B, xb.data(), cb.data(), eb.data(), nullptr, nullptr, T, L, tt.data(),
                                          tt.data(), ob.data(), nullptr) == ACE_GGML_OK);
        const float sched[4] = {1.0f, 0.75f, 0.5f, 0.25f};
        EXPECT(ace_mi_dit_sample_ex(ctx, B, xb.data(), cb.data(), eb.data(), nullptr, nullptr, T, L, sched, 4, 1,
                                    noise.data(), 2, cnc.data(), enc2.data(), 1, nullptr) == ACE_GGML_OK);
    }
    // condition encoders
    {
        ace_mi_cond_info ci{};
        EXPECT(ace_mi_cond_get_info(ctx, &ci) == ACE_GGML_OK);
        const int nl = 33, ns = 7, nr = 2, rl = 19;
        auto lyr = randn((size_t)nl * ci.lyric_in_dim, 10), sty = randn((size_t)ns * ci.text_projector_in, 11);
        auto ref = randn((size_t)nr * rl * ci.timbre_in_dim, 12);
        std::vector<float> out((size_t)(nl + ns + nr) * H);
        std::vector<int32_t> mask(nl + ns + nr);
        EXPECT(ace_mi_lyric_encode(ctx, lyr.data(), nl, out.data(), out.size() * 4) == ACE_GGML_OK);
        EXPECT(ace_mi_timbre_encode(ctx, ref.data(), nullptr, nr, rl, out.data(), out.size() * 4) == ACE_GGML_OK);
        EXPECT(ace_mi_text_project(ctx, sty.data(), ns, ci.text_projector_in, out.data(), out.size() * 4) == ACE_GGML_OK);
        int32_t len = 0;
        EXPECT(ace_mi_build_condition(ctx, sty.data(), ns, lyr.data(), nl, ci.lyric_in_dim, ref.data(), nullptr, nr, rl,
                                      out.data(), out.size() * 4, mask.data(), mask.size() * 4, &len) == ACE_GGML_OK);
        EXPECT(len == nl + ns + nr);
        EXPECT(ace_mi_build_condition(ctx, sty.data(), ns, lyr.data(), nl, ci.lyric_in_dim, ref.data(), nullptr, nr, rl,
                                      out.data(), 64, mask.data(), mask.size() * 4, &len) == ACE_GGML_ERR_INVALID_ARG);
    }
    // VAE
    EXPECT(ace_ggml_load_vae(ctx, vae) == ACE_GGML_OK);
    int32_t lat_ch = 0, aud_ch = 0, hop = 0;
    EXPECT(ace_ggml_vae_get_info(ctx, &lat_ch, &aud_ch, &hop) == ACE_GGML_OK);
    {
        const int n = 7;
        auto lat = randn((size_t)n * lat_ch, 13);
        std::vector<float> audio((size_t)n * hop * aud_ch);
        EXPECT(ace_ggml_vae_decode(ctx, lat.data(), n, audio.data(), audio.size() * 4) == ACE_GGML_OK);
        auto wav = randn((size_t)5 * hop * aud_ch, 14);
        std::vector<float> z((size_t)5 * lat_ch);
        EXPECT(ace_ggml_vae_encode(ctx, wav.data(), 5 * hop, z.data(), z.size() * 4) == ACE_GGML_OK);
    }
    // text encoder + end-to-end
    EXPECT(ace_ggml_load_text_encoder(ctx, text) == ACE_GGML_OK);
    {
        std::vector<int32_t> ids = {1, 5, 9, 77, 300, 999, 2, 3, 4, 5, 6};
        std::vector<int32_t> m(ids.size(), 1);
        m.back() = 0;
        std::vector<float> out(ids.size() * 4096);
        EXPECT(ace_ggml_text_encoder_forward(ctx, ids.data(), (int)ids.size(), out.data(), out.size() * 4) == ACE_GGML_OK);
        EXPECT(ace_ggml_text_encoder_forward_masked(ctx, ids.data(), m.data(), (int)ids.size(), out.data(),
                                                    out.size() * 4) == ACE_GGML_OK);
        EXPECT(ace_ggml_text_encoder_forward_layers(ctx, ids.data(), m.data(), (int)ids.size(), 1, 1, out.data(),
                                                    out.size() * 4) == ACE_GGML_OK);
        EXPECT(ace_ggml_text_encoder_forward_embeddings(ctx, ids.data(), (int)ids.size(), out.data(), out.size() * 4) ==
               ACE_GGML_OK);
        ids[2] = 1 << 30;
        EXPECT(ace_ggml_text_encoder_forward(ctx, ids.data(), (int)ids.size(), out.data(), out.size() * 4) ==
               ACE_GGML_ERR_INVALID_ARG);
        ids[2] = 9;
        for (int seq : {20, 150}) {
            std::vector<float> audio((size_t)seq * hop * aud_ch);
            int32_t ns = 0, nc = 0;
            auto refer = randn((size_t)10 * 64, 15);
            EXPECT(ace_ggml_generate_audio_style_lyric_timbre_simple(ctx, ids.data(), 5, ids.data() + 5, 6, refer.data(),
                                                                     nullptr, 1, 10, seq, 3.0f, 7, audio.data(),
                                                                     audio.size() * 4, &ns, &nc) == ACE_GGML_OK);
            EXPECT(ace_ggml_generate_audio_simple(ctx, ids.data(), 5, seq, 2.0f, 8, audio.data(), audio.size() * 4, &ns,
                                                  &nc) == ACE_GGML_OK);
        }
    }
    ace_ggml_destroy(ctx);

    // GGUF DiT and online-quantized DiT in fresh contexts
    for (int mode = 0; mode < 2; ++mode) {
        ace_ggml_context* c2 = nullptr;
        EXPECT(ace_ggml_create(nullptr, &c2) == ACE_GGML_OK);
        if (mode == 1) setenv("ACE_GGML_DIT_WEIGHT_QTYPE", "Q4_K", 1);
        EXPECT(ace_ggml_load_dit(c2, mode == 0 ? gguf : dit) == ACE_GGML_OK);
        const int T = 20, L = 4;
        auto h = randn((size_t)T * A, 16), c = randn((size_t)T * C, 17), e = randn((size_t)L * H, 18);
        std::vector<float> out((size_t)T * A);
        EXPECT(ace_ggml_dit_forward(c2, h.data(), c.data(), e.data(), nullptr, nullptr, T, L, 0.5f, 0.5f, out.data(),
                                    out.size() * 4) == ACE_GGML_OK);
        unsetenv("ACE_GGML_DIT_WEIGHT_QTYPE");
        ace_ggml_destroy(c2);
    }
    // malformed safetensors headers (short data_offsets, end < begin, past the end of the file): the
    // loader must refuse them with IO before any read runs past a tensor's bytes
    for (int i = 5; i < argc; ++i) {
        ace_ggml_context* c3 = nullptr;
        EXPECT(ace_ggml_create(nullptr, &c3) == ACE_GGML_OK);
        EXPECT(ace_ggml_load_dit(c3, argv[i]) == ACE_GGML_ERR_IO);
        ace_ggml_destroy(c3);
    }
    std::printf("asan_driver: %d failures\n", failures);
    return failures == 0 ? 0 : 1;
}
