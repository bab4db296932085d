// VAE decoder: load (weight-norm fold, fp16 GEMM layouts) and decode orchestration (see vae.h).
#include "vae.h"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <filesystem>

#include "json.h"
#include "safetensors.h"

namespace acemi {
namespace {

uint16_t f32_to_f16_bits(float f) {  // GGML_FP32_TO_FP16 (round to nearest even)
    _Float16 h = (_Float16)f;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}

struct VaeLoader {
    VaeModel& m;
    StFile st;
    explicit VaeLoader(VaeModel& mm) : m(mm) {}

    template <typename T>
    T* upload(const void* host, size_t bytes) {
        void* d = nullptr;
        ACEMI_HIP(hipMalloc(&d, bytes));
        m.allocs.push_back(d);
        ACEMI_HIP(hipMemcpy(d, host, bytes, hipMemcpyHostToDevice));
        ACEMI_HIP(hipDeviceSynchronize());  // null-stream copy: done before any stream reads it
        m.weight_bytes += bytes;
        return static_cast<T*>(d);
    }
    std::vector<float> tensor(const std::string& name, std::vector<int64_t>& shape) {
        const auto& t = st.get(name);
        shape = t.shape;
        return to_f32(t, st.read(t));
    }
    // load_snake (:489-503): alpha/beta [1][C][1] -> exp() on the host (ggml_exp of the CPU graph)
    VaeSnake snake(const std::string& prefix, int C) {
        VaeSnake s;
        s.C = C;
        for (int which = 0; which < 2; ++which) {
            std::vector<int64_t> sh;
            auto v = tensor(prefix + (which ? ".beta" : ".alpha"), sh);
            if ((int64_t)v.size() != C) throw IoError("invalid tensor shape for " + prefix);
            for (auto& x : v) x = expf(x);
            (which ? s.eb : s.ea) = upload<float>(v.data(), v.size() * 4);
        }
        return s;
    }
    // load_conv_weight_norm (:520-588): w = v * (g / sqrtf((float)sum(v^2) + 1e-12f)) per dim-0 slice
    std::vector<float> fold(const std::string& prefix, std::vector<int64_t>& vshape) {
        std::vector<int64_t> gshape;
        auto g = tensor(prefix + ".weight_g", gshape);
        auto v = tensor(prefix + ".weight_v", vshape);
        if (vshape.size() != 3 || gshape.size() != 3) throw IoError("invalid weight-norm tensor shape for " + prefix);
        const int64_t d0 = vshape[0], row = vshape[1] * vshape[2];
        if ((int64_t)g.size() != d0) throw IoError("weight_g size mismatch for " + prefix);
        std::vector<float> w(v.size());
        for (int64_t i = 0; i < d0; ++i) {
            double ss = 0.0;
            for (int64_t j = 0; j < row; ++j) ss += (double)v[i * row + j] * (double)v[i * row + j];
            const float scale = g[i] / std::sqrt(static_cast<float>(ss) + 1e-12f);
            for (int64_t j = 0; j < row; ++j) w[i * row + j] = v[i * row + j] * scale;
        }
        return w;
    }
    float* bias(const std::string& prefix, int cout) {
        std::vector<int64_t> sh;
        auto b = tensor(prefix + ".bias", sh);
        if ((int64_t)b.size() != cout) throw IoError("invalid tensor shape for " + prefix + ".bias");
        return upload<float>(b.data(), b.size() * 4);
    }
    // ggml_conv_1d weight [Cout][Cin][K] -> W [Cout][K][Cin_pad] fp16 (zero columns past Cin)
    VaeConv conv(const std::string& prefix, bool with_bias, int dil, int pad, int stride = 1, int cin_pad_to = 1) {
        std::vector<int64_t> sh;
        auto w = fold(prefix, sh);
        VaeConv c;
        c.cout = (int)sh[0];
        c.cin_real = (int)sh[1];
        c.cin = (c.cin_real + cin_pad_to - 1) / cin_pad_to * cin_pad_to;
        c.taps = (int)sh[2];
        c.dil = dil;
        c.pad = pad;
        c.stride = stride;
        std::vector<uint16_t> h((size_t)c.cout * c.taps * c.cin, 0);
        for (int co = 0; co < c.cout; ++co)
            for (int ci = 0; ci < c.cin_real; ++ci)
                for (int k = 0; k < c.taps; ++k)
                    h[((size_t)co * c.taps + k) * c.cin + ci] =
                        f32_to_f16_bits(w[((size_t)co * c.cin_real + ci) * c.taps + k]);
        c.w = upload<uint16_t>(h.data(), h.size() * 2);
        if (with_bias) c.b = bias(prefix, c.cout);
        return c;
    }
    // ConvTranspose1d weight [Cin][Cout][2s] -> W [s*Cout][2*Cin]: W[r*Cout+co][tap*Cin+ci] = w[ci][co][r+tap*s]
    VaeConv conv_t(const std::string& prefix, int stride) {
        std::vector<int64_t> sh;
        auto w = fold(prefix, sh);
        VaeConv c;
        c.transposed = true;
        c.cin = c.cin_real = (int)sh[0];
        c.cout = (int)sh[1];
        c.stride = stride;
        c.pad = (stride + 1) / 2;  // ceil(stride / 2) (:575)
        c.taps = 2;
        if (sh[2] != 2LL * stride) throw Unsupported("conv_t kernel must be 2*stride (" + prefix + ")");
        std::vector<uint16_t> h((size_t)stride * c.cout * 2 * c.cin);
        for (int r = 0; r < stride; ++r)
            for (int co = 0; co < c.cout; ++co)
                for (int tap = 0; tap < 2; ++tap)
                    for (int ci = 0; ci < c.cin; ++ci)
                        h[((size_t)(r * c.cout + co) * 2 + tap) * c.cin + ci] =
                            f32_to_f16_bits(w[((size_t)ci * c.cout + co) * (2 * stride) + r + tap * stride]);
        c.w = upload<uint16_t>(h.data(), h.size() * 2);
        c.b = bias(prefix, c.cout);
        return c;
    }
};

void check_gemm_conv(const VaeConv& c, const std::string& what) {
    if (c.cin % 64 != 0) throw Unsupported(what + ": input channels must be a multiple of 64");
    const int n = c.transposed ? c.stride * c.cout : c.cout;
    if (n % 128 != 0) throw Unsupported(what + ": output columns must be a multiple of 128");
}

}  // namespace

VaeModel::~VaeModel() {
    for (void* p : allocs) (void)hipFree(p);
}

void load_vae_model(const std::string& dir, VaeModel& m, int& status_hint) {
    status_hint = 3;
    try {
        namespace fs = std::filesystem;
        const fs::path p(dir);
        const fs::path root = p.extension() == ".gguf" ? p.parent_path() : p;
        for (const char* key : {"ACE_GGML_VAE_GGUF", "ACE_GGML_VAE_GGUF_PATH"}) {  // resolve_gguf_path (:127-150)
            const char* v = std::getenv(key);
            if (v && v[0] && fs::exists(v)) throw Unsupported("GGUF VAE weights are not supported by the MI355X engine yet");
        }
        if ((p.extension() == ".gguf" && fs::exists(p)) || (fs::is_directory(p) && fs::exists(p / "model.gguf")))
            throw Unsupported("GGUF VAE weights are not supported by the MI355X engine yet");
        if (const char* f = std::getenv("ACE_GGML_VAE_TRANSPOSE_CONV_F32"); f && f[0] && std::strcmp(f, "0") != 0)
            throw Unsupported("ACE_GGML_VAE_TRANSPOSE_CONV_F32 (f32 transposed-conv weights) is not supported");

        // load_config (:55-125)
        VaeConfig& c = m.cfg;
        std::string text;
        try {
            text = read_file((root / "config.json").string());
        } catch (const std::exception&) {
            throw IoError("failed to open file: " + (root / "config.json").string());
        }
        Json o;
        try {
            o = Json::parse(text);
        } catch (const std::exception& e) {
            throw IoError(std::string("failed to parse VAE config: ") + e.what());
        }
        if (o.kind != Json::Object) throw IoError("VAE config is not a JSON object");
        auto get_int = [&](const char* key, int& out) {
            if (!o.has(key) || o.at(key).kind != Json::Number)
                throw IoError(std::string("missing or invalid integer key: ") + key);
            out = (int)o.at(key).as_int();
        };
        auto get_arr = [&](const char* key, std::vector<int>& out) {
            if (!o.has(key) || o.at(key).kind != Json::Array)
                throw IoError(std::string("missing or invalid array key: ") + key);
            out.clear();
            for (const auto& v : o.at(key).arr) {
                if (v.kind != Json::Number) throw IoError(std::string("non-numeric value in array: ") + key);
                out.push_back((int)v.as_int());
            }
        };
        get_int("audio_channels", c.audio_channels);
        get_int("encoder_hidden_size", c.encoder_hidden_size);
        get_int("decoder_channels", c.decoder_channels);
        get_int("decoder_input_channels", c.decoder_input_channels);
        get_int("sampling_rate", c.sampling_rate);
        get_arr("downsampling_ratios", c.downsampling_ratios);
        get_arr("channel_multiples", c.channel_multiples);
        if (c.downsampling_ratios.empty() || c.channel_multiples.empty())
            throw IoError("invalid VAE config: empty ratios or channel multiples");
        c.upsampling_ratios.assign(c.downsampling_ratios.rbegin(), c.downsampling_ratios.rend());
        c.hop_length = 1;
        for (int r : c.downsampling_ratios) c.hop_length *= r;

        VaeLoader L(m);
        L.st.open((root / "diffusion_pytorch_model.safetensors").string());
        m.conv1 = L.conv("decoder.conv1", true, 1, 3);
        check_gemm_conv(m.conv1, "decoder.conv1");
        if (m.conv1.cin != c.decoder_input_channels) throw IoError("decoder.conv1 input channels mismatch");
        int C = m.conv1.cout;
        m.blocks.resize(c.upsampling_ratios.size());
        for (size_t i = 0; i < m.blocks.size(); ++i) {
            const std::string p2 = "decoder.block." + std::to_string(i);
            VaeBlock& b = m.blocks[i];
            b.stride = c.upsampling_ratios[i];
            b.s1 = L.snake(p2 + ".snake1", C);
            b.ct = L.conv_t(p2 + ".conv_t1", b.stride);
            if (b.ct.cin != C) throw IoError("channel mismatch at " + p2 + ".conv_t1");
            check_gemm_conv(b.ct, p2 + ".conv_t1");
            C = b.ct.cout;
            const int dils[3] = {1, 3, 9};
            for (int j = 0; j < 3; ++j) {
                const std::string q = p2 + ".res_unit" + std::to_string(j + 1);
                VaeRes& r = b.res[j];
                r.dil = dils[j];
                r.s1 = L.snake(q + ".snake1", C);
                r.c1 = L.conv(q + ".conv1", true, dils[j], ((7 - 1) * dils[j]) / 2);
                r.s2 = L.snake(q + ".snake2", C);
                r.c2 = L.conv(q + ".conv2", true, 1, 0);
                if (r.c1.cin != C || r.c1.cout != C || r.c2.cin != C || r.c2.cout != C || r.c1.taps != 7 ||
                    r.c2.taps != 1)
                    throw IoError("invalid residual unit shape at " + q);
                check_gemm_conv(r.c1, q + ".conv1");
                check_gemm_conv(r.c2, q + ".conv2");
            }
        }
        m.snake1 = L.snake("decoder.snake1", C);
        m.conv2 = L.conv("decoder.conv2", false, 1, 3);
        if (m.conv2.cin != C || m.conv2.taps != 7 || m.conv2.cout != c.audio_channels)
            throw IoError("invalid decoder.conv2 shape");
        if (C % 8 != 0) throw Unsupported("decoder.conv2 input channels must be a multiple of 8");

        // encoder (load_model_from_dir :925-937): conv1 (k7, pad 3), blocks (3 residual units, Snake,
        // conv k=2s stride s pad ceil(s/2)), snake1, conv2 (k3, pad 1) -> [mean | scale]
        if (L.st.has("encoder.conv1.weight_v")) {
            m.enc_conv1 = L.conv("encoder.conv1", true, 1, 3, 1, 64);
            if (m.enc_conv1.cin_real != c.audio_channels) throw IoError("encoder.conv1 input channels mismatch");
            check_gemm_conv(m.enc_conv1, "encoder.conv1");
            int Ce = m.enc_conv1.cout;
            m.enc_blocks.resize(c.downsampling_ratios.size());
            for (size_t i = 0; i < m.enc_blocks.size(); ++i) {
                const std::string p2 = "encoder.block." + std::to_string(i);
                VaeEncBlock& b = m.enc_blocks[i];
                b.stride = c.downsampling_ratios[i];
                const int dils[3] = {1, 3, 9};
                for (int j = 0; j < 3; ++j) {
                    const std::string q = p2 + ".res_unit" + std::to_string(j + 1);
                    VaeRes& r = b.res[j];
                    r.dil = dils[j];
                    r.s1 = L.snake(q + ".snake1", Ce);
                    r.c1 = L.conv(q + ".conv1", true, dils[j], ((7 - 1) * dils[j]) / 2);
                    r.s2 = L.snake(q + ".snake2", Ce);
                    r.c2 = L.conv(q + ".conv2", true, 1, 0);
                    if (r.c1.cin != Ce || r.c1.cout != Ce || r.c2.cin != Ce || r.c2.cout != Ce || r.c1.taps != 7 ||
                        r.c2.taps != 1)
                        throw IoError("invalid residual unit shape at " + q);
                    check_gemm_conv(r.c1, q + ".conv1");
                    check_gemm_conv(r.c2, q + ".conv2");
                }
                b.s1 = L.snake(p2 + ".snake1", Ce);
                b.conv = L.conv(p2 + ".conv1", true, 1, (b.stride + 1) / 2, b.stride);
                if (b.conv.cin != Ce || b.conv.taps != 2 * b.stride) throw IoError("invalid shape at " + p2 + ".conv1");
                check_gemm_conv(b.conv, p2 + ".conv1");
                Ce = b.conv.cout;
            }
            m.enc_snake1 = L.snake("encoder.snake1", Ce);
            m.enc_conv2 = L.conv("encoder.conv2", true, 1, 1);
            if (m.enc_conv2.cin != Ce || m.enc_conv2.cout < c.decoder_input_channels)
                throw IoError("invalid encoder.conv2 shape");
            check_gemm_conv(m.enc_conv2, "encoder.conv2");
            m.has_encoder = true;
        }
    } catch (const Unsupported& e) {
        status_hint = 4;
        throw std::runtime_error(e.what());
    } catch (const HipError&) {
        status_hint = 1;
        throw;
    }
}

VaeEngine::~VaeEngine() {
    for (Buf* b : {&x_, &sa_, &sb_, &sc_, &lat_, &zero_})
        if (b->p) (void)hipFree(b->p);
}

void VaeEngine::ensure(Buf& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return;
    if (b.p) {
        ACEMI_HIP(hipDeviceSynchronize());
        ACEMI_HIP(hipFree(b.p));
        b.p = nullptr;
        b.bytes = 0;
    }
    const size_t alloc = (bytes + 255) & ~size_t(255);
    ACEMI_HIP(hipMalloc(&b.p, alloc));
    ACEMI_HIP(hipMemset(b.p, 0, alloc));
    // hipMemset runs on the legacy null stream, which does not order against the library's
    // non-blocking streams: finish it before any kernel can write the new buffer
    ACEMI_HIP(hipDeviceSynchronize());
    b.bytes = alloc;
}

int64_t VaeEngine::out_len(int n_frames) const {
    int64_t L = n_frames;
    for (const auto& b : model_.blocks) {
        // PyTorch ConvTranspose1d length with padding ceil(s/2), kernel 2s (conv_forward :697-708)
        const int64_t full = (L + 1) * b.stride;
        const int64_t target = full - 2 * b.ct.pad;
        if (b.ct.pad > 0 && target > 0 && target < full) L = target;
        else L = full;
    }
    return L;
}

void VaeEngine::run_conv(const VaeConv& c, const uint16_t* S, int T_in, int T_out, float* X, bool resid, bool store,
                         uint16_t* S_out, const VaeSnake* next, hipStream_t s) {
    ConvGemmArgs a;
    a.S = S;
    a.zero = static_cast<const uint16_t*>(zero_.p);
    a.W = c.w;
    a.T_in = T_in;
    a.Cin = c.cin;
    a.taps = c.taps;
    a.bias = c.b;
    a.Cout = c.cout;
    a.T_out = T_out;
    if (c.transposed) {
        a.dil = -1;  // tap 0 -> input row j, tap 1 -> row j-1
        a.pad = 0;
        a.M = T_in + 1;
        a.N = c.stride * c.cout;
        a.up = c.stride;
        a.crop = c.pad;
    } else {
        a.dil = c.dil;
        a.pad = c.pad;
        a.in_stride = c.stride;
        a.M = T_out;
        a.N = c.cout;
    }
    a.X = X;
    a.resid = resid ? 1 : 0;
    a.store_x = store ? 1 : 0;
    a.S_out = S_out;
    a.items = items_;
    a.M *= items_;
    if (next) {
        a.snake_ea = next->ea;
        a.snake_eb = next->eb;
    }
    if (fused2_) {
        a.W2 = fused2_->c2.w;
        a.bias2 = fused2_->c2.b;
        a.snake2_ea = fused2_->s2.ea;
        a.snake2_eb = fused2_->s2.eb;
    }
    launch_conv_gemm(a, s);
}

// residual_forward (:724-733): x += conv2(snake2(conv1(snake1(x)))); Sin holds snake1(x); the new x's
// Snake for the next consumer goes to Snext_out
// residual_forward (:724-733): x += conv2(snake2(conv1(snake1(x)))); Sin holds snake1(x).  The new x's Snake
// for the next consumer goes to Sout, or (Sout null) to any free buffer of {Sin, Sspare}; returns that buffer.
uint16_t* VaeEngine::run_res(const VaeRes& r, int L, float* X, uint16_t* Sin, uint16_t* Sspare, uint16_t* Sout,
                             const VaeSnake* next, hipStream_t s) {
    if (fuse_res_ && r.c1.cout == 128 && r.c2.cin == 128 && r.c2.cout == 128 && r.c2.taps == 1 && !r.c1.transposed) {
        // one launch: the k1 conv runs on the k7 conv's output tile (ConvGemmArgs::W2), no Stmp round trip;
        // its output cannot overwrite Sin, which other tiles still read (dilated taps)
        uint16_t* out = Sout ? Sout : Sspare;
        fused2_ = &r;
        run_conv(r.c1, Sin, L, L, X, true, true, out, next, s);
        fused2_ = nullptr;
        return out;
    }
    uint16_t* out = Sout ? Sout : Sin;
    run_conv(r.c1, Sin, L, L, nullptr, false, false, Sspare, &r.s2, s);
    run_conv(r.c2, Sspare, L, L, X, true, true, out, next, s);
    return out;
}

namespace {
int64_t convt_len(int64_t L, const VaeConv& c) {  // PyTorch ConvTranspose1d length (conv_forward :697-708)
    const int64_t full = (L + 1) * c.stride, target = full - 2 * c.pad;
    return (c.pad > 0 && target > 0 && target < full) ? target : full;
}
int64_t conv_len(int64_t L, const VaeConv& c) {  // ggml_conv_1d output length
    return (L + 2 * c.pad - (int64_t)c.dil * (c.taps - 1) - 1) / c.stride + 1;
}
}  // namespace

void VaeEngine::decode(const float* d_latents, int n_frames, float* d_out, hipStream_t s, int items) {
    const VaeModel& m = model_;
    ACEMI_CHECK(n_frames >= 1, "vae decode: n_frames must be > 0");
    ACEMI_CHECK(items >= 1, "vae decode: items must be > 0");
    // buffer sizes: the largest (length x channels) over the stages
    int64_t L = n_frames, maxe = (int64_t)n_frames * m.conv1.cout;
    for (const auto& b : m.blocks) {
        L = convt_len(L, b.ct);
        maxe = std::max(maxe, L * b.ct.cout);
    }
    ACEMI_CHECK(L * items < (1LL << 31), "vae decode: sequence too long");
    maxe *= items;
    ensure(x_, (size_t)maxe * 4);
    ensure(sa_, (size_t)maxe * 2);
    ensure(sb_, (size_t)maxe * 2);
    ensure(sc_, (size_t)maxe * 2);
    ensure(lat_, (size_t)items * n_frames * m.conv1.cin * 2);
    ensure(zero_, 4096);  // >= 64 fp16 zeros (hipMemset in ensure())

    float* X = static_cast<float*>(x_.p);
    uint16_t* Sa = static_cast<uint16_t*>(sa_.p);
    uint16_t* Sb = static_cast<uint16_t*>(sb_.p);
    uint16_t* Sc = static_cast<uint16_t*>(sc_.p);

    // latents -> fp16 (ggml im2col of decoder.conv1's input)
    launch_to_f16(d_latents, (int64_t)items * n_frames * m.conv1.cin, static_cast<uint16_t*>(lat_.p), s);
    items_ = items;
    const VaeSnake* first = m.blocks.empty() ? &m.snake1 : &m.blocks[0].s1;
    // decoder.conv1 -> X, Sa = snake(next)(X)
    run_conv(m.conv1, static_cast<const uint16_t*>(lat_.p), n_frames, n_frames, X, false, true, Sa, first, s);
    L = n_frames;
    for (size_t i = 0; i < m.blocks.size(); ++i) {
        const VaeBlock& b = m.blocks[i];
        const int64_t Lo = convt_len(L, b.ct);
        // snake1 was applied by the producer of Sa; conv_t1 -> X, Sb = res1.snake1(X)
        run_conv(b.ct, Sa, (int)L, (int)Lo, X, false, true, Sb, &b.res[0].s1, s);
        L = Lo;
        uint16_t* cur = Sb;
        for (int j = 0; j < 3; ++j) {
            const VaeSnake* next = j < 2 ? &b.res[j + 1].s1 : (i + 1 < m.blocks.size() ? &m.blocks[i + 1].s1 : &m.snake1);
            cur = run_res(b.res[j], (int)L, X, cur, cur == Sb ? Sc : Sb, j < 2 ? nullptr : Sa, next, s);
            // test-only negative control: one 16 x 128 tile of the residual stream after the block's first unit (the
            // next unit's input Snake was already formed from the clean X, so the fault enters through the residual)
            if (j == 0 && fault_.block == (int)i)
                launch_fault_tile(X, b.ct.cout, (int)(L * items), fault_.row, fault_.col, fault_.amp, s);
        }
    }
    // decoder.snake1 (applied into Sa) -> decoder.conv2
    items_ = 1;
    launch_conv_out(Sa, (int)L, m.conv2.cin, m.conv2.w, m.conv2.cout, d_out, s, items);
}

int64_t VaeEngine::enc_out_len(int n_samples) const {
    const VaeModel& m = model_;
    int64_t L = conv_len(n_samples, m.enc_conv1);
    for (const auto& b : m.enc_blocks) L = conv_len(L, b.conv);
    return conv_len(L, m.enc_conv2);
}

// forward_encode (acestep_vae_model.cpp:1004-1044)
void VaeEngine::encode(const float* d_audio, int n_samples, float* d_out, hipStream_t s) {
    const VaeModel& m = model_;
    ACEMI_CHECK(m.has_encoder, "vae encoder weights not loaded");
    ACEMI_CHECK(n_samples >= 1, "vae encode: n_samples must be > 0");
    items_ = 1;
    int64_t L = conv_len(n_samples, m.enc_conv1);
    int64_t maxe = (int64_t)n_samples * m.enc_conv1.cin;  // padded input
    maxe = std::max(maxe, L * m.enc_conv1.cout);
    for (const auto& b : m.enc_blocks) {
        maxe = std::max(maxe, L * b.conv.cin);
        L = conv_len(L, b.conv);
        ACEMI_CHECK(L >= 1, "vae encode: input too short");
        maxe = std::max(maxe, L * b.conv.cout);
    }
    const int64_t Lf = conv_len(L, m.enc_conv2);
    ACEMI_CHECK(Lf >= 1, "vae encode: input too short");
    maxe = std::max(maxe, Lf * m.enc_conv2.cout);
    ensure(x_, (size_t)maxe * 4);
    ensure(sa_, (size_t)maxe * 2);
    ensure(sb_, (size_t)maxe * 2);
    ensure(sc_, (size_t)maxe * 2);
    ensure(zero_, 4096);
    float* X = static_cast<float*>(x_.p);
    uint16_t* Sa = static_cast<uint16_t*>(sa_.p);
    uint16_t* Sb = static_cast<uint16_t*>(sb_.p);
    uint16_t* Sc = static_cast<uint16_t*>(sc_.p);

    // audio [n][C] -> fp16 [n][64] (zero-padded channels; ggml im2col of encoder.conv1's input)
    launch_pack_f16(d_audio, n_samples, m.enc_conv1.cin_real, m.enc_conv1.cin, Sa, s);
    L = conv_len(n_samples, m.enc_conv1);
    const VaeSnake* first = m.enc_blocks.empty() ? &m.enc_snake1 : &m.enc_blocks[0].res[0].s1;
    run_conv(m.enc_conv1, Sa, n_samples, (int)L, X, false, true, Sb, first, s);
    for (size_t i = 0; i < m.enc_blocks.size(); ++i) {
        const VaeEncBlock& b = m.enc_blocks[i];
        uint16_t* cur = Sb;
        for (int j = 0; j < 3; ++j) {
            const VaeSnake* next = j < 2 ? &b.res[j + 1].s1 : &b.s1;
            cur = run_res(b.res[j], (int)L, X, cur, cur == Sb ? Sc : Sb, j < 2 ? nullptr : Sa, next, s);
        }
        // block snake1 (in Sa) -> strided conv -> X, Sb = snake(next)(X)
        const int64_t Lo = conv_len(L, b.conv);
        const VaeSnake* next = i + 1 < m.enc_blocks.size() ? &m.enc_blocks[i + 1].res[0].s1 : &m.enc_snake1;
        run_conv(b.conv, Sa, (int)L, (int)Lo, X, false, true, Sb, next, s);
        L = Lo;
    }
    // encoder.snake1 (in Sb) -> conv2 -> X [Lf][2*latent]; keep the mean half (:1037-1043)
    run_conv(m.enc_conv2, Sb, (int)L, (int)Lf, X, false, true, nullptr, nullptr, s);
    const int lat = model_.cfg.decoder_input_channels;
    ACEMI_HIP(hipMemcpy2DAsync(d_out, (size_t)lat * 4, X, (size_t)m.enc_conv2.cout * 4, (size_t)lat * 4, (size_t)Lf,
                               hipMemcpyDeviceToDevice, s));
}

}  // namespace acemi
