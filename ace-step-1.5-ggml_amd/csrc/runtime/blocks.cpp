// BlockRunner (blocks.h): the encoder-layer loop of the condition encoders and the Qwen3 text encoder.
#include "blocks.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace acemi {

BlockRunner::BlockRunner() {
    // the condition / text encoders (once per request) keep the f32-faithful default
    const AttnPrecision prec = attn_precision_from_env(AttnPrecision::F32);
    split_ = prec != AttnPrecision::FP16;
    pv_split_ = prec == AttnPrecision::F32;
}

BlockRunner::~BlockRunner() {
    for (Buf* b : {&x_, &act_, &attn_, &act2_, &qkv_, &qh_, &kh_, &vt_, &kbias_, &cos_, &sin_})
        if (b->p) (void)hipFree(b->p);
}

void BlockRunner::ensure(Buf& b, size_t bytes) {
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

float* BlockRunner::x(int64_t rows, int H) {
    ensure(x_, (size_t)rows * H * 4);
    return get<float>(x_);
}

void BlockRunner::run(const BlockShape& sh, const std::vector<DevLayer>& layers, int n_layers, ActType at, int B,
                      int n, const int32_t* key_mask, bool causal, hipStream_t s) {
    const int H = sh.hidden, D = sh.head_dim, I = sh.intermediate;
    ACEMI_CHECK(B >= 1 && n >= 1 && D == 128, "blocks: bad shape");
    ACEMI_CHECK(n_layers >= 0 && n_layers <= (int)layers.size(), "blocks: layer count");
    const int64_t M = (int64_t)B * n;
    const int Npad = (int)round_up(n, 128);
    const int qd = sh.hq * D, kd = sh.hkv * D;
    const int64_t q_plane = (int64_t)B * sh.hq * Npad * D;
    const int64_t k_plane = (int64_t)B * sh.hkv * Npad * D;
    ACEMI_CHECK(x_.bytes >= (size_t)M * H * 4, "blocks: residual stream not initialised");
    ensure(act_, (size_t)M * std::max(H, qd) * 2);
    ensure(attn_, (size_t)M * qd * 2);
    ensure(act2_, (size_t)M * std::max(I, 1) * 2);
    ensure(qkv_, (size_t)M * (qd + 2 * kd) * 4);
    ensure(qh_, (size_t)2 * q_plane * 2);
    ensure(kh_, (size_t)2 * k_plane * 2);
    ensure(vt_, (size_t)2 * k_plane * 2);
    ensure(kbias_, (size_t)B * Npad * 4);
    if (rope_n_ != n || rope_theta_ != sh.rope_theta) {  // positions 0..n-1 of each item, ggml's recurrence
        const int half = D / 2;
        const float theta_scale = powf(sh.rope_theta, -2.0f / (float)D);
        std::vector<float> cs((size_t)n * half), sn((size_t)n * half);
        for (int p = 0; p < n; ++p) {
            float theta = (float)p;
            for (int i = 0; i < half; ++i) {
                cs[(size_t)p * half + i] = (float)std::cos((double)theta);  // correctly rounded cosf / sinf
                sn[(size_t)p * half + i] = (float)std::sin((double)theta);
                theta *= theta_scale;
            }
        }
        ACEMI_HIP(hipStreamSynchronize(s));  // the previous pass may still read the old table
        ensure(cos_, cs.size() * 4);
        ensure(sin_, sn.size() * 4);
        ACEMI_HIP(hipMemcpy(cos_.p, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));
        ACEMI_HIP(hipMemcpy(sin_.p, sn.data(), sn.size() * 4, hipMemcpyHostToDevice));
        ACEMI_HIP(hipDeviceSynchronize());  // null-stream copy: done before any stream reads it
        rope_n_ = n;
        rope_theta_ = sh.rope_theta;
    }
    float* x = get<float>(x_);
    uint16_t* act = get<uint16_t>(act_);
    uint16_t* attn = get<uint16_t>(attn_);
    uint16_t* act2 = get<uint16_t>(act2_);
    float* qkv = get<float>(qkv_);
    launch_key_bias(key_mask, B, n, 1, n, Npad, get<float>(kbias_), s);
    const float scale = 1.0f / std::sqrt((float)D);
    for (int li = 0; li < n_layers; ++li) {
        const DevLayer& ly = layers[li];
        launch_rmsnorm_mod(at, x, (int)M, H, ly.self_norm, nullptr, nullptr, 0, n, sh.eps, act, s);
        {
            GemmEpilogue g;
            g.kind = EPI_STORE_F32;
            g.c_f32 = qkv;
            g.ldc = qd + 2 * kd;
            launch_gemm(act, H, ly.w_qkv.view(), (int)M, qd + 2 * kd, H, g, s);
        }
        {
            PrepArgs pa{};
            pa.src = qkv;
            pa.ld = qd + 2 * kd;
            pa.q_col = 0;
            pa.k_col = qd;
            pa.v_col = qd + kd;
            pa.hq = sh.hq;
            pa.hkv = sh.hkv;
            pa.n_tok = n;
            pa.n_pad = Npad;
            pa.B = B;
            pa.q_norm = ly.sq_norm;
            pa.k_norm = ly.sk_norm;
            pa.rope_cos = get<float>(cos_);
            pa.rope_sin = get<float>(sin_);
            pa.eps = sh.eps;
            pa.qh = get<uint16_t>(qh_);
            pa.kh = get<uint16_t>(kh_);
            pa.vt = get<uint16_t>(vt_);
            pa.q_plane = split_ ? q_plane : 0;
            pa.k_plane = split_ ? k_plane : 0;
            pa.v_plane = pv_split_ ? k_plane : 0;
            launch_attn_prep(pa, s);
        }
        {
            AttnArgs aa{};
            aa.q = get<uint16_t>(qh_);
            aa.k = get<uint16_t>(kh_);
            aa.vt = get<uint16_t>(vt_);
            aa.kbias = key_mask ? get<float>(kbias_) : nullptr;  // padding keys are masked in-kernel
            aa.out = attn;
            aa.B = B;
            aa.Hq = sh.hq;
            aa.Hkv = sh.hkv;
            aa.nq = n;
            aa.nq_pad = Npad;
            aa.nk = n;
            aa.nk_pad = Npad;
            aa.window = ly.sliding ? std::max(sh.sliding_window, 0) : 0;
            aa.causal = causal;
            aa.scale = scale;
            aa.split = split_;
            aa.pv_split = pv_split_;
            aa.q_plane = q_plane;
            aa.k_plane = k_plane;
            aa.v_plane = k_plane;
            launch_attention(at, aa, s);
        }
        {
            GemmEpilogue g;  // h = x + o_proj(attn)
            g.kind = EPI_RESID;
            g.c_f32 = x;
            g.ldc = H;
            launch_gemm(attn, qd, ly.w_o.view(), (int)M, H, qd, g, s);
        }
        launch_rmsnorm_mod(at, x, (int)M, H, ly.mlp_norm, nullptr, nullptr, 0, n, sh.eps, act, s);
        {
            GemmEpilogue g;
            g.kind = EPI_SWIGLU;
            g.c_act = act2;
            g.ldc = I;
            launch_gemm(act, H, ly.w_gu.view(), (int)M, 2 * I, H, g, s);
        }
        {
            GemmEpilogue g;  // x = h + down(act)
            g.kind = EPI_RESID;
            g.c_f32 = x;
            g.ldc = H;
            launch_gemm(act2, I, ly.w_down.view(), (int)M, H, I, g, s);
        }
    }
}

void BlockRunner::finish(const BlockShape& sh, const float* w, int B, int n, bool first_only, float* out,
                         hipStream_t s) {
    const int H = sh.hidden;
    const int rows = first_only ? B : B * n;
    const int64_t step = first_only ? n : 1;
    const float* x = get<float>(x_);
    if (w) {
        launch_rmsnorm_f32(x, rows, step, H, w, sh.eps, out, s);
    } else {
        ACEMI_HIP(hipMemcpy2DAsync(out, (size_t)H * 4, x, (size_t)step * H * 4, (size_t)H * 4, rows,
                                   hipMemcpyDeviceToDevice, s));
    }
}

}  // namespace acemi
