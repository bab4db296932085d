// The ggml-faithful quantized-activation forward (ACE_MI_QUANT_ACT=q8): forward_dit (acestep_dit_model.cpp:1316-1560)
// with ggml's own arithmetic for block-format weights.  Every ggml_mul_mat against a Q8_0 / Q4_K / Q6_K weight
// (:1194-1196, 1257, 1295-1302, 1381, 1412, 1528-1531, 1551) converts its f32 input rows to Q8_0 / Q8_K blocks and
// sums d_w * d_a * (integer block dot) in f32 (kernels/gemm_a8.hip); the tensors between the mul_mats stay f32, as in
// the ggml graph: the RMSNorm / AdaLN rows, the attention output (two key-range parts merged in f32), the SwiGLU rows,
// the condition embedding and the timestep MLP's hidden rows.  Attention runs at the f32 precision (hi/lo fp16 for
// both products).  The product forward (engine.cpp) keeps bf16 activations and bf16(dequant(W)); this one exists so
// the quantized configs can be checked against ggml's semantics within the oracle's floor (tests/test_gpu_qact.py).
#include <algorithm>
#include <cmath>

#include "engine.h"

namespace acemi {

void DitEngine::qlinear(const float* x, int64_t ldx, int M, const WeightView& w, int N, int K, const GemmEpilogue& e,
                        const char* name, hipStream_t s, bool silu_in) {
    tic(s);
    if (weight_quantized(w.fmt) && gemm_a8_bf16_path(w.fmt, K)) {
        // Q8_0 on the bf16 MFMA: the activation blocks as bf16(q) rows, the weight as its bf16(q) image (same bits as
        // the i8 kernel below, kernels/gemm_a8.hip gemm_a8s_kernel)
        const int64_t ld_s = round_up(M, 128);
        ensure(qa16_, (size_t)M * K * 2);
        ensure(qs_, (size_t)(K / 32) * ld_s * 4);
        const uint16_t* w16 = q8_image(w, N, K, s);
        launch_quantize_act(QACT_Q8_0, x, ldx, M, K, silu_in, nullptr, get<float>(qs_), nullptr, ld_s, s,
                            get<uint16_t>(qa16_));
        QAct a;
        a.kind = QACT_Q8_0;
        a.q16 = get<uint16_t>(qa16_);
        a.s = get<float>(qs_);
        a.ld_s = ld_s;
        launch_gemm_a8(a, w, M, N, K, e, s, w16);
    } else if (weight_quantized(w.fmt)) {
        const int kind = qact_kind_for(w.fmt);
        const int64_t ld_s = round_up(M, 128);
        ensure(qa_, (size_t)M * K);
        ensure(qs_, (size_t)(K / 32) * ld_s * 4);
        ensure(qb_, (size_t)(K / 32) * ld_s * 4);
        launch_quantize_act(kind, x, ldx, M, K, silu_in, get<int8_t>(qa_), get<float>(qs_), get<float>(qb_), ld_s, s);
        QAct a;
        a.kind = kind;
        a.q = get<int8_t>(qa_);
        a.s = get<float>(qs_);
        a.bsum = get<float>(qb_);
        a.ld_s = ld_s;
        launch_gemm_a8(a, w, M, N, K, e, s);
    } else {
        // a 16-bit weight: ggml rounds the activation to the weight's type (its vec_dot_type) -- the dense GEMM
        ACEMI_CHECK(w.fmt == WF_BF16 || w.fmt == WF_F16, "quantized-activation mode: F32 2-D weights are not supported");
        ACEMI_CHECK(ldx == K && e.kind != EPI_SWIGLU_F32, "quantized-activation mode: unsupported dense linear");
        ensure(qa_, (size_t)M * K * 2);
        uint16_t* xa = get<uint16_t>(qa_);
        launch_to_act(weight_act(w.fmt), x, (int64_t)M * K, silu_in, xa, s);
        launch_gemm(xa, K, w, M, N, K, e, s);
    }
    toc(name, s);
}

// bf16(q) image of a Q8_0 weight's int8 plane, made once on the stream that first needs it and kept while the model is
// loaded (the engine is rebuilt with every load, so a plane pointer names one weight for the cache's lifetime)
const uint16_t* DitEngine::q8_image(const WeightView& w, int N, int K, hipStream_t s) {
    Buf& b = q8img_[w.q];
    if (!b.p) {
        ensure(b, (size_t)N * K * 2);
        launch_q8_image(static_cast<const int8_t*>(w.q), (int64_t)N * K, static_cast<uint16_t*>(b.p), s);
    }
    return static_cast<const uint16_t*>(b.p);
}

void DitEngine::timestep_embed_qact(const float* t, const float* r, int rows, float* proj, float* temb_t,
                                    float* temb_r, hipStream_t s) {
    const DitModel& m = model_;
    const int H = m.cfg.hidden;
    const float log_max = std::log(10000.0f);
    ensure(freq_, (size_t)8 * 256 * 4);
    ensure(th_, (size_t)8 * H * 4);
    float* freq = get<float>(freq_);
    float* th = get<float>(th_);
    for (int e = 0; e < 2; ++e)
        ACEMI_CHECK(m.te[e].q1.q && m.te[e].q2.q && m.te[e].qp.q,
                    "quantized-activation mode: load the model with ACE_MI_QUANT_ACT=q8 set");
    for (int r0 = 0; r0 < rows; r0 += 8) {
        const int n = std::min(8, rows - r0);
        float* pr = proj + (size_t)r0 * 6 * H;
        for (int e = 0; e < 2; ++e) {
            const DevTimestep& te = m.te[e];
            float* temb = (e == 0 ? temb_t : temb_r) + (size_t)r0 * H;
            // timestep_forward (:1286-1308): h = silu(W1 f + b1); temb = W2 h + b2; proj = Wp silu(temb) + bp,
            // proj of t - r added to that of t (:1420-1424); each silu is applied to the rows the next linear quantizes
            launch_timestep_freq(t + r0, e == 0 ? nullptr : r + r0, n, 256, 1000.0f, log_max, freq, s);
            GemmEpilogue e1;
            e1.kind = EPI_STORE_F32;
            e1.bias = te.b1;
            e1.c_f32 = th;
            e1.ldc = H;
            qlinear(freq, 256, n, te.q1.view(), H, 256, e1, "timestep_l1", s);
            GemmEpilogue e2;
            e2.kind = EPI_STORE_F32;
            e2.bias = te.b2;
            e2.c_f32 = temb;
            e2.ldc = H;
            qlinear(th, H, n, te.q2.view(), H, H, e2, "timestep_l2", s, true);
            GemmEpilogue e3;
            e3.kind = e == 0 ? EPI_STORE_F32 : EPI_RESID;
            e3.bias = te.bp;
            e3.c_f32 = pr;
            e3.ldc = 6 * H;
            qlinear(temb, H, n, te.qp.view(), 6 * H, H, e3, "timestep_proj", s, true);
        }
    }
}

void DitEngine::forward_qact(const ForwardIO& io, hipStream_t s) {
    const DitModel& m = model_;
    const DitConfig& c = m.cfg;
    const ActType at = m.act;
    const int B = io.B, T = io.T, L = io.L > 0 ? io.L : 0;
    const int P = c.patch, H = c.hidden, I = c.intermediate, D = c.head_dim;
    const int Np = (T + P - 1) / P;
    const int64_t M = (int64_t)B * Np;
    const int Npad = (int)round_up(Np, 128);
    const int Lpad = (int)round_up(std::max(L, 1), 64);
    const int qd = c.hq * D, kd = c.hkv * D;
    const int64_t q_plane = (int64_t)B * c.hq * Npad * D;
    const int64_t k_plane = (int64_t)B * c.hkv * Npad * D;
    const int64_t kc_plane = (int64_t)c.layers * B * c.hkv * Lpad * D;
    ACEMI_CHECK(B >= 1 && B <= 8, "batch must be 1..8 per GPU");
    ACEMI_CHECK(T >= 1, "seq_len must be > 0");
    ACEMI_CHECK(L == 0 || io.enc != nullptr, "encoder_hidden_states required when enc_len > 0");
    ACEMI_CHECK(m.proj_in_w.k_mult() == 1 && m.proj_out_w.k_mult() == 1,
                "quantized-activation mode: F32 proj_in / proj_out (GGUF) are not supported");
    prepare_shape(B, Np, L);
    rope_for(Np, s);
    if (stage_ev_set_) ACEMI_HIP(hipStreamWaitEvent(s, stage_ev_, 0));
    cross_key_.valid = false;  // the cross K/V planes below are this mode's (f32 precision), not the cached ones

    int n_layers = c.layers;
    if (io.max_layers > 0) n_layers = std::min(n_layers, io.max_layers);
    const int kin = P * c.in_channels;
    ensure(qf_, (size_t)M * std::max({H, qd, I, kin}) * 4);
    float* xf = get<float>(qf_);
    float* x = get<float>(x_);

    // ---- input pack + proj_in (:1343-1382)
    tic(s);
    launch_pack_input_f32(io.hidden, io.context, B, T, Np, P, c.audio_dim, c.ctx_dim(), xf, s);
    toc("pack_input", s);
    {
        GemmEpilogue e;
        e.kind = EPI_STORE_F32;
        e.bias = m.proj_in_b;
        e.c_f32 = x;
        e.ldc = H;
        qlinear(xf, kin, (int)M, m.proj_in_w.view(), H, kin, e, "gemm_proj_in", s);
    }

    // ---- timestep embeddings (:1416-1424), or the sampler's precomputed rows
    const float* proj = io.ts_proj;
    const float* temb_t = io.ts_temb_t;
    const float* temb_r = io.ts_temb_r;
    if (!proj) {
        timestep_embed_qact(io.t, io.r, B, get<float>(proj_), get<float>(temb_t_), get<float>(temb_r_), s);
        proj = get<float>(proj_);
        temb_t = get<float>(temb_t_);
        temb_r = get<float>(temb_r_);
    }
    launch_layer_mods(m.tables, proj, n_layers, B, H, get<float>(mods_), s);
    launch_out_mods(m.out_table, temb_t, temb_r, B, H, get<float>(outmod_), s);

    launch_key_bias(io.mask, B, T, P, Np, Npad, get<float>(kbias_), s);
    if (L > 0) launch_key_bias(io.enc_mask, B, L, 1, L, Lpad, get<float>(kbias_c_), s);

    // ---- condition embedder (:1384-1414) in f32, then every layer's cross K/V
    if (L > 0) {
        const int64_t Me = (int64_t)B * L;
        ensure(encf_, (size_t)Me * H * 4);
        GemmEpilogue e;
        e.kind = EPI_STORE_F32;
        e.bias = m.cond_b;
        e.c_f32 = get<float>(encf_);
        e.ldc = H;
        qlinear(io.enc, H, (int)Me, m.cond_w.view(), H, H, e, "gemm_condition", s);
        const bool fused = m.w_ckv_all.q != nullptr;
        const int ld_ckv = fused ? n_layers * 2 * kd : 2 * kd;
        for (int li = 0; li < n_layers; ++li) {
            if (li == 0 || !fused) {
                GemmEpilogue ek;
                ek.kind = EPI_STORE_F32;
                ek.c_f32 = get<float>(ckv_);
                ek.ldc = ld_ckv;
                const WeightView wv = fused ? m.w_ckv_all.view() : m.layers[li].w_ckv.view();
                qlinear(get<float>(encf_), H, (int)Me, wv, ld_ckv, H, ek, "gemm_cross_kv", s);
            }
            PrepArgs pa{};
            pa.src = get<float>(ckv_) + (fused ? (size_t)li * 2 * kd : 0);
            pa.ld = ld_ckv;
            pa.q_col = -1;
            pa.k_col = 0;
            pa.v_col = kd;
            pa.hq = c.hq;
            pa.hkv = c.hkv;
            pa.n_tok = L;
            pa.n_pad = Lpad;
            pa.B = B;
            pa.k_norm = m.layers[li].ck_norm;
            pa.eps = c.eps;
            pa.kh = get<uint16_t>(kc_) + (size_t)li * B * c.hkv * Lpad * D;
            pa.vt = get<uint16_t>(vc_) + (size_t)li * B * c.hkv * D * Lpad;
            pa.k_plane = kc_plane;
            pa.v_plane = kc_plane;
            tic(s);
            launch_attn_prep(pa, s);
            toc("attn_prep", s);
        }
    }

    const float* mods = get<float>(mods_);
    const int64_t mstride = 6LL * H;
    const float scale = 1.0f / std::sqrt((float)D);
    auto attention = [&](const uint16_t* q, const uint16_t* k, const uint16_t* vt, const float* kbias, int nk, int nk_pad,
                         int window, int64_t kvp, const char* name) {
        AttnArgs aa{};
        aa.q = q;
        aa.k = k;
        aa.vt = vt;
        aa.kbias = kbias;
        aa.part = get<float>(attn_part_);
        aa.out = get<uint16_t>(attn_);
        aa.out_f32 = xf;
        aa.B = B;
        aa.Hq = c.hq;
        aa.Hkv = c.hkv;
        aa.nq = Np;
        aa.nq_pad = Npad;
        aa.nk = nk;
        aa.nk_pad = nk_pad;
        aa.window = window;
        aa.scale = scale;
        aa.split = true;
        aa.pv_split = true;
        aa.f8 = false;
        aa.q_plane = q_plane;
        aa.k_plane = kvp;
        aa.v_plane = kvp;
        tic(s);
        launch_attention(at, aa, s);
        toc(name, s);
    };

    for (int li = 0; li < n_layers; ++li) {  // :1466-1535
        const DevLayer& ly = m.layers[li];
        const float* lm = mods + (size_t)li * B * 6 * H;
        const float* shift_msa = lm + 0 * H;
        const float* scale_msa = lm + 1 * H;
        const float* gate_msa = lm + 2 * H;
        const float* c_shift = lm + 3 * H;
        const float* c_scale = lm + 4 * H;
        const float* c_gate = lm + 5 * H;

        // self-attention block
        tic(s);
        launch_rmsnorm_mod_f32(x, (int)M, H, ly.self_norm, scale_msa, shift_msa, mstride, Np, c.eps, xf, s);
        toc("rmsnorm_mod", s);
        {
            GemmEpilogue e;
            e.kind = EPI_QKV_PREP;
            PrepArgs& pa = e.prep;
            pa.q_col = 0;
            pa.k_col = qd;
            pa.v_col = qd + kd;
            pa.hq = c.hq;
            pa.hkv = c.hkv;
            pa.n_tok = Np;
            pa.n_pad = Npad;
            pa.B = B;
            pa.q_norm = ly.sq_norm;
            pa.k_norm = ly.sk_norm;
            pa.rope_cos = get<float>(cos_);
            pa.rope_sin = get<float>(sin_);
            pa.eps = c.eps;
            pa.qh = get<uint16_t>(qh_);
            pa.kh = get<uint16_t>(kh_);
            pa.vt = get<uint16_t>(vt_);
            pa.q_plane = q_plane;
            pa.k_plane = k_plane;
            pa.v_plane = k_plane;
            qlinear(xf, H, (int)M, ly.w_qkv.view(), qd + 2 * kd, H, e, "gemm_qkv", s);
        }
        const int window = ly.sliding ? std::max(c.sliding_window, 0) : 0;
        attention(get<uint16_t>(qh_), get<uint16_t>(kh_), get<uint16_t>(vt_), io.mask ? get<float>(kbias_) : nullptr, Np,
                  Npad, window, k_plane, ly.sliding ? "attn_self_sliding" : "attn_self_full");
        {
            GemmEpilogue e;
            e.kind = EPI_RESID_GATED;
            e.c_f32 = x;
            e.ldc = H;
            e.gate = gate_msa;
            e.gate_stride = mstride;
            e.rows_per_item = Np;
            qlinear(xf, qd, (int)M, ly.w_o.view(), H, qd, e, "gemm_o", s);
        }

        // cross-attention block (:1502-1520)
        if (ly.cross && L > 0) {
            tic(s);
            launch_rmsnorm_mod_f32(x, (int)M, H, ly.cross_norm, nullptr, nullptr, 0, Np, c.eps, xf, s);
            toc("rmsnorm_mod", s);
            {
                GemmEpilogue e;
                e.kind = EPI_QKV_PREP;
                PrepArgs& pa = e.prep;
                pa.q_col = 0;
                pa.k_col = -1;
                pa.v_col = -1;
                pa.hq = c.hq;
                pa.hkv = c.hkv;
                pa.n_tok = Np;
                pa.n_pad = Npad;
                pa.B = B;
                pa.q_norm = ly.cq_norm;
                pa.eps = c.eps;
                pa.qh = get<uint16_t>(qh_);
                pa.q_plane = q_plane;
                qlinear(xf, H, (int)M, ly.w_cq.view(), qd, H, e, "gemm_cross_q", s);
            }
            attention(get<uint16_t>(qh_), get<uint16_t>(kc_) + (size_t)li * B * c.hkv * Lpad * D,
                      get<uint16_t>(vc_) + (size_t)li * B * c.hkv * D * Lpad, io.enc_mask ? get<float>(kbias_c_) : nullptr,
                      L, Lpad, 0, kc_plane, "attn_cross");
            {
                GemmEpilogue e;
                e.kind = EPI_RESID;
                e.c_f32 = x;
                e.ldc = H;
                qlinear(xf, qd, (int)M, ly.w_co.view(), H, qd, e, "gemm_cross_o", s);
            }
        }

        // MLP block (:1522-1534)
        tic(s);
        launch_rmsnorm_mod_f32(x, (int)M, H, ly.mlp_norm, c_scale, c_shift, mstride, Np, c.eps, xf, s);
        toc("rmsnorm_mod", s);
        {
            GemmEpilogue e;
            e.kind = EPI_SWIGLU_F32;
            e.c_f32 = xf;  // its input rows are quantized already
            e.ldc = I;
            qlinear(xf, H, (int)M, ly.w_gu.view(), 2 * I, H, e, "gemm_gate_up", s);
        }
        {
            GemmEpilogue e;
            e.kind = EPI_RESID_GATED;
            e.c_f32 = x;
            e.ldc = H;
            e.gate = c_gate;
            e.gate_stride = mstride;
            e.rows_per_item = Np;
            qlinear(xf, I, (int)M, ly.w_down.view(), H, I, e, "gemm_down", s);
        }
    }

    // ---- output head (:1537-1559)
    {
        const float* om = get<float>(outmod_);
        tic(s);
        launch_rmsnorm_mod_f32(x, (int)M, H, m.norm_out, om + H, om, 2LL * H, Np, c.eps, xf, s);
        toc("rmsnorm_mod", s);
        GemmEpilogue e;
        e.kind = EPI_PROJ_OUT;
        e.bias = m.proj_out_b;
        e.c_f32 = io.out;
        e.rows_per_item = Np;
        e.out_T = T;
        e.out_ch = c.audio_dim;
        e.patch = P;
        qlinear(xf, H, (int)M, m.proj_out_w.view(), P * c.audio_dim, H, e, "gemm_proj_out", s);
    }
    if (pf_stream_) {
        ACEMI_HIP(hipEventRecord(pf_done_, pf_stream_));
        ACEMI_HIP(hipStreamWaitEvent(s, pf_done_, 0));
    }
}

}  // namespace acemi
