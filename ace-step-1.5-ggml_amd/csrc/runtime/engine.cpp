// DiT forward orchestration: the ggml graph of ace_dit::forward_dit
// (acestep_dit_model.cpp:1316-1560) as a fixed sequence of fused gfx950 kernels.
#include "engine.h"

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>

namespace acemi {

DitEngine::DitEngine(int device) : device_(device) {
    // DiT: the f32-class f8c mode by default (hi/lo operands for Q.K and P.V, the correction products as block-scaled
    // e4m3 MFMAs): ggml runs both products in F32 (acestep_dit_model.cpp:1238-1251) and f8c is the fastest mode that
    // meets the literal 1e-3 one-layer bound at full width (DESIGN.md "Parity"); the condition / text encoders keep
    // the hi/lo fp16 `f32` default
    const AttnPrecision prec = attn_precision_from_env(AttnPrecision::F8C);
    set_attn_precision(prec);
    const char* u = std::getenv("ACE_MI_UNFUSED_PREP");
    fused_prep_ = !(u && u[0] && u[0] != '0');
    const char* q = std::getenv("ACE_MI_QUANT_STAGED");
    staged_quant_ = !(q && q[0] == '0');
    const char* h = std::getenv("ACE_MI_QUANT_STAGE_SCOPE");
    stage_per_call_ = !(h && std::strcmp(h, "layer") == 0);
    stage_model_ = !(h && (std::strcmp(h, "call") == 0 || std::strcmp(h, "layer") == 0));  // default: model
    if (const char* pf = std::getenv("ACE_MI_WEIGHT_PREFETCH")) prefetch_blocks_ = std::max(0, std::atoi(pf));
    qact_ = quant_act_from_env();
    // TEST ONLY (self-test library builds): ACE_MI_TEST_FAULT, runtime/test_hooks.cpp
    if (!test_fault_from_env(fault_.layer, fault_.row, fault_.col, fault_.amp)) fault_.layer = -1;
}

DitEngine::~DitEngine() {
    for (Buf* b : {&a0_, &x_, &act_, &attn_, &act2_, &qkv_, &qh_, &kh_, &vt_, &kbias_, &enc_act_, &encp_, &ckv_, &kc_,
                   &vc_, &kbias_c_, &attn_part_, &freq_, &freq_act_, &th_, &th_act_, &temb_t_, &temb_r_, &temb_act_, &proj_,
                   &mods_, &outmod_, &cos_, &sin_, &ein_, &knorm_tab_, &ts_proj_, &ts_temb_t_, &ts_temb_r_, &qf_, &qa_,
                   &qs_, &qb_, &encf_}) {
        if (b->p) (void)hipFree(b->p);
    }
    if (pf_stream_) {
        (void)hipStreamSynchronize(pf_stream_);
        (void)hipStreamDestroy(pf_stream_);
    }
    if (pf_ev_) (void)hipEventDestroy(pf_ev_);
    if (pf_done_) (void)hipEventDestroy(pf_done_);
    if (pf_sink_.p) (void)hipFree(pf_sink_.p);
    if (stage_ev_) (void)hipEventDestroy(stage_ev_);
    if (ev0_) (void)hipEventDestroy(ev0_);
    if (ev1_) (void)hipEventDestroy(ev1_);
    if (wring_.p) (void)hipFree(wring_.p);
    for (auto& kv : img_)
        if (kv.second.p) (void)hipFree(kv.second.p);
    for (auto& kv : q8img_)
        if (kv.second.p) (void)hipFree(kv.second.p);
    if (qa16_.p) (void)hipFree(qa16_.p);
}

namespace {
size_t wbytes(const DevWeight& w) { return (size_t)w.rows * w.cols * 2; }
}  // namespace

// The six block matrices of layer li: views of the bf16 staging slot (staged) or of the resident weights.
DitEngine::LayerViews DitEngine::layer_views(int li, bool staged) {
    const DevLayer& ly = model_.layers[li];
    const DevWeight* ws[6] = {&ly.w_qkv, &ly.w_o, &ly.w_cq, &ly.w_co, &ly.w_gu, &ly.w_down};
    WeightView v[6];
    char* base = staged ? stage_slot(li) : nullptr;
    size_t off = 0;
    for (int i = 0; i < 6; ++i) {
        v[i] = ws[i]->view();
        if (staged && weight_quantized(ws[i]->fmt)) {
            v[i].fmt = WF_BF16;
            v[i].q = base + off;
            v[i].s = nullptr;
            v[i].ld = ws[i]->cols;
        }
        off += wbytes(*ws[i]);
    }
    return LayerViews{v[0], v[1], v[2], v[3], v[4], v[5]};
}

void DitEngine::stage_layer(int li, hipStream_t st) {
    const DevLayer& ly = model_.layers[li];
    const DevWeight* ws[6] = {&ly.w_qkv, &ly.w_o, &ly.w_cq, &ly.w_co, &ly.w_gu, &ly.w_down};
    char* base = stage_slot(li);
    size_t off = 0;
    DequantJob jobs[6];
    int n = 0;
    for (int i = 0; i < 6; ++i) {
        if (weight_quantized(ws[i]->fmt) && ws[i]->q) {
            if (n > 0 && ws[i]->fmt != jobs[0].w.fmt) {  // one launch per weight format
                launch_dequant_bf16_batch(jobs, n, st);
                n = 0;
            }
            jobs[n++] = DequantJob{ws[i]->view(), ws[i]->rows, ws[i]->cols, reinterpret_cast<uint16_t*>(base + off)};
        }
        off += wbytes(*ws[i]);
    }
    tic(st);
    if (n > 0) launch_dequant_bf16_batch(jobs, n, st);
    toc("dequant_stage", st);
    images_written_ = true;
}

WeightView DitEngine::dense_view(const DevWeight& w, hipStream_t s) {
    WeightView v = w.view();
    if (!staged_quant_ || !stage_per_call_ || !weight_quantized(v.fmt) || !v.q) return v;
    Buf& b = img_[v.q];
    if (!b.p) {
        ensure(b, (size_t)w.rows * w.cols * 2);
        launch_dequant_bf16(v, w.rows, w.cols, static_cast<uint16_t*>(b.p), s);
        images_written_ = true;
    }
    v.fmt = WF_BF16;
    v.q = b.p;
    v.s = nullptr;
    v.ld = w.cols;
    return v;
}

// Side-stream sweep of layer li's block weights (ACE_MI_WEIGHT_PREFETCH), ordered after the work already queued
// on s; the forward joins the side stream before it returns.
void DitEngine::prefetch_layer(int li, bool staged, hipStream_t s) {
    if (!pf_stream_) {
        ACEMI_HIP(hipStreamCreateWithFlags(&pf_stream_, hipStreamNonBlocking));
        ACEMI_HIP(hipEventCreateWithFlags(&pf_ev_, hipEventDisableTiming));
        ACEMI_HIP(hipEventCreateWithFlags(&pf_done_, hipEventDisableTiming));
    }
    ensure(pf_sink_, 256);
    const LayerViews lw = layer_views(li, staged);
    const DevLayer& ly = model_.layers[li];
    const DevWeight* ws[6] = {&ly.w_qkv, &ly.w_o, &ly.w_cq, &ly.w_co, &ly.w_gu, &ly.w_down};
    const WeightView* vs[6] = {&lw.qkv, &lw.o, &lw.cq, &lw.co, &lw.gu, &lw.down};
    const void* ptrs[6];
    size_t bytes[6];
    int n = 0;
    for (int i = 0; i < 6; ++i) {
        if (weight_quantized(vs[i]->fmt) || !vs[i]->q) continue;  // bf16 / fp16 images only
        ptrs[n] = vs[i]->q;
        bytes[n] = (size_t)ws[i]->rows * ws[i]->cols * 2;
        ++n;
    }
    if (n == 0) return;
    ACEMI_HIP(hipEventRecord(pf_ev_, s));
    ACEMI_HIP(hipStreamWaitEvent(pf_stream_, pf_ev_, 0));
    launch_prefetch(ptrs, bytes, n, prefetch_blocks_, get<unsigned>(pf_sink_), pf_stream_);
}

// Layer li's bf16 image: its own slot when the images of the whole model are kept for the sampling call,
// else the single slot every layer shares.
char* DitEngine::stage_slot(int li) {
    return static_cast<char*>(wring_.p) + (stage_per_call_ ? (size_t)li * stage_slot_bytes_ : 0);
}

// Device table of every layer's cross-attention k-norm weights (PrepArgs::k_norm_layers), built once.
const float* const* DitEngine::cross_norm_table() {
    const size_t n = model_.layers.size();
    if (!knorm_tab_.p || knorm_tab_n_ != n) {
        std::vector<const float*> h(n);
        for (size_t i = 0; i < n; ++i) h[i] = model_.layers[i].ck_norm;
        ensure(knorm_tab_, n * sizeof(const float*));
        ACEMI_HIP(hipMemcpy(knorm_tab_.p, h.data(), n * sizeof(const float*), hipMemcpyHostToDevice));
        knorm_tab_n_ = n;
    }
    return static_cast<const float* const*>(knorm_tab_.p);
}

void DitEngine::ensure(Buf& b, size_t bytes) {
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

void DitEngine::set_profiling(bool on) {
    profiling_ = on;
    if (on && !ev0_) {
        ACEMI_HIP(hipEventCreate(&ev0_));
        ACEMI_HIP(hipEventCreate(&ev1_));
    }
}

void DitEngine::reset_times() { times_ = KernelTimes{}; }

void DitEngine::tic(hipStream_t s) {
    if (profiling_) ACEMI_HIP(hipEventRecord(ev0_, s));
}

void DitEngine::toc(const char* name, hipStream_t s) {
    if (!profiling_) return;
    ACEMI_HIP(hipEventRecord(ev1_, s));
    ACEMI_HIP(hipEventSynchronize(ev1_));
    float ms = 0.f;
    ACEMI_HIP(hipEventElapsedTime(&ms, ev0_, ev1_));
    for (size_t i = 0; i < times_.names.size(); ++i) {
        if (times_.names[i] == name) {
            times_.ms[i] += ms;
            times_.count[i] += 1;
            return;
        }
    }
    times_.names.emplace_back(name);
    times_.ms.push_back(ms);
    times_.count.push_back(1);
}

void DitEngine::prepare_shape(int B, int Np, int L) {
    const DitConfig& c = model_.cfg;
    const int H = c.hidden, I = c.intermediate, D = c.head_dim;
    const int64_t M = (int64_t)B * Np;
    const int64_t Npad = round_up(Np, 128);
    const int qd = c.hq * D, kd = c.hkv * D;
    const size_t act = 2;
    ensure(a0_, M * c.patch * c.in_channels * act * 3);                 // x3 layout for F32 proj_in
    ensure(act2_, M * std::max(I, 3 * H) * act);                        // also the x3 proj_out input
    ensure(x_, M * H * 4);
    ensure(act_, M * std::max(H, qd) * act);
    ensure(attn_, M * qd * act);
    ensure(qkv_, M * (qd + 2 * kd) * 4);
    ensure(qh_, (size_t)2 * B * c.hq * Npad * D * 2);   // hi + lo planes
    ensure(kh_, (size_t)2 * B * c.hkv * Npad * D * 2);
    ensure(vt_, (size_t)2 * B * c.hkv * D * Npad * 2);
    ensure(kbias_, (size_t)B * Npad * 4);
    ensure(attn_part_, attn_part_floats(B, (int)Np, c.hq) * 4);
    if (L > 0) {
        const int64_t Lpad = round_up(L, 64);
        const int64_t Me = (int64_t)B * L;
        ensure(enc_act_, Me * H * act);
        ensure(encp_, Me * H * act);
        ensure(ckv_, Me * c.layers * 2 * kd * 4);  // all layers' cross k|v (one GEMM)
        const void* kc_old = kc_.p;
        const void* vc_old = vc_.p;
        ensure(kc_, (size_t)2 * c.layers * B * c.hkv * Lpad * D * 2);
        ensure(vc_, (size_t)2 * c.layers * B * c.hkv * D * Lpad * 2);
        if (kc_.p != kc_old || vc_.p != vc_old) cross_key_.valid = false;
        ensure(kbias_c_, (size_t)B * Lpad * 4);
    }
    ensure(freq_, (size_t)B * 256 * 4);
    ensure(freq_act_, (size_t)B * 256 * act);
    ensure(th_, (size_t)B * H * 4);
    ensure(th_act_, (size_t)B * H * act);
    ensure(temb_t_, (size_t)B * H * 4);
    ensure(temb_r_, (size_t)B * H * 4);
    ensure(temb_act_, (size_t)B * H * act);
    ensure(proj_, (size_t)B * 6 * H * 4);
    ensure(mods_, (size_t)c.layers * B * 6 * H * 4);
    ensure(outmod_, (size_t)B * 2 * H * 4);
}

// NEOX RoPE table with the reference's own float arithmetic: ggml_rope_cache_init runs
// theta = p; theta *= theta_scale per pair, theta_scale = powf(base, -2/n_dims), cos/sinf on the CPU
// (acestep_dit_model.cpp:1205-1210).  Computed once per sequence length on the host.
void DitEngine::rope_table(int n, Buf& cb, Buf& sb, hipStream_t s) {
    const DitConfig& c = model_.cfg;
    const int half = c.head_dim / 2;
    const float theta_scale = powf(c.rope_theta, -2.0f / (float)c.head_dim);
    std::vector<float> cs((size_t)n * half), sn((size_t)n * half);
    for (int p = 0; p < n; ++p) {
        float theta = (float)p;
        for (int i = 0; i < half; ++i) {
            cs[(size_t)p * half + i] = (float)std::cos((double)theta);  // correctly rounded cosf / sinf
            sn[(size_t)p * half + i] = (float)std::sin((double)theta);
            theta *= theta_scale;
        }
    }
    // a forward still queued on `s` (a non-blocking stream) may read the old table: drain it first
    ACEMI_HIP(hipStreamSynchronize(s));
    ensure(cb, cs.size() * 4);
    ensure(sb, sn.size() * 4);
    ACEMI_HIP(hipMemcpy(cb.p, cs.data(), cs.size() * 4, hipMemcpyHostToDevice));
    ACEMI_HIP(hipMemcpy(sb.p, sn.data(), sn.size() * 4, hipMemcpyHostToDevice));
    ACEMI_HIP(hipDeviceSynchronize());  // null-stream copy: done before any stream reads it
}

void DitEngine::rope_for(int Np, hipStream_t s) {
    if (rope_np_ == Np) return;
    rope_table(Np, cos_, sin_, s);
    rope_np_ = Np;
}

void DitEngine::forward(const ForwardIO& io, hipStream_t s) {
    if (qact_) {
        forward_qact(io, s);
        return;
    }
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
    const bool split = attn_split_;
    const int64_t q_plane = (int64_t)B * c.hq * Npad * D;        // lo plane offsets (elements)
    const int64_t k_plane = (int64_t)B * c.hkv * Npad * D;
    const int64_t kc_plane = (int64_t)c.layers * B * c.hkv * Lpad * D;
    ACEMI_CHECK(B >= 1 && B <= 8, "batch must be 1..8 per GPU");
    ACEMI_CHECK(T >= 1, "seq_len must be > 0");
    ACEMI_CHECK(L == 0 || io.enc != nullptr, "encoder_hidden_states required when enc_len > 0");
    prepare_shape(B, Np, L);
    rope_for(Np, s);
    // bf16 images written by an earlier forward (possibly on another stream) are complete before this one reads them
    if (stage_ev_set_) ACEMI_HIP(hipStreamWaitEvent(s, stage_ev_, 0));
    images_written_ = false;

    int n_layers = c.layers;
    if (io.max_layers > 0) n_layers = std::min(n_layers, io.max_layers);

    uint16_t* a0 = get<uint16_t>(a0_);
    float* x = get<float>(x_);
    uint16_t* act = get<uint16_t>(act_);
    uint16_t* attn = get<uint16_t>(attn_);
    uint16_t* act2 = get<uint16_t>(act2_);
    float* qkv = get<float>(qkv_);

    // ---- input pack + proj_in (:1343-1382)
    tic(s);
    const int kin = m.proj_in_w.k_mult();
    launch_pack_input(m.proj_in_w.act(), io.hidden, io.context, B, T, Np, P, c.audio_dim, c.ctx_dim(), a0, s,
                      kin == 3);
    toc("pack_input", s);
    {
        GemmEpilogue e;
        e.kind = EPI_STORE_F32;
        e.bias = m.proj_in_b;
        e.c_f32 = x;
        e.ldc = H;
        tic(s);
        launch_gemm(a0, kin * P * c.in_channels, dense_view(m.proj_in_w, s), (int)M, H, kin * P * c.in_channels, e, s);
        toc("gemm_proj_in", s);
    }

    // ---- timestep embeddings (:1416-1424, timestep_forward :1286-1308), or the sampler's precomputed rows
    {
        tic(s);
        const float* proj = io.ts_proj;
        const float* temb_t = io.ts_temb_t;
        const float* temb_r = io.ts_temb_r;
        if (!proj) {
            timestep_embed(io.t, io.r, B, get<float>(proj_), get<float>(temb_t_), get<float>(temb_r_), s);
            proj = get<float>(proj_);
            temb_t = get<float>(temb_t_);
            temb_r = get<float>(temb_r_);
        }
        launch_layer_mods(m.tables, proj, n_layers, B, H, get<float>(mods_), s);
        launch_out_mods(m.out_table, temb_t, temb_r, B, H, get<float>(outmod_), s);
        toc("timestep", s);
    }

    // ---- key masks
    tic(s);
    launch_key_bias(io.mask, B, T, P, Np, Npad, get<float>(kbias_), s);
    if (L > 0) launch_key_bias(io.enc_mask, B, L, 1, L, Lpad, get<float>(kbias_c_), s);
    toc("key_bias", s);

    // ---- condition embedder (:1384-1414) + per-layer cross K/V (constant over the layer loop)
    const bool reuse = io.reuse_cross && cross_key_.valid && cross_key_.B == B && cross_key_.L == L &&
                       cross_key_.layers >= n_layers && cross_key_.enc == io.enc;
    if (L > 0 && !reuse) {
        cross_key_ = CrossKey{true, B, L, n_layers, io.enc};
        const int64_t Me = (int64_t)B * L;
        uint16_t* enc_act = get<uint16_t>(enc_act_);
        uint16_t* encp = get<uint16_t>(encp_);
        tic(s);
        launch_to_act(at, io.enc, Me * H, false, enc_act, s);
        GemmEpilogue e;
        e.kind = EPI_STORE_ACT;
        e.bias = m.cond_b;
        e.c_act = encp;
        e.ldc = H;
        launch_gemm(enc_act, H, dense_view(m.cond_w, s), (int)Me, H, H, e, s);
        toc("gemm_condition", s);
        // one GEMM for every layer's cross k|v when the weights are fused: ckv [Me][n_layers*2kd]
        const bool fused = m.w_ckv_all.q != nullptr;
        const int ld_ckv = fused ? n_layers * 2 * kd : 2 * kd;
        if (fused) {
            GemmEpilogue ek;
            ek.kind = EPI_STORE_F32;
            ek.c_f32 = get<float>(ckv_);
            ek.ldc = ld_ckv;
            tic(s);
            launch_gemm(encp, H, dense_view(m.w_ckv_all, s), (int)Me, ld_ckv, H, ek, s);  // first n_layers layers
            toc("gemm_cross_kv", s);
        }
        for (int li = 0; li < n_layers; ++li) {
            const DevLayer& ly = m.layers[li];
            if (!fused) {
                GemmEpilogue ek;
                ek.kind = EPI_STORE_F32;
                ek.c_f32 = get<float>(ckv_);
                ek.ldc = 2 * kd;
                tic(s);
                launch_gemm(encp, H, dense_view(ly.w_ckv, s), (int)Me, 2 * kd, H, ek, s);
                toc("gemm_cross_kv", s);
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
            pa.k_norm = ly.ck_norm;
            pa.eps = c.eps;
            pa.kh = get<uint16_t>(kc_) + (size_t)li * B * c.hkv * Lpad * D;
            pa.vt = get<uint16_t>(vc_) + (size_t)li * B * c.hkv * D * Lpad;
            pa.k_plane = split ? kc_plane : 0;
            pa.v_plane = attn_pv_split_ ? kc_plane : 0;
            pa.f8 = attn_f8_ ? 1 : 0;
            if (fused) {  // every layer's cross K/V re-layout in one launch (PrepArgs::layers)
                pa.layers = n_layers;
                pa.src_layer = 2 * kd;
                pa.kh_layer = (int64_t)B * c.hkv * Lpad * D;
                pa.vt_layer = (int64_t)B * c.hkv * D * Lpad;
                pa.k_norm_layers = cross_norm_table();
            }
            tic(s);
            launch_attn_prep(pa, s);
            toc("attn_prep", s);
            if (fused) break;
        }
    }

    const float* mods = get<float>(mods_);
    const int64_t mstride = 6LL * H;  // per item within a layer
    const float scale = 1.0f / std::sqrt((float)D);

    // staged dequant: each layer's quantized block matrices are expanded to their bf16 image right before the
    // layer, in stream order, into one workspace slot (see engine.h)
    const bool staged = staged_quant_ && n_layers > 0 && weight_quantized(m.layers[0].w_gu.fmt);
    bool restage = true;
    if (staged) {
        const DevLayer& l0 = m.layers[0];
        stage_slot_bytes_ = wbytes(l0.w_qkv) + wbytes(l0.w_o) + wbytes(l0.w_cq) + wbytes(l0.w_co) +
                            wbytes(l0.w_gu) + wbytes(l0.w_down);
        ensure(wring_, stage_slot_bytes_ * (stage_per_call_ ? n_layers : 1));
        // per-call scope: the images written by the first forward of a sampling call serve its later steps
        // (the weights are loop-invariant); any other forward expands them again
        // "model" scope: the images stay valid across calls (the weights never change after load), so the
        // reference's per-step decoder.forward hook does not re-expand them either
        restage = !(stage_per_call_ && (io.reuse_stage || stage_model_) && stage_layers_ >= n_layers);
        stage_layers_ = stage_per_call_ ? n_layers : 0;
    }

    for (int li = 0; li < n_layers; ++li) {  // :1466-1535
        const DevLayer& ly = m.layers[li];
        if (staged && restage) stage_layer(li, s);
        if (prefetch_blocks_ > 0 && li + 1 < n_layers && !(staged && restage)) prefetch_layer(li + 1, staged, s);
        const LayerViews lw = layer_views(li, staged);
        const float* lm = mods + (size_t)li * B * 6 * H;
        const float* shift_msa = lm + 0 * H;
        const float* scale_msa = lm + 1 * H;
        const float* gate_msa = lm + 2 * H;
        const float* c_shift = lm + 3 * H;
        const float* c_scale = lm + 4 * H;
        const float* c_gate = lm + 5 * H;

        // self-attention block
        tic(s);
        launch_rmsnorm_mod(at, x, (int)M, H, ly.self_norm, scale_msa, shift_msa, mstride, Np, c.eps, act, s);
        toc("rmsnorm_mod", s);
        {
            // QKV projection with QK-RMSNorm, RoPE and the attention re-layout fused into its epilogue
            // (EPI_QKV_PREP; ACE_MI_UNFUSED_PREP=1 runs the f32 store + attn_prep pair instead)
            PrepArgs pa{};
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
            pa.q_plane = split ? q_plane : 0;
            pa.k_plane = split ? k_plane : 0;
            pa.v_plane = attn_pv_split_ ? k_plane : 0;
            pa.f8 = attn_f8_ ? 1 : 0;
            qkv_gemm(act, lw.qkv, (int)M, qd + 2 * kd, pa, qkv, "gemm_qkv", s);
        }
        {
            AttnArgs aa{};
            aa.q = get<uint16_t>(qh_);
            aa.k = get<uint16_t>(kh_);
            aa.vt = get<uint16_t>(vt_);
            aa.kbias = io.mask ? get<float>(kbias_) : nullptr;  // padding keys are masked in-kernel
            aa.part = get<float>(attn_part_);
            aa.out = attn;
            aa.B = B;
            aa.Hq = c.hq;
            aa.Hkv = c.hkv;
            aa.nq = Np;
            aa.nq_pad = Npad;
            aa.nk = Np;
            aa.nk_pad = Npad;
            aa.window = ly.sliding ? std::max(c.sliding_window, 0) : 0;
            if (ly.sliding && c.sliding_window <= 0) aa.window = 0;
            aa.scale = scale;
            aa.split = split;
            aa.pv_split = attn_pv_split_;
            aa.f8 = attn_f8_;
            aa.q_plane = q_plane;
            aa.k_plane = k_plane;
            aa.v_plane = k_plane;
            tic(s);
            launch_attention(at, aa, s);
            toc(ly.sliding ? "attn_self_sliding" : "attn_self_full", s);
        }
        {
            GemmEpilogue e;
            e.kind = EPI_RESID_GATED;
            e.c_f32 = x;
            e.ldc = H;
            e.gate = gate_msa;
            e.gate_stride = mstride;
            e.rows_per_item = Np;
            tic(s);
            if (li == fault_.layer) {  // (the injected fault must reach the norm that follows)
                launch_gemm(attn, qd, lw.o, (int)M, H, qd, e, s);
                launch_fault_tile(x, H, (int)M, fault_.row, fault_.col, fault_.amp, s);
            } else {
                launch_gemm(attn, qd, lw.o, (int)M, H, qd, e, s);
            }
            toc("gemm_o", s);
        }

        // cross-attention block (:1502-1520): no AdaLN, no gate, no RoPE
        if (ly.cross && L > 0) {
            tic(s);
            launch_rmsnorm_mod(at, x, (int)M, H, ly.cross_norm, nullptr, nullptr, 0, Np, c.eps, act, s);
            toc("rmsnorm_mod", s);
            {
                PrepArgs pa{};
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
                pa.q_plane = split ? q_plane : 0;
                pa.f8 = attn_f8_ ? 1 : 0;
                qkv_gemm(act, lw.cq, (int)M, qd, pa, qkv, "gemm_cross_q", s);
            }
            {
                AttnArgs aa{};
                aa.q = get<uint16_t>(qh_);
                aa.k = get<uint16_t>(kc_) + (size_t)li * B * c.hkv * Lpad * D;
                aa.vt = get<uint16_t>(vc_) + (size_t)li * B * c.hkv * D * Lpad;
                aa.kbias = io.enc_mask ? get<float>(kbias_c_) : nullptr;
                aa.part = get<float>(attn_part_);
                aa.out = attn;
                aa.B = B;
                aa.Hq = c.hq;
                aa.Hkv = c.hkv;
                aa.nq = Np;
                aa.nq_pad = Npad;
                aa.nk = L;
                aa.nk_pad = Lpad;
                aa.window = 0;
                aa.scale = scale;
                aa.split = split;
                aa.pv_split = attn_pv_split_;
            aa.f8 = attn_f8_;
                aa.q_plane = q_plane;
                aa.k_plane = kc_plane;
                aa.v_plane = kc_plane;
                tic(s);
                launch_attention(at, aa, s);
                toc("attn_cross", s);
            }
            {
                GemmEpilogue e;
                e.kind = EPI_RESID;
                e.c_f32 = x;
                e.ldc = H;
                tic(s);
                launch_gemm(attn, qd, lw.co, (int)M, H, qd, e, s);
                toc("gemm_cross_o", s);
            }
        }

        // MLP block (:1522-1534)
        tic(s);
        launch_rmsnorm_mod(at, x, (int)M, H, ly.mlp_norm, c_scale, c_shift, mstride, Np, c.eps, act, s);
        toc("rmsnorm_mod", s);
        {
            GemmEpilogue e;
            e.kind = EPI_SWIGLU;
            e.c_act = act2;
            e.ldc = I;
            tic(s);
            launch_gemm(act, H, lw.gu, (int)M, 2 * I, H, e, s);
            toc("gemm_gate_up", s);
        }
        {
            GemmEpilogue e;
            e.kind = EPI_RESID_GATED;
            e.c_f32 = x;
            e.ldc = H;
            e.gate = c_gate;
            e.gate_stride = mstride;
            e.rows_per_item = Np;
            tic(s);
            launch_gemm(act2, I, lw.down, (int)M, H, I, e, s);
            toc("gemm_down", s);
        }
    }

    // ---- output head (:1537-1559)
    {
        const float* om = get<float>(outmod_);
        const int kout = m.proj_out_w.k_mult();
        uint16_t* head_in = kout == 3 ? get<uint16_t>(act2_) : act;  // act2_ is sized for M x 3H too
        tic(s);
        launch_rmsnorm_mod(m.proj_out_w.act(), x, (int)M, H, m.norm_out, om + H, om, 2LL * H, Np, c.eps, head_in,
                           s, kout == 3);
        toc("rmsnorm_mod", s);
        GemmEpilogue e;
        e.kind = EPI_PROJ_OUT;
        e.bias = m.proj_out_b;
        e.c_f32 = io.out;
        e.rows_per_item = Np;
        e.out_T = T;
        e.out_ch = c.audio_dim;
        e.patch = P;
        tic(s);
        launch_gemm(head_in, kout * H, dense_view(m.proj_out_w, s), (int)M, P * c.audio_dim, kout * H, e, s);
        toc("gemm_proj_out", s);
    }
    if (images_written_) {
        if (!stage_ev_) ACEMI_HIP(hipEventCreateWithFlags(&stage_ev_, hipEventDisableTiming));
        ACEMI_HIP(hipEventRecord(stage_ev_, s));
        stage_ev_set_ = true;
    }
    if (pf_stream_) {  // the side stream's sweeps end before anything ordered after this forward on s
        ACEMI_HIP(hipEventRecord(pf_done_, pf_stream_));
        ACEMI_HIP(hipStreamWaitEvent(s, pf_done_, 0));
    }
}

void DitEngine::timestep_embed(const float* t, const float* r, int rows, float* proj, float* temb_t, float* temb_r,
                               hipStream_t s) {
    if (qact_) {
        timestep_embed_qact(t, r, rows, proj, temb_t, temb_r, s);
        return;
    }
    const DitModel& m = model_;
    const int H = m.cfg.hidden;
    const float log_max = std::log(10000.0f);
    ensure(freq_, (size_t)8 * 256 * 4);
    ensure(th_, (size_t)8 * H * 4);
    float* freq = get<float>(freq_);
    float* th = get<float>(th_);
    // rows are independent: chunks of up to 8 (the GEMV kernel's row limit), the same arithmetic per row
    for (int r0 = 0; r0 < rows; r0 += 8) {
        const int n = std::min(8, rows - r0);
        float* pr = proj + (size_t)r0 * 6 * H;
        for (int e = 0; e < 2; ++e) {
            float* temb = (e == 0 ? temb_t : temb_r) + (size_t)r0 * H;
            launch_timestep_freq(t + r0, e == 0 ? nullptr : r + r0, n, 256, 1000.0f, log_max, freq, s);
            const ActType ta = m.te[e].act;
            // each linear rounds its f32 input to the weight type itself (launch_gemv_f32 = to_act + gemv)
            launch_gemv_f32(ta, freq, false, n, m.te[e].w1, H, 256, m.te[e].b1, true, false, th, s);
            launch_gemv_f32(ta, th, false, n, m.te[e].w2, H, H, m.te[e].b2, false, false, temb, s);
            launch_gemv_f32(ta, temb, true, n, m.te[e].wp, 6 * H, H, m.te[e].bp, false, e == 1, pr, s);
        }
    }
}

DitEngine::TimestepRows DitEngine::precompute_timesteps(const float* t, const float* r, int rows, hipStream_t s) {
    const int H = model_.cfg.hidden;
    ensure(ts_proj_, (size_t)rows * 6 * H * 4);
    ensure(ts_temb_t_, (size_t)rows * H * 4);
    ensure(ts_temb_r_, (size_t)rows * H * 4);
    tic(s);
    timestep_embed(t, r, rows, get<float>(ts_proj_), get<float>(ts_temb_t_), get<float>(ts_temb_r_), s);
    toc("timestep_precompute", s);
    return TimestepRows{get<float>(ts_proj_), get<float>(ts_temb_t_), get<float>(ts_temb_r_)};
}

// A projection feeding attention: with EPI_QKV_PREP the GEMM epilogue writes the attention operands of
// `pa` directly; the unfused path (ACE_MI_UNFUSED_PREP=1, A/B and debugging) stores f32 to `scratch`
// and runs attn_prep over it.
void DitEngine::qkv_gemm(const uint16_t* act, const WeightView& w, int M, int N, PrepArgs pa, float* scratch,
                         const char* name, hipStream_t s) {
    const int H = model_.cfg.hidden;
    GemmEpilogue e;
    if (fused_prep_) {
        e.kind = EPI_QKV_PREP;
        e.prep = pa;
        tic(s);
        launch_gemm(act, H, w, M, N, H, e, s);
        toc(name, s);
        return;
    }
    e.kind = EPI_STORE_F32;
    e.c_f32 = scratch;
    e.ldc = N;
    tic(s);
    launch_gemm(act, H, w, M, N, H, e, s);
    toc(name, s);
    pa.src = scratch;
    pa.ld = N;
    tic(s);
    launch_attn_prep(pa, s);
    toc("attn_prep", s);
}

void DitEngine::encode(const EncodeIO& io, hipStream_t s) {
    const DitModel& m = model_;
    const DitConfig& c = m.cfg;
    const int H = c.hidden;
    const int B = io.B, n = io.n;
    ACEMI_CHECK(io.proj && io.proj->q, "encoder: input projection not loaded");
    ACEMI_CHECK(B >= 1 && n >= 1 && io.in && io.out, "encoder: bad arguments");
    ACEMI_CHECK(io.proj->rows == H && io.proj->k_mult() == 1, "encoder: projection weight shape mismatch");
    const int in_dim = io.proj->cols;
    const int64_t M = (int64_t)B * n;
    ensure(ein_, (size_t)M * in_dim * 2);
    uint16_t* ein = get<uint16_t>(ein_);
    launch_to_act(io.proj->act(), io.in, M * in_dim, false, ein, s);
    GemmEpilogue pe;
    pe.kind = EPI_STORE_F32;
    pe.bias = io.proj_b;
    pe.ldc = H;
    if (!io.enc) {  // projection only (the text projector)
        ACEMI_CHECK(!io.first_only, "encoder: first_only needs an encoder");
        pe.c_f32 = io.out;
        launch_gemm(ein, in_dim, io.proj->view(), (int)M, H, in_dim, pe, s);
        return;
    }
    const DevEncoder& e = *io.enc;
    int n_layers = (int)e.layers.size();
    if (io.max_layers >= 0) n_layers = std::min(n_layers, io.max_layers);
    BlockShape sh;
    sh.hidden = H;
    sh.hq = c.hq;
    sh.hkv = c.hkv;
    sh.head_dim = c.head_dim;
    sh.intermediate = e.intermediate;
    sh.eps = c.eps;
    sh.rope_theta = c.rope_theta;
    sh.sliding_window = c.sliding_window;
    pe.c_f32 = cond_.x(M, H);
    launch_gemm(ein, in_dim, io.proj->view(), (int)M, H, in_dim, pe, s);  // x = in W^T + b
    // all-ones token mask (acestep_ggml.cpp:1692 / :1838), bidirectional
    cond_.run(sh, e.layers, n_layers, e.act, B, n, nullptr, false, s);
    cond_.finish(sh, e.norm, B, n, io.first_only, io.out, s);
}

void DitEngine::probe_gemm(int which, int M, int iters, hipStream_t s) {
    const DitModel& m = model_;
    const DitConfig& c = m.cfg;
    const int H = c.hidden, I = c.intermediate;
    prepare_shape(1, M, 0);
    const DevLayer& ly = m.layers[0];
    for (int it = 0; it < iters; ++it) {
        GemmEpilogue e;
        if (which == 0) {
            e.kind = EPI_SWIGLU;
            e.c_act = get<uint16_t>(act2_);
            e.ldc = I;
            tic(s);
            launch_gemm(get<uint16_t>(act_), H, ly.w_gu.view(), M, 2 * I, H, e, s);
            toc("probe_gemm_gate_up", s);
        } else {
            e.kind = EPI_RESID_GATED;
            e.c_f32 = get<float>(x_);
            e.ldc = H;
            e.gate = get<float>(mods_);
            e.gate_stride = 0;
            e.rows_per_item = M;
            tic(s);
            launch_gemm(get<uint16_t>(act2_), I, ly.w_down.view(), M, H, I, e, s);
            toc("probe_gemm_down", s);
        }
    }
}

}  // namespace acemi
