// Weight ingestion: config.json + model.safetensors -> HBM (see model.h).
#include "model.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <sstream>

#include "json.h"
#include "loader.h"

namespace acemi {

DitModel::~DitModel() {
    for (void* p : allocs) (void)hipFree(p);
}

bool quant_act_from_env() {
    const char* e = std::getenv("ACE_MI_QUANT_ACT");
    if (!e || !e[0] || std::strcmp(e, "bf16") == 0) return false;
    if (std::strcmp(e, "q8") == 0) return true;
    throw std::runtime_error("ACE_MI_QUANT_ACT must be bf16 or q8");
}

void load_config(const std::string& path, DitConfig& c) {
    // acestep_dit_config.cpp:19-93 (required keys + optional ones)
    std::string text;
    try {
        text = read_file(path);
    } catch (const std::exception&) {
        throw IoError("failed to read config");
    }
    Json o;
    try {
        o = Json::parse(text);
    } catch (const std::exception& e) {
        throw IoError(e.what());
    }
    if (o.kind != Json::Object) throw IoError("config is not object");
    try {
        c.hidden = (int)o.at("hidden_size").as_int();
        c.intermediate = (int)o.at("intermediate_size").as_int();
        c.layers = (int)o.at("num_hidden_layers").as_int();
        c.hq = (int)o.at("num_attention_heads").as_int();
        c.hkv = (int)o.at("num_key_value_heads").as_int();
        c.head_dim = (int)o.at("head_dim").as_int();
        c.max_pos = (int)o.at("max_position_embeddings").as_int();
        c.eps = (float)o.at("rms_norm_eps").as_num();
        c.patch = (int)o.at("patch_size").as_int();
        c.in_channels = (int)o.at("in_channels").as_int();
        c.audio_dim = (int)o.at("audio_acoustic_hidden_dim").as_int();
        if (o.has("use_sliding_window")) c.use_sliding_window = o.at("use_sliding_window").as_bool();
        if (o.has("sliding_window") && o.at("sliding_window").kind == Json::Number)
            c.sliding_window = (int)o.at("sliding_window").as_int();
        if (o.has("rope_theta")) c.rope_theta = (float)o.at("rope_theta").as_num();
        auto opt_int = [&](const char* k, int& dst) {
            if (o.has(k) && o.at(k).kind == Json::Number) dst = (int)o.at(k).as_int();
        };
        opt_int("text_hidden_dim", c.text_hidden_dim);
        opt_int("num_lyric_encoder_hidden_layers", c.lyric_layers);
        opt_int("timbre_hidden_dim", c.timbre_hidden_dim);
        opt_int("num_timbre_encoder_hidden_layers", c.timbre_layers);
        opt_int("timbre_fix_frame", c.timbre_fix_frame);
        const auto& lt = o.at("layer_types");
        if (lt.kind != Json::Array) throw IoError("missing layer_types");
        c.layer_types.clear();
        for (const auto& v : lt.arr) c.layer_types.push_back(v.as_str());
    } catch (const IoError&) {
        throw;
    } catch (const std::exception& e) {
        throw IoError(std::string("config: ") + e.what());
    }
}

void load_dit_model(const std::string& dir, DitModel& m, int& status_hint) {
    status_hint = 3;
    try {
        namespace fs = std::filesystem;
        const fs::path p(dir);
        const fs::path root = p.extension() == ".gguf" ? p.parent_path() : p;
        // GGUF resolution order of resolve_gguf_path (acestep_dit_model.cpp:47-70)
        std::string gguf_path;
        for (const char* key : {"ACE_GGML_DIT_GGUF", "ACE_GGML_DIT_GGUF_PATH"}) {
            const char* v = std::getenv(key);
            if (gguf_path.empty() && v && v[0] && fs::exists(v)) gguf_path = v;
        }
        if (gguf_path.empty() && p.extension() == ".gguf" && fs::exists(p)) gguf_path = p.string();
        if (gguf_path.empty() && fs::is_directory(p) && fs::exists(p / "model.gguf")) gguf_path = (p / "model.gguf").string();
        // online quantization request (get_quant_type_from_env, acestep_dit_model.cpp:27-45); the GGUF
        // loaders keep the file's types and never quantize (:526-718)
        const quant::QType qt = gguf_path.empty() ? quant::from_env() : quant::QNONE;

        DitConfig& c = m.cfg;
        load_config((root / "config.json").string(), c);
        if (c.head_dim != 128) throw Unsupported("head_dim must be 128");
        if (c.hidden % 128 != 0 || c.intermediate % 128 != 0) throw Unsupported("hidden/intermediate must be multiples of 128");
        if (c.hkv <= 0 || c.hq % c.hkv != 0) throw Unsupported("num_attention_heads must be a multiple of num_key_value_heads");
        const int rep = c.hq / c.hkv;
        if (rep != 1 && rep != 2 && rep != 4) throw Unsupported("GQA ratio must be 1, 2 or 4");
        if ((c.patch * c.in_channels) % 64 != 0) throw Unsupported("patch*in_channels must be a multiple of 64");
        if ((c.patch * c.audio_dim) % 128 != 0) throw Unsupported("patch*audio_dim must be a multiple of 128");

        Loader L(m.allocs, m.weight_bytes);
        L.qt = qt;
        m.qtype = qt;
        if (!gguf_path.empty()) {
            L.gguf = true;
            L.gg.open(gguf_path);
        } else {
            L.st.open((root / "model.safetensors").string());
        }
        const int H = c.hidden, I = c.intermediate, D = c.head_dim, P = c.patch, Cin = c.in_channels, A = c.audio_dim;
        const int qd = c.hq * D, kd = c.hkv * D;

        // proj_in: conv1d [H][Cin][P] -> [H][P*Cin] (load_conv1d_weight_as_linear :334-411; GGUF :602-637)
        {
            const Mat w = L.conv_f32("decoder.proj_in.1.weight", H, Cin, P);
            m.proj_in_w = L.finish(Loader::permute(
                                       w, H, (int64_t)P * Cin, [](int64_t r) { return r; },
                                       [&](int64_t col) { return (col % Cin) * P + col / Cin; }),
                                   true);
            m.proj_in_b = L.vec_f32("decoder.proj_in.1.bias", H);
        }
        // proj_out: convtranspose1d [H][A][P] -> [(o + k*A)][H] (load_convtranspose1d_weight_as_linear :413-490;
        // GGUF :639-677)
        {
            const Mat w = L.gguf ? L.conv_f32("decoder.proj_out.1.weight", H, A, P)
                                 : L.mat("decoder.proj_out.1.weight", H, (int64_t)A * P);
            // source element (i, o, k) sits at row i, column o*P + k; target (o + k*A, i)
            Mat wt;
            wt.dtype = w.dtype;
            wt.rows = (int64_t)A * P;
            wt.cols = H;
            if (w.dtype == "F32")
                wt.f32.resize((size_t)wt.rows * H);
            else
                wt.u16.resize((size_t)wt.rows * H);
            for (int i = 0; i < H; ++i)
                for (int o = 0; o < A; ++o)
                    for (int k = 0; k < P; ++k) {
                        const size_t si = ((size_t)i * A + o) * P + k, di = (size_t)(o + k * A) * H + i;
                        if (w.dtype == "F32")
                            wt.f32[di] = w.f32[si];
                        else
                            wt.u16[di] = w.u16[si];
                    }
            m.proj_out_w = L.finish(wt, true);
            m.proj_out_b = L.vec_f32("decoder.proj_out.1.bias", A);
        }
        m.cond_w = L.finish(L.mat("decoder.condition_embedder.weight", H, H));
        m.cond_b = L.vec_f32("decoder.condition_embedder.bias", H);
        m.norm_out = L.vec_f32("decoder.norm_out.weight", H);
        {
            auto ot = L.table("decoder.scale_shift_table", 2, H);
            m.out_table = L.upload<float>(ot.data(), ot.size() * 4);
        }
        const char* tags[2] = {"decoder.time_embed.", "decoder.time_embed_r."};
        for (int e = 0; e < 2; ++e) {
            const std::string p2 = tags[e];
            int64_t fin = 0;
            if (L.gguf) {
                const auto& t1 = L.gg.get(p2 + "linear_1.weight");
                if (t1.ne_at(1) != H || t1.ne_at(2) != 1) throw IoError("invalid tensor shape for " + p2 + "linear_1.weight");
                fin = t1.ne_at(0);
            } else {
                const auto& t1 = L.st.get(p2 + "linear_1.weight");
                if (t1.shape.size() != 2 || t1.shape[0] != H) throw IoError("invalid tensor shape for " + p2 + "linear_1.weight");
                fin = t1.shape[1];
            }
            if (fin != 256) throw Unsupported("timestep embedding input dim must be 256");
            ActType a1, a2, a3;
            m.te[e].w1 = L.finish16(L.mat(p2 + "linear_1.weight", H, fin), a1);
            m.te[e].b1 = L.vec_f32(p2 + "linear_1.bias", H);
            m.te[e].w2 = L.finish16(L.mat(p2 + "linear_2.weight", H, H), a2);
            m.te[e].b2 = L.vec_f32(p2 + "linear_2.bias", H);
            m.te[e].wp = L.finish16(L.mat(p2 + "time_proj.weight", 6LL * H, H), a3);
            m.te[e].bp = L.vec_f32(p2 + "time_proj.bias", 6LL * H);
            if (a1 != a2 || a2 != a3) throw Unsupported("mixed timestep weight types");
            m.te[e].act = a1;
            if (quant_act_from_env()) {
                m.te[e].q1 = L.finish(L.mat(p2 + "linear_1.weight", H, fin));
                m.te[e].q2 = L.finish(L.mat(p2 + "linear_2.weight", H, H));
                m.te[e].qp = L.finish(L.mat(p2 + "time_proj.weight", 6LL * H, H));
            }
        }
        std::vector<float> tables((size_t)c.layers * 6 * H);
        std::vector<Mat> ckv(c.layers);  // cross k|v rows per layer, uploaded as one matrix below
        m.layers.resize(c.layers);
        for (int i = 0; i < c.layers; ++i) {
            const std::string p2 = "decoder.layers." + std::to_string(i) + ".";
            DevLayer& ly = m.layers[i];
            ly.self_norm = L.vec_f32(p2 + "self_attn_norm.weight", H);
            ly.cross_norm = L.vec_f32(p2 + "cross_attn_norm.weight", H);
            ly.mlp_norm = L.vec_f32(p2 + "mlp_norm.weight", H);
            ly.sq_norm = L.vec_f32(p2 + "self_attn.q_norm.weight", D);
            ly.sk_norm = L.vec_f32(p2 + "self_attn.k_norm.weight", D);
            ly.cq_norm = L.vec_f32(p2 + "cross_attn.q_norm.weight", D);
            ly.ck_norm = L.vec_f32(p2 + "cross_attn.k_norm.weight", D);
            {
                const Mat wq = L.mat(p2 + "self_attn.q_proj.weight", qd, H);
                const Mat wk = L.mat(p2 + "self_attn.k_proj.weight", kd, H);
                const Mat wv = L.mat(p2 + "self_attn.v_proj.weight", kd, H);
                ly.w_qkv = L.finish(Loader::concat_rows({&wq, &wk, &wv}));
            }
            ly.w_o = L.finish(L.mat(p2 + "self_attn.o_proj.weight", H, qd));
            ly.w_cq = L.finish(L.mat(p2 + "cross_attn.q_proj.weight", qd, H));
            {
                const Mat wk = L.mat(p2 + "cross_attn.k_proj.weight", kd, H);
                const Mat wv = L.mat(p2 + "cross_attn.v_proj.weight", kd, H);
                ckv[i] = Loader::concat_rows({&wk, &wv});
            }
            ly.w_co = L.finish(L.mat(p2 + "cross_attn.o_proj.weight", H, qd));
            ly.w_gu = L.gate_up(p2, I, H);
            ly.w_down = L.finish(L.mat(p2 + "mlp.down_proj.weight", H, I));
            {
                auto v = L.table(p2 + "scale_shift_table", 6, H);
                std::memcpy(&tables[(size_t)i * 6 * H], v.data(), v.size() * 4);
            }
            ly.sliding = i < (int)c.layer_types.size() && c.layer_types[i] == "sliding_attention";
        }
        m.tables = L.upload<float>(tables.data(), tables.size() * 4);
        // every layer's cross k|v in one [layers*2kd][H] matrix when they share a type (always, except a
        // GGUF file mixing types across layers): the encoder-side projections become one GEMM with
        // N = layers*2kd instead of `layers` GEMMs of M = L rows that fill a quarter of the GPU
        bool one_type = true;
        for (int i = 1; i < c.layers; ++i)
            one_type = one_type && ckv[i].dtype == ckv[0].dtype && ckv[i].qt == ckv[0].qt;
        if (one_type && c.layers > 0) {
            std::vector<const Mat*> parts;
            for (const Mat& x : ckv) parts.push_back(&x);
            m.w_ckv_all = L.finish(Loader::concat_rows(parts));
            for (int i = 0; i < c.layers; ++i) {
                DevWeight v = m.w_ckv_all;
                v.rows = 2 * kd;
                const int64_t r0 = (int64_t)i * 2 * kd;
                const quant::QType q = v.fmt == WF_Q8_0 ? quant::Q8_0
                                       : v.fmt == WF_Q4_K ? quant::Q4_K
                                       : v.fmt == WF_Q6_K ? quant::Q6_K
                                                          : quant::QNONE;
                if (q == quant::QNONE) {
                    v.q = static_cast<char*>(v.q) + r0 * v.cols * 2;
                } else {
                    v.q = static_cast<char*>(v.q) + quant::q_plane_bytes(q, r0, v.cols);
                    v.s = v.s + quant::s_plane_floats(q, r0, v.cols);
                }
                m.layers[i].w_ckv = v;
            }
        } else {
            for (int i = 0; i < c.layers; ++i) m.layers[i].w_ckv = L.finish(ckv[i]);
        }
        ckv.clear();

        // ---- condition encoders (optional; acestep_dit_model.cpp:885-996)
        if (L.has("encoder.text_projector.weight")) {
            const auto sh = L.shape2("encoder.text_projector.weight");
            if (sh.first != H) throw IoError("invalid tensor shape for encoder.text_projector.weight");
            m.text_proj = L.finish(L.mat("encoder.text_projector.weight", sh.first, sh.second));
        }
        auto load_encoder = [&](const std::string& pre, int n_layers, DevEncoder& e) {
            if (L.has(pre + "embed_tokens.weight")) {
                const auto sh = L.shape2(pre + "embed_tokens.weight");
                e.embed = L.finish(L.mat(pre + "embed_tokens.weight", sh.first, sh.second));
            }
            if (L.has(pre + "embed_tokens.bias")) e.embed_b = L.vec_f32(pre + "embed_tokens.bias", H);
            if (L.has(pre + "norm.weight")) e.norm = L.vec_f32(pre + "norm.weight", H);
            e.layers.resize(std::max(0, n_layers));
            if (n_layers > 0) {
                const auto sh = L.shape2(pre + "layers.0.mlp.gate_proj.weight");
                if (sh.second != H || sh.first <= 0 || sh.first % 128 != 0)
                    throw Unsupported("encoder MLP width must be a multiple of 128: " + pre);
                e.intermediate = (int)sh.first;
            }
            const int EI = e.intermediate;
            for (int i = 0; i < n_layers; ++i) {  // EncoderLayer (:903-937 / :960-994)
                const std::string p2 = pre + "layers." + std::to_string(i) + ".";
                DevLayer& ly = e.layers[i];
                ly.cross = false;
                ly.self_norm = L.vec_f32(p2 + "input_layernorm.weight", H);
                ly.mlp_norm = L.vec_f32(p2 + "post_attention_layernorm.weight", H);
                ly.sq_norm = L.vec_f32(p2 + "self_attn.q_norm.weight", D);
                ly.sk_norm = L.vec_f32(p2 + "self_attn.k_norm.weight", D);
                const Mat wq = L.mat(p2 + "self_attn.q_proj.weight", qd, H);
                const Mat wk = L.mat(p2 + "self_attn.k_proj.weight", kd, H);
                const Mat wv = L.mat(p2 + "self_attn.v_proj.weight", kd, H);
                ly.w_qkv = L.finish(Loader::concat_rows({&wq, &wk, &wv}));
                ly.w_o = L.finish(L.mat(p2 + "self_attn.o_proj.weight", H, qd));
                ly.w_gu = L.gate_up(p2, EI, H);
                ly.w_down = L.finish(L.mat(p2 + "mlp.down_proj.weight", H, EI));
                ly.sliding = i < (int)c.layer_types.size() && c.layer_types[i] == "sliding_attention";
            }
            e.act = e.layers.empty() ? ActType::BF16 : e.layers[0].w_qkv.act();
            for (const DevLayer& ly : e.layers)
                for (const DevWeight* w : {&ly.w_qkv, &ly.w_o, &ly.w_gu, &ly.w_down})
                    if (w->act() != e.act) throw Unsupported("mixed encoder block weight types");
        };
        load_encoder("encoder.lyric_encoder.", c.lyric_layers, m.lyric);
        load_encoder("encoder.timbre_encoder.", c.timbre_layers, m.timbre);
        m.act = m.layers.empty() ? m.cond_w.act() : m.layers[0].w_qkv.act();
        for (const DevLayer& ly : m.layers)
            for (const DevWeight* w : {&ly.w_qkv, &ly.w_o, &ly.w_cq, &ly.w_ckv, &ly.w_co, &ly.w_gu, &ly.w_down})
                if (w->act() != m.act) throw Unsupported("mixed DiT block weight types");
        if (m.cond_w.act() != m.act) throw Unsupported("mixed DiT weight types");
        if (m.proj_out_w.fmt != WF_F32X3 && m.proj_out_w.act() != m.act) throw Unsupported("mixed DiT weight types");
    } catch (const Unsupported& e) {
        status_hint = 4;
        throw std::runtime_error(e.what());
    } catch (const HipError&) {
        status_hint = 1;
        throw;
    }
}

}  // namespace acemi
