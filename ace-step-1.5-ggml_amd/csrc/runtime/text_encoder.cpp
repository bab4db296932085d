// Qwen3 text encoder: loader + forward (text_encoder.h).
#include "text_encoder.h"

#include <algorithm>
#include <cstdlib>
#include <filesystem>

#include "json.h"
#include "loader.h"

namespace acemi {

TextModel::~TextModel() {
    for (void* p : allocs) (void)hipFree(p);
}

namespace {

void load_text_config(const std::string& path, TextConfig& c) {  // qwen_config.cpp:19-64
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
        c.vocab = (int)o.at("vocab_size").as_int();
        c.hidden = (int)o.at("hidden_size").as_int();
        c.layers = (int)o.at("num_hidden_layers").as_int();
        c.hq = (int)o.at("num_attention_heads").as_int();
        c.hkv = (int)o.at("num_key_value_heads").as_int();
        c.intermediate = (int)o.at("intermediate_size").as_int();
        c.head_dim = (int)o.at("head_dim").as_int();
        c.max_pos = (int)o.at("max_position_embeddings").as_int();
        c.eps = (float)o.at("rms_norm_eps").as_num();
        if (o.has("rope_theta")) c.rope_theta = (float)o.at("rope_theta").as_num();
        if (o.has("dtype") && o.at("dtype").kind == Json::String) c.dtype = o.at("dtype").as_str();
    } catch (const IoError&) {
        throw;
    } catch (const std::exception& e) {
        throw IoError(std::string("config: ") + e.what());
    }
}

// resolve_gguf_path (qwen_model.cpp:46-72)
std::string resolve_text_gguf(const std::string& dir) {
    namespace fs = std::filesystem;
    for (const char* key : {"ACE_GGML_QWEN_GGUF", "ACE_GGML_TEXT_ENCODER_GGUF", "ACE_GGML_LM_GGUF"}) {
        const char* v = std::getenv(key);
        if (v && v[0] && fs::exists(v)) return v;
    }
    const fs::path p(dir);
    if (p.extension() == ".gguf" && fs::exists(p)) return p.string();
    if (fs::is_directory(p) && fs::exists(p / "model.gguf")) return (p / "model.gguf").string();
    return "";
}

}  // namespace

void load_text_model(const std::string& dir, TextModel& m) {
    namespace fs = std::filesystem;
    const fs::path p(dir);
    const fs::path root = p.extension() == ".gguf" ? p.parent_path() : p;
    const std::string gguf_path = resolve_text_gguf(dir);
    TextConfig& c = m.cfg;
    load_text_config((root / "config.json").string(), c);
    if (c.head_dim != 128) throw Unsupported("text encoder head_dim must be 128");
    if (c.hidden % 128 != 0 || c.intermediate % 128 != 0 || c.hidden > 4096)
        throw Unsupported("text encoder hidden/intermediate must be multiples of 128 (hidden <= 4096)");
    if (c.hkv <= 0 || c.hq % c.hkv != 0) throw Unsupported("num_attention_heads must be a multiple of num_key_value_heads");
    const int rep = c.hq / c.hkv;
    if (rep != 1 && rep != 2 && rep != 4) throw Unsupported("GQA ratio must be 1, 2 or 4");
    if (c.vocab <= 0 || c.layers < 0) throw IoError("invalid text encoder config");

    Loader L(m.allocs, m.weight_bytes);
    // get_quant_type_from_env (qwen_model.cpp:38-44); the GGUF loaders keep the file's types
    L.qt = gguf_path.empty() ? quant::from_env("ACE_GGML_QWEN_WEIGHT_QTYPE") : quant::QNONE;
    m.qtype = L.qt;
    if (!gguf_path.empty()) {
        L.gguf = true;
        L.gg.open(gguf_path);
    } else {
        L.st.open((root / "model.safetensors").string());
    }
    const int H = c.hidden, I = c.intermediate, D = c.head_dim, qd = c.hq * D, kd = c.hkv * D;
    {  // embed_tokens: ggml_get_rows + cast_f32 yields the stored values (dequantized if quantized)
        const Mat e = L.mat("embed_tokens.weight", c.vocab, H);
        if (e.dtype == "BF16" || e.dtype == "F16") {
            if (!quant::applies(L.qt, H)) {
                m.embed_fmt = e.dtype == "BF16" ? 0 : 1;
                m.embed = L.upload<uint16_t>(e.u16.data(), e.u16.size() * 2);
            }
        }
        if (!m.embed) {
            std::vector<float> v = L.values(e);
            if (e.dtype != "Q" && quant::applies(L.qt, H)) {  // quantized at load, read back by get_rows
                std::vector<uint8_t> blocks((size_t)c.vocab * quant::row_bytes(L.qt, H));
                quant::quantize_rows(L.qt, v.data(), c.vocab, H, blocks.data());
                quant::dequantize_rows(L.qt, blocks.data(), c.vocab, H, v.data());
            }
            m.embed_fmt = 2;
            m.embed = L.upload<float>(v.data(), v.size() * 4);
        }
    }
    m.norm = L.vec_f32("norm.weight", H);
    m.layers.resize(c.layers);
    for (int i = 0; i < c.layers; ++i) {  // qwen_model.cpp:438-471
        const std::string p2 = "layers." + std::to_string(i) + ".";
        DevLayer& ly = m.layers[i];
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
        ly.w_gu = L.gate_up(p2, I, H);
        ly.w_down = L.finish(L.mat(p2 + "mlp.down_proj.weight", H, I));
    }
    m.act = m.layers.empty() ? ActType::BF16 : m.layers[0].w_qkv.act();
    for (const DevLayer& ly : m.layers)
        for (const DevWeight* w : {&ly.w_qkv, &ly.w_o, &ly.w_gu, &ly.w_down})
            if (w->act() != m.act) throw Unsupported("mixed text encoder weight types");
}

BlockShape TextEncoderEngine::shape() const {
    const TextConfig& c = model_.cfg;
    BlockShape sh;
    sh.hidden = c.hidden;
    sh.hq = c.hq;
    sh.hkv = c.hkv;
    sh.head_dim = c.head_dim;
    sh.intermediate = c.intermediate;
    sh.eps = c.eps;
    sh.rope_theta = c.rope_theta;
    return sh;
}

void TextEncoderEngine::embeddings(const int32_t* d_ids, int n, float* d_out, hipStream_t s) {
    launch_embed_rows(model_.embed, model_.embed_fmt, d_ids, n, model_.cfg.hidden, d_out, s);
}

void TextEncoderEngine::forward(const int32_t* d_ids, const int32_t* d_mask, int n, int n_layers, bool final_norm,
                                float* d_out, hipStream_t s) {
    const TextModel& m = model_;
    const int total = m.cfg.layers;
    const int run = n_layers < 0 ? total : std::min(n_layers, total);
    const BlockShape sh = shape();
    float* x = blocks_.x(n, sh.hidden);
    launch_embed_rows(m.embed, m.embed_fmt, d_ids, n, sh.hidden, x, s);
    blocks_.run(sh, m.layers, run, m.act, 1, n, d_mask, true, s);
    blocks_.finish(sh, (final_norm && run == total) ? m.norm : nullptr, 1, n, false, d_out, s);
}

}  // namespace acemi
