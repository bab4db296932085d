// DiT weights resident in HBM, laid out for the gfx950 kernels.
//
// Mirrors ace_dit::Model / Layer / AttnWeights / MLPWeights / TimestepWeights
// (acestep_ggml/cpp/acestep_dit_model.h:15-91) and ace_dit::Config
// (acestep_dit_config.h:10-32), loaded like ace_dit::load_model_from_dir
// (acestep_dit_model.cpp:753-1088) but fused for the MI355X kernels:
//   * q|k|v rows concatenated into one [ (Hq+2Hkv)*D ][H] matrix (one GEMM),
//   * cross k|v concatenated, gate|up interleaved in 16-row groups so the
//     GEMM epilogue sees matching gate/up columns in one wave,
//   * norms, biases and AdaLN tables widened to f32 once (ggml cast_f32).
#pragma once

#include <string>
#include <vector>

#include "../common.h"
#include "../kernels.h"

namespace acemi {

struct DitConfig {
    int hidden = 0, intermediate = 0, layers = 0, hq = 0, hkv = 0, head_dim = 0;
    int max_pos = 0, patch = 0, in_channels = 0, audio_dim = 0;
    float eps = 1e-6f, rope_theta = 1000000.0f;
    int sliding_window = 0;
    bool use_sliding_window = false;
    std::vector<std::string> layer_types;
    // condition encoders (acestep_dit_config.h:21-27; 0 = absent)
    int text_hidden_dim = 0, lyric_layers = 0, timbre_hidden_dim = 0, timbre_layers = 0, timbre_fix_frame = 0;
    int ctx_dim() const { return in_channels - audio_dim; }
    // input width of the lyric encoder / timbre encoder (forward_lyric_encoder :1572, forward_timbre_encoder
    // :1659-1661)
    int lyric_in_dim() const { return text_hidden_dim > 0 ? text_hidden_dim : 1024; }
    int timbre_in_dim() const { return timbre_hidden_dim > 0 ? timbre_hidden_dim : (audio_dim > 0 ? audio_dim : 64); }
};

// A 2-D linear weight [rows = out][cols = in] in HBM: dense 16-bit (file dtype) or one of the
// ggml block formats re-laid out as q/s planes (runtime/quant.h) when online quantization is on.
struct DevWeight {
    int fmt = WF_BF16;
    void* q = nullptr;
    float* s = nullptr;
    int rows = 0, cols = 0;
    WeightView view() const {
        WeightView v;
        v.fmt = fmt == WF_F32X3 ? WF_F16 : fmt;
        v.q = q;
        v.s = s;
        v.ld = fmt == WF_F32X3 ? 3 * cols : cols;
        return v;
    }
    int k_mult() const { return fmt == WF_F32X3 ? 3 : 1; }  // GEMM K = k_mult * cols
    ActType act() const { return weight_act(fmt); }
};

struct DevLayer {
    DevWeight w_qkv;   // [(hq+2hkv)*D][H]
    DevWeight w_o;     // [H][hq*D]
    DevWeight w_cq;    // [hq*D][H]
    DevWeight w_ckv;   // [2*hkv*D][H]
    DevWeight w_co;    // [H][hq*D]
    DevWeight w_gu;    // [2I][H] (16-row interleave)
    DevWeight w_down;  // [H][I]
    float* self_norm = nullptr;
    float* cross_norm = nullptr;
    float* mlp_norm = nullptr;
    float* sq_norm = nullptr;
    float* sk_norm = nullptr;
    float* cq_norm = nullptr;
    float* ck_norm = nullptr;
    bool sliding = false;
    bool cross = true;  // Layer::use_cross_attention default
};

// A condition encoder (ace_dit::Model lyric_* / timbre_*, acestep_dit_model.h; loaded at
// acestep_dit_model.cpp:889-996): input projection (+ bias), Qwen-style blocks without AdaLN stored in
// DevLayer (self_norm = input_layernorm, mlp_norm = post_attention_layernorm, no cross-attention), and
// an optional final RMSNorm weight.
struct DevEncoder {
    DevWeight embed;              // [H][in_dim] (embed_tokens.weight)
    float* embed_b = nullptr;     // [H] or null
    float* norm = nullptr;        // [H] or null
    std::vector<DevLayer> layers;
    int intermediate = 0;         // MLP width of the blocks (from mlp.gate_proj)
    ActType act = ActType::BF16;  // activation type of the block GEMMs
    bool has_embed() const { return embed.q != nullptr; }
};

// Timestep MLPs run as small-M GEMVs on dense 16-bit weights; when the checkpoint is quantized
// online they hold bf16(dequant(q)) — the same values the dequant-fused GEMM feeds its MFMAs.
struct DevTimestep {
    ActType act = ActType::BF16;
    uint16_t* w1 = nullptr;  // [H][256]
    uint16_t* w2 = nullptr;  // [H][H]
    uint16_t* wp = nullptr;  // [6H][H]
    float* b1 = nullptr;
    float* b2 = nullptr;
    float* bp = nullptr;
    // the same three weights in their ggml block format, kept only for the quantized-activation mode
    // (ACE_MI_QUANT_ACT=q8 at load: ggml multiplies Q8 activation blocks with the quantized weights themselves)
    DevWeight q1, q2, qp;
};

struct DitModel {
    DitConfig cfg;
    ActType act = ActType::BF16;     // activation type of every GEMM except proj_in
    int qtype = 0;                   // quant::QType of the online quantization (0 = none)
    DevWeight proj_in_w;             // [H][P*Cin], column k*Cin + c
    float* proj_in_b = nullptr;
    DevWeight proj_out_w;            // [P*audio][H], row o + k*audio
    float* proj_out_b = nullptr;
    DevWeight w_ckv_all;             // [layers * 2*hkv*D][H]: every layer's cross k|v rows in one matrix
                                     // (one GEMM per forward); DevLayer::w_ckv are views into it
    DevWeight cond_w;                // [H][H]
    float* cond_b = nullptr;
    float* norm_out = nullptr;
    float* out_table = nullptr;      // [2][H]
    float* tables = nullptr;         // [layers][6][H]
    DevTimestep te[2];               // time_embed, time_embed_r
    std::vector<DevLayer> layers;
    // condition encoders (optional tensors; acestep_dit_model.cpp:885-996)
    DevWeight text_proj;             // encoder.text_projector.weight [H][text_hidden] (no bias)
    DevEncoder lyric, timbre;
    std::vector<void*> allocs;
    size_t weight_bytes = 0;

    ~DitModel();
};

// ACE_MI_QUANT_ACT=q8: the ggml-faithful quantized-activation mode (DitEngine::forward_qact); anything else (the
// default, "bf16") = the product arithmetic, bf16 activations x bf16(dequant(W))
bool quant_act_from_env();

// Throws std::runtime_error with a reference-style message on failure.
// `status_hint` receives 3 (IO) or 4 (UNSUPPORTED) for the ABI status code.
void load_config(const std::string& path, DitConfig& cfg);
void load_dit_model(const std::string& dir, DitModel& m, int& status_hint);

}  // namespace acemi
