// Qwen3 text encoder resident in HBM: ace_qwen::Model / Config
// (acestep_ggml/cpp/qwen_model.h, qwen_config.cpp:19-64), loaded like load_model_from_dir
// (qwen_model.cpp:340-478) and run like forward_text_encoder_layers (:528-677) — token-embedding
// gather, causal pre-norm blocks on the shared BlockRunner, optional final RMSNorm.
#pragma once

#include <string>
#include <vector>

#include "blocks.h"
#include "model.h"

namespace acemi {

struct TextConfig {
    int vocab = 0, hidden = 0, layers = 0, hq = 0, hkv = 0, intermediate = 0, head_dim = 0, max_pos = 0;
    float eps = 1e-6f, rope_theta = 1000000.0f;
    std::string dtype;
};

struct TextModel {
    TextConfig cfg;
    void* embed = nullptr;  // [vocab][hidden]: bf16 / fp16 bits as stored, or f32 values (F32 or quantized)
    int embed_fmt = 0;      // launch_embed_rows fmt: 0 bf16, 1 fp16, 2 f32
    float* norm = nullptr;  // [hidden]
    std::vector<DevLayer> layers;
    ActType act = ActType::BF16;
    int qtype = 0;
    std::vector<void*> allocs;
    size_t weight_bytes = 0;
    ~TextModel();
};

// Throws std::runtime_error (the ABI reports ACE_GGML_ERR_IO like load_qwen_dir, acestep_ggml.cpp:238-244).
void load_text_model(const std::string& dir, TextModel& m);

class TextEncoderEngine {
   public:
    TextModel& model() { return model_; }
    BlockShape shape() const;
    // ids [n] (device) -> out [n][hidden] f32 token embeddings
    void embeddings(const int32_t* d_ids, int n, float* d_out, hipStream_t s);
    // forward_text_encoder_layers with causal = true: n_layers < 0 = all; the final norm only when
    // final_norm and every layer ran (:671-674); mask [n] int32 (device) or null
    void forward(const int32_t* d_ids, const int32_t* d_mask, int n, int n_layers, bool final_norm, float* d_out,
                 hipStream_t s);

   private:
    TextModel model_;
    BlockRunner blocks_;
};

}  // namespace acemi
