// Pre-norm transformer blocks without AdaLN — the Qwen3 layer shape shared by the lyric / timbre
// condition encoders (acestep_dit_model.cpp:1614-1645, :1705-1725) and the Qwen3 text encoder
// (qwen_model.cpp:567-677):
//   h = x + o_proj(attn(rope(qk_norm(qkv(rms_norm(x))))));  x = h + down(silu(gate(hn)) * up(hn)),
//   hn = rms_norm(h),
// run on the DiT's kernels (fused QKV GEMM, attn_prep, flash attention, residual / SwiGLU GEMM
// epilogues).  A BlockRunner owns its workspace, so a condition-encoder pass never touches the DiT
// engine's buffers (or its cross-attention cache).
#pragma once

#include <vector>

#include "../kernels.h"
#include "model.h"

namespace acemi {

struct BlockShape {
    int hidden = 0, hq = 0, hkv = 0, head_dim = 128, intermediate = 0;
    float eps = 1e-6f, rope_theta = 1000000.0f;
    int sliding_window = 0;  // |q - k| <= window on layers flagged sliding
};

class BlockRunner {
   public:
    BlockRunner();
    ~BlockRunner();
    BlockRunner(const BlockRunner&) = delete;
    BlockRunner& operator=(const BlockRunner&) = delete;
    // the residual stream [rows][H] f32 (grown on demand; contents kept while the size fits)
    float* x(int64_t rows, int H);
    // layers [0, n_layers) over x = [B][n][H] in place; key_mask [B][n] int32 (device) or null;
    // causal: key k > query q masked (the text encoder, qwen_model.cpp:618-637)
    void run(const BlockShape& sh, const std::vector<DevLayer>& layers, int n_layers, ActType act, int B, int n,
             const int32_t* key_mask, bool causal, hipStream_t s);
    // out = RMSNorm(x) * w (w null: a plain copy) for all B*n rows, or each item's token 0 when first_only
    void finish(const BlockShape& sh, const float* w, int B, int n, bool first_only, float* out, hipStream_t s);

   private:
    struct Buf {
        void* p = nullptr;
        size_t bytes = 0;
    };
    void ensure(Buf& b, size_t bytes);
    template <typename T>
    T* get(Buf& b) {
        return static_cast<T*>(b.p);
    }
    Buf x_, act_, attn_, act2_, qkv_, qh_, kh_, vt_, kbias_, cos_, sin_;
    int rope_n_ = -1;
    float rope_theta_ = 0.f;
    bool split_ = true;  // hi/lo fp16 Q.K operands (ACE_MI_ATTN_PRECISION)
    bool pv_split_ = true;  // hi/lo fp16 P.V operands too
};

}  // namespace acemi
