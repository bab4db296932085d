// Batched DiT forward on one MI355X (stream-ordered, device pointers).
//
// One call = one denoising step for B samples that share (T, L): the token
// dimension of every linear becomes M = B * ceil(T / patch), so the GEMMs stay
// MFMA-bound even at batch 1 for long audio.  Functionally equal to B calls
// of ace_ggml_dit_forward (acestep_ggml.cpp:1304-1482), which the reference
// issues serially per item (scripts/run_non_ggml_real_case.py:518-527).
#pragma once

#include <map>
#include <memory>
#include <vector>

#include "../kernels.h"
#include "blocks.h"
#include "model.h"

namespace acemi {

struct ForwardIO {
    int B = 1, T = 0, L = 0;
    const float* hidden = nullptr;    // [B][T][audio] or null (zeros)
    const float* context = nullptr;   // [B][T][ctx]   or null (zeros)
    const float* enc = nullptr;       // [B][L][H]     (L > 0)
    const int32_t* mask = nullptr;    // [B][T] or null
    const int32_t* enc_mask = nullptr;// [B][L] or null
    const float* t = nullptr;         // [B]
    const float* r = nullptr;         // [B]
    float* out = nullptr;             // [B][T][audio]
    int max_layers = -1;              // ACE_GGML_DIT_MAX_LAYERS
    // Reuse the encoder-side tensors (condition_embedder output, every layer's cross K/V) computed
    // by the previous forward of this engine: the cross-attention cache of the reference generation
    // loop (acestep/mlx_dit/generate.py:150-171, MLXCrossAttentionCache / use_cache=True).  Only
    // valid when enc / enc_mask / B / L / layer count are those of that forward; the sampler entry
    // guarantees it.
    bool reuse_cross = false;
    // Reuse the bf16 images of the quantized block weights written by the previous forward of this engine
    // (staged dequant at sampling-call scope): set by the sampler entry for steps 1.. of one call.
    bool reuse_stage = false;
    // Timestep embeddings precomputed for this forward's B items (DitEngine::precompute_timesteps, the sampler
    // entry: every step's t is known when the sampling call starts): proj [B][6H] = the summed AdaLN projections
    // of t and t - r, temb_t / temb_r [B][H].  Null: computed from t / r inside the forward.
    const float* ts_proj = nullptr;
    const float* ts_temb_t = nullptr;
    const float* ts_temb_r = nullptr;
};

// One condition-encoder pass for B items of n tokens each (forward_lyric_encoder /
// forward_timbre_encoder, acestep_dit_model.cpp:1562-1739; the text projector of
// ace_project_tokens_linear, acestep_ggml.cpp:1624-1678, is the enc == null case):
//   x = in . proj^T (+ proj_b); x = block(x) for each layer; out = RMSNorm(x) * norm.
struct EncodeIO {
    const DevEncoder* enc = nullptr;  // blocks + final norm; null = projection only
    const DevWeight* proj = nullptr;  // input projection [H][in_dim]
    const float* proj_b = nullptr;    // [H] or null
    const float* in = nullptr;        // [B][n][in_dim] f32 (device)
    int B = 1, n = 0;
    bool first_only = false;          // out [B][H] = token 0 of each item (timbre embedding)
    float* out = nullptr;             // [B][n][H] or [B][H] f32 (device)
    int max_layers = -1;              // ACE_GGML_{LYRIC,TIMBRE}_MAX_LAYERS
};

// Per-kernel-class timing, filled when profiling is enabled (hipEvents on the launch stream).
struct KernelTimes {
    std::vector<std::string> names;
    std::vector<double> ms;
    std::vector<int> count;
};

class DitEngine {
   public:
    explicit DitEngine(int device);
    ~DitEngine();
    DitModel& model() { return model_; }
    int device() const { return device_; }
    void forward(const ForwardIO& io, hipStream_t s);
    // The timestep embeddings of `rows` (t, r) pairs in one pass (the weights read once per 8 rows instead of once
    // per forward): into engine buffers, returned as [rows][6H] proj and [rows][H] temb_t / temb_r pointers
    // (valid until the next call), bit-identical to what forward() computes for each row.
    struct TimestepRows {
        const float* proj;
        const float* temb_t;
        const float* temb_r;
    };
    TimestepRows precompute_timesteps(const float* t, const float* r, int rows, hipStream_t s);
    void encode(const EncodeIO& io, hipStream_t s);
    // attention operand precision of subsequent forwards (DiT blocks; the encoders keep their own)
    void set_attn_precision(AttnPrecision p) {
        attn_split_ = p == AttnPrecision::SPLIT || p == AttnPrecision::F32 || p == AttnPrecision::F8C;
        attn_pv_split_ = p == AttnPrecision::F32 || p == AttnPrecision::F8C || p == AttnPrecision::PV8;
        attn_f8_ = p == AttnPrecision::F8C || p == AttnPrecision::PV8;
        cross_key_.valid = false;  // cached cross K/V planes are in the previous mode's encoding
    }
    // enable per-kernel-class event timing for subsequent forwards
    void set_profiling(bool on);
    const KernelTimes& times() const { return times_; }
    void reset_times();
    // launch only the MLP gate/up GEMM of layer 0 for a given M (bench / roofline probe)
    void probe_gemm(int which, int M, int iters, hipStream_t s);

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
    void prepare_shape(int B, int Np, int L);
    void rope_for(int Np, hipStream_t s);
    void tic(hipStream_t s);
    void toc(const char* name, hipStream_t s);

    int device_;
    DitModel model_;
    // workspace
    Buf a0_, x_, act_, attn_, act2_, qkv_, qh_, kh_, vt_, kbias_, enc_act_, encp_, ckv_, kc_, vc_, kbias_c_;
    Buf attn_part_;  // key-range split partials of the attention kernel (AttnArgs::part)
    struct CrossKey {  // what kc_/vc_ currently hold (ForwardIO::reuse_cross)
        bool valid = false;
        int B = 0, L = 0, layers = 0;
        const float* enc = nullptr;
    } cross_key_;
    Buf freq_, freq_act_, th_, th_act_, temb_t_, temb_r_, temb_act_, proj_, mods_, outmod_, cos_, sin_;
    Buf ts_proj_, ts_temb_t_, ts_temb_r_;  // precompute_timesteps outputs
    // timestep MLPs for rows items (t, r pointers per row): proj [rows][6H] (t and t - r summed), temb_t / temb_r
    // [rows][H]; freq_ / th_ serve as scratch for up to 8 rows at a time
    void timestep_embed(const float* t, const float* r, int rows, float* proj, float* temb_t, float* temb_r,
                        hipStream_t s);
    int rope_np_ = -1;
    Buf knorm_tab_;  // [layers] device pointers to the cross k-norm weights
    size_t knorm_tab_n_ = 0;
    const float* const* cross_norm_table();
    Buf ein_;             // condition-encoder input activations
    BlockRunner cond_;    // condition-encoder blocks (own workspace: the DiT buffers stay untouched)
    void rope_table(int n, Buf& cs, Buf& sn, hipStream_t s);
    bool attn_split_ = false;  // hi/lo fp16 Q.K operands (ACE_MI_ATTN_PRECISION)
    bool attn_pv_split_ = false;  // hi/lo fp16 P.V operands too
    bool attn_f8_ = false;        // f8c: the lo planes hold fp8 operands (AttnArgs::f8)
    bool fused_prep_ = true;      // EPI_QKV_PREP (ACE_MI_UNFUSED_PREP=1: f32 store + attn_prep)
    void qkv_gemm(const uint16_t* act, const WeightView& w, int M, int N, PrepArgs pa, float* scratch,
                  const char* name, hipStream_t s);
    // ggml-faithful quantized-activation mode (ACE_MI_QUANT_ACT=q8, runtime/engine_qact.cpp): every linear with a
    // block-format weight quantizes its f32 input rows to Q8_0 / Q8_K blocks and runs the integer-dot GEMM
    // (launch_gemm_a8), the activations between the linears stay f32 (RMSNorm, attention output, SwiGLU), and
    // attention runs at the f32 precision -- the arithmetic of the reference's ggml graph.  A parity mode: the
    // product path keeps bf16 activations.
    bool qact_ = false;
    Buf qf_, qa_, qs_, qb_, encf_;  // f32 activation rows, their int8 blocks, block scales / sums, f32 condition
    Buf qa16_;                      // Q8_0 activation blocks as bf16(q) rows (the bf16-MFMA form, gemm_a8_bf16_path)
    std::map<const void*, Buf> q8img_;  // bf16(q) image of each Q8_0 plane, made at its first q8-mode use
    const uint16_t* q8_image(const WeightView& w, int N, int K, hipStream_t s);
    void forward_qact(const ForwardIO& io, hipStream_t s);
    void qlinear(const float* x, int64_t ldx, int M, const WeightView& w, int N, int K, const GemmEpilogue& e,
                 const char* name, hipStream_t s, bool silu_in = false);
    void timestep_embed_qact(const float* t, const float* r, int rows, float* proj, float* temb_t, float* temb_r,
                             hipStream_t s);
    // Staged dequant of quantized block weights (ACE_MI_QUANT_STAGED, default on; 0 = the dequant-fused GEMMs):
    // right before each layer its Q8_0 / Q4_K / Q6_K matrices are expanded to their bf16 image
    // (launch_dequant_bf16, bit-identical to the dequant-fused GEMM's LDS tiles) in one workspace slot, and
    // the block GEMMs run the dense bf16 kernels.  In stream order: a side-stream ring overlapped with the
    // previous layer gained nothing measurable (the GEMMs leave no CU resources for it) and, for Q4_K only,
    // changed the results of the concurrently running layer (tools/diag_staged.py) — not understood, so
    // not used.
    struct LayerViews {
        WeightView qkv, o, cq, co, gu, down;
    };
    // Scope of the staged images (ACE_MI_QUANT_STAGE_SCOPE): "model" (default since round 3) expands every layer's
    // image once, at the first forward after the load, and keeps it while the weights are loaded (they never change),
    // so the per-step decoder.forward hook and the ABI forward do not re-expand them either; "call" keeps one
    // slot per layer for one sampling call (expanded at its step 0); both cost a bf16 image of the block weights
    // as workspace (2.8 GB for the 24-layer DiT: 1 % of HBM); "layer" = the single shared 117 MB slot, expanded
    // before every layer of every forward (the low-memory mode: weights + one slot).
    bool staged_quant_ = true;
    bool stage_per_call_ = true;
    bool stage_model_ = true;  // images kept across calls while the weights are loaded (ACE_MI_QUANT_STAGE_SCOPE)
    size_t stage_slot_bytes_ = 0;
    int stage_layers_ = 0;  // layers whose images wring_ holds (per-call scope)
    Buf wring_;
    // bf16 images of the quantized weights outside the six block matrices (condition embedder, every layer's
    // cross k|v, proj in / out), expanded at their first use and kept while the weights are loaded (model and
    // call scope; the layer scope runs them through the dequant-fused GEMM)
    std::map<const void*, Buf> img_;
    // recorded after a forward that wrote bf16 images (staged slots or dense_view images); every later forward's
    // stream waits on it, so a forward on another stream never reads an image still being expanded
    hipEvent_t stage_ev_ = nullptr;
    bool stage_ev_set_ = false;
    bool images_written_ = false;
    WeightView dense_view(const DevWeight& w, hipStream_t s);
    char* stage_slot(int li);
    LayerViews layer_views(int li, bool staged);
    void stage_layer(int li, hipStream_t st);
    struct Fault {  // ACE_MI_TEST_FAULT (test-only fault injection); layer -1 = off
        int layer = -1, row = 0, col = 0;
        float amp = 0.f;
    } fault_;
    // ACE_MI_WEIGHT_PREFETCH=B: at the start of layer l, a side stream sweeps layer l+1's block weights (B
    // workgroups) so the memory-side cache holds them when its GEMMs start (short sequences read every weight
    // cold: tools/gemm_msweep.py with ACE_MI_BENCH_COLD); 0 = off (default)
    int prefetch_blocks_ = 0;
    hipStream_t pf_stream_ = nullptr;
    hipEvent_t pf_ev_ = nullptr, pf_done_ = nullptr;
    Buf pf_sink_;
    void prefetch_layer(int li, bool staged, hipStream_t s);
    // profiling
    bool profiling_ = false;
    hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
    KernelTimes times_;
};

}  // namespace acemi
