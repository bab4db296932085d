// Oobleck VAE decoder resident in HBM + decode orchestration (ace_vae::forward_decode,
// acestep_ggml/cpp/acestep_vae_model.cpp:957-1002, loaded like load_model_from_dir :760-955).
//
// Weights: weight-norm folded at load exactly as load_conv_weight_norm (:520-588) and stored
// fp16 in the implicit-GEMM layouts of kernels/vae.hip:
//   conv (k taps):      W [Cout][k][Cin]          (K index = tap*Cin + ci)
//   conv_t (2s, s):     W [s*Cout][2][Cin]         W[r*Cout+co][tap*Cin+ci] = w[ci][co][r + tap*s]
// Snake parameters as exp(alpha), exp(beta) (expf on the host, as ggml_exp does on the CPU).
#pragma once

#include <cstdlib>

#include <string>
#include <vector>

#include "../common.h"
#include "../kernels.h"

namespace acemi {

struct VaeConfig {
    int audio_channels = 2, encoder_hidden_size = 128, decoder_channels = 128, decoder_input_channels = 64;
    int sampling_rate = 48000;
    std::vector<int> downsampling_ratios, upsampling_ratios, channel_multiples;
    int hop_length = 1;
};

struct VaeConv {
    uint16_t* w = nullptr;
    float* b = nullptr;
    int cin = 0, cout = 0, taps = 1, dil = 1, pad = 0, stride = 1;
    int cin_real = 0;  // < cin when the input channels were zero-padded to a multiple of 64
    bool transposed = false;
};
struct VaeSnake {
    float* ea = nullptr;
    float* eb = nullptr;
    int C = 0;
};
struct VaeRes {
    VaeSnake s1, s2;
    VaeConv c1, c2;
    int dil = 1;
};
struct VaeBlock {
    VaeSnake s1;
    VaeConv ct;
    VaeRes res[3];
    int stride = 1;
};

struct VaeEncBlock {  // diffusers OobleckEncoderBlock: 3 residual units, Snake, strided conv (k 2s)
    VaeRes res[3];
    VaeSnake s1;
    VaeConv conv;
    int stride = 1;
};

struct VaeModel {
    VaeConfig cfg;
    VaeConv conv1;
    std::vector<VaeBlock> blocks;
    VaeSnake snake1;
    VaeConv conv2;
    // encoder (optional: loaded when encoder.* tensors exist; required by encode)
    bool has_encoder = false;
    VaeConv enc_conv1;  // audio channels zero-padded to 64
    std::vector<VaeEncBlock> enc_blocks;
    VaeSnake enc_snake1;
    VaeConv enc_conv2;
    std::vector<void*> allocs;
    size_t weight_bytes = 0;
    ~VaeModel();
};

// Throws std::runtime_error; status_hint 3 (IO) / 4 (UNSUPPORTED) / 1 (ERR).
void load_vae_model(const std::string& dir, VaeModel& m, int& status_hint);

class VaeEngine {
public:
    explicit VaeEngine(int device) : device_(device) {
        const char* e = std::getenv("ACE_MI_VAE_FUSE_RES");
        fuse_res_ = !(e && e[0] == '0');
        // TEST ONLY (self-test library builds): ACE_MI_TEST_VAE_FAULT, runtime/test_hooks.cpp
        if (!test_vae_fault_from_env(fault_.block, fault_.row, fault_.col, fault_.amp)) fault_.block = -1;
    }
    ~VaeEngine();
    VaeModel& model() { return model_; }
    int device() const { return device_; }
    // samples produced for n_frames latent frames (= n_frames * hop for even strides; PyTorch
    // ConvTranspose1d lengths for odd ones)
    int64_t out_len(int n_frames) const;
    // latents [n_frames][latent_channels] f32 -> out [out_len][audio_channels] f32, device pointers
    // `items` windows of n_frames each in one pass: d_latents [items][n_frames][C], d_out
    // [items][out_len(n_frames)][audio_channels] (the windows of a tiled decode share every launch)
    void decode(const float* d_latents, int n_frames, float* d_out, hipStream_t s, int items = 1);
    // latent frames produced by encode (ggml_conv_1d output lengths of the strided convs)
    int64_t enc_out_len(int n_samples) const;
    // audio [n_samples][audio_channels] f32 -> latent mean [enc_out_len][latent_channels] f32
    void encode(const float* d_audio, int n_samples, float* d_out, hipStream_t s);

private:
    struct Buf {
        void* p = nullptr;
        size_t bytes = 0;
    };
    void ensure(Buf& b, size_t bytes);
    int device_;
    VaeModel model_;
    Buf x_, sa_, sb_, sc_, lat_, zero_;
    int items_ = 1;  // sequences per conv launch during decode (ConvGemmArgs::items)
    // 128-channel residual units as one launch (ConvGemmArgs::W2); ACE_MI_VAE_FUSE_RES=0: two launches
    bool fuse_res_ = true;
    struct {
        int block = -1, row = 0, col = 0;
        float amp = 0.f;
    } fault_;  // test-only negative control (ACE_MI_TEST_VAE_FAULT)
    const VaeRes* fused2_ = nullptr;  // set while run_conv launches the fused k7 + k1 of this unit
    void run_conv(const VaeConv& c, const uint16_t* S, int T_in, int T_out, float* X, bool resid, bool store,
                  uint16_t* S_out, const VaeSnake* next, hipStream_t s);
    uint16_t* run_res(const VaeRes& r, int L, float* X, uint16_t* Sin, uint16_t* Sspare, uint16_t* Sout,
                      const VaeSnake* next, hipStream_t s);
};

}  // namespace acemi
