// Shared definitions for the MI355X (gfx950) ACE-Step DiT engine.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace acemi {

// Arithmetic type of the GEMM operands.  ggml's mul_mat converts the f32
// activation to the weight's vec_dot_type before the dot product
// (BF16 -> bf16, F16 -> fp16; acestep_dit_model.cpp:1194-1196 etc.), so the
// activation type always equals the weight type.
enum class ActType : int { BF16 = 0, F16 = 1 };

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

#define ACEMI_HIP(call)                                                                  \
    do {                                                                                 \
        hipError_t e_ = (call);                                                          \
        if (e_ != hipSuccess) {                                                          \
            throw ::acemi::HipError(std::string(#call) + ": " + hipGetErrorString(e_)); \
        }                                                                                \
    } while (0)

#define ACEMI_CHECK(cond, msg)                                   \
    do {                                                         \
        if (!(cond)) throw std::runtime_error(std::string(msg)); \
    } while (0)

inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace acemi
