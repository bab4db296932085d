// ggml block quantization of DiT weights (host side, load time).
//
// `try_quantize_matrix` (acestep_dit_model.cpp:156-192) quantizes every 2-D
// weight whose in-dim is a multiple of the block size when
// ACE_GGML_DIT_WEIGHT_QTYPE / ACE_GGML_WEIGHT_QTYPE asks for Q8_0, Q6_K or Q4_K
// (parse_quant_type :27-45).  The encoders below produce the ggml block bytes
// (quantize_row_*_ref of ggml 0.9.5, restated — see oracle/ggml_numerics.py),
// and `to_planes` re-lays the blocks out for the gfx950 dequant-fused GEMM:
//   Q8_0: q int8 [rows][cols]          s f32 [rows][cols/32]     (d)
//   Q4_K: q u8   [rows][cols/2]        s f32 [rows][cols/32][2]  (d*sc, dmin*m)
//         per 32-block 16 bytes; byte i: low nibble k = 8(i/4) + i%4, high nibble k + 4
//   Q6_K: q int8 [rows][cols] (q - 32) s f32 [rows][cols/16]     (d*sc)
// so that a GEMM thread turns one 32-value block into bf16 with one scale
// (two for Q6_K) and no bit gathering across bytes.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace acemi {
namespace quant {

enum QType : int { QNONE = 0, Q8_0 = 1, Q4_K = 2, Q6_K = 3 };

// parse_quant_type (acestep_dit_model.cpp:27-37): Q8/Q8_0, Q6/Q6_K, Q4/Q4_K/Q4_K_M (case-insensitive)
QType parse(const char* s);
// get_quant_type_from_env (:39-45): ACE_GGML_DIT_WEIGHT_QTYPE, else ACE_GGML_WEIGHT_QTYPE
QType from_env();
// the same rule with another model-specific key first (qwen_model.cpp:38-44: ACE_GGML_QWEN_WEIGHT_QTYPE)
QType from_env(const char* primary_key);
const char* name(QType t);

int block_values(QType t);       // 32 / 256 / 256
size_t block_bytes(QType t);     // 34 / 144 / 210
size_t row_bytes(QType t, int64_t cols);
bool applies(QType t, int64_t cols);  // in-dim % block == 0

// ggml block bytes of `rows` rows of `cols` f32 values (multithreaded over rows).
void quantize_rows(QType t, const float* src, int64_t rows, int64_t cols, uint8_t* dst);
// ggml dequantize_row_* to f32.
void dequantize_rows(QType t, const uint8_t* src, int64_t rows, int64_t cols, float* dst);

// Plane sizes (bytes) and conversion for the device layout described above.
size_t q_plane_bytes(QType t, int64_t rows, int64_t cols);
size_t s_plane_floats(QType t, int64_t rows, int64_t cols);
void to_planes(QType t, const uint8_t* blocks, int64_t rows, int64_t cols, uint8_t* qplane, float* splane);

}  // namespace quant
}  // namespace acemi
