// Host-side C-ABI utilities of the product library (include/acestep_mi355x.h): the loader's ggml block
// encoders (quantize_row_*_ref restated, runtime/quant.cpp; used by the GGUF exporter and the tests) and the
// GEMM tile override used for A/B measurements.
#include "../../../include/acestep_mi355x.h"
#include "../kernels.h"
#include "quant.h"

extern "C" {

// Force a GEMM kernel variant for subsequent launches (-1 = automatic).
ace_ggml_status ace_mi_gemm_variant(int32_t variant) {
    if (variant < -1 || variant % 100 > 25 || variant > 424) return ACE_GGML_ERR_INVALID_ARG;
    acemi::gemm_force_variant(variant);
    return ACE_GGML_OK;
}

// ggml block quantization of rows (the loader's encoders): returns bytes written, or -1.
int64_t ace_mi_quantize(int32_t qtype, const float* src, int64_t rows, int64_t cols, uint8_t* dst, size_t dst_size) {
    using namespace acemi;
    const auto t = static_cast<quant::QType>(qtype);
    if (!src || !dst || rows <= 0 || (t != quant::Q8_0 && t != quant::Q4_K && t != quant::Q6_K)) return -1;
    if (!quant::applies(t, cols)) return -1;
    const size_t need = (size_t)rows * quant::row_bytes(t, cols);
    if (dst_size < need) return -1;
    try {
        quant::quantize_rows(t, src, rows, cols, dst);
    } catch (const std::exception&) {
        return -1;
    }
    return (int64_t)need;
}

ace_ggml_status ace_mi_dequantize(int32_t qtype, const uint8_t* src, int64_t rows, int64_t cols, float* dst) {
    using namespace acemi;
    const auto t = static_cast<quant::QType>(qtype);
    if (!src || !dst || rows <= 0 || (t != quant::Q8_0 && t != quant::Q4_K && t != quant::Q6_K) ||
        !quant::applies(t, cols))
        return ACE_GGML_ERR_INVALID_ARG;
    quant::dequantize_rows(t, src, rows, cols, dst);
    return ACE_GGML_OK;
}

}  // extern "C"
