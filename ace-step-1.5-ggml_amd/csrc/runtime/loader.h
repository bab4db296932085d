// Weight-ingestion toolkit shared by the DiT and text-encoder loaders: safetensors / GGUF tensor
// reads, the reference's online quantization rule (try_quantize_matrix, acestep_dit_model.cpp:156-192;
// load_tensor_2d_transposed, qwen_model.cpp:185-240) and the device layouts of model.h
// (dense 16-bit, ggml block planes, F32 as an fp16 hi/lo triple).
#pragma once

#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "gguf.h"
#include "model.h"
#include "quant.h"
#include "safetensors.h"

namespace acemi {


// A 2-D weight as read from the file: raw 16-bit values, f32 (F32 files / quantization input), or
// ggml block rows (GGUF Q8_0 / Q4_K / Q6_K tensors, `qblocks` [rows][row_bytes]).
struct Mat {
    std::string dtype;  // BF16 | F16 | F32 | Q (blocks)
    int64_t rows = 0, cols = 0;
    std::vector<uint16_t> u16;
    std::vector<float> f32;
    quant::QType qt = quant::QNONE;
    std::vector<uint8_t> qblocks;
    float at(size_t i) const {
        if (dtype == "F32") return f32[i];
        if (dtype == "BF16") {
            uint32_t u = static_cast<uint32_t>(u16[i]) << 16;
            float r;
            std::memcpy(&r, &u, 4);
            return r;
        }
        return half_to_f32(u16[i]);
    }
};

inline quant::QType qtype_of_ggml(int t) {
    return t == GGML_Q8_0 ? quant::Q8_0 : (t == GGML_Q4_K ? quant::Q4_K : (t == GGML_Q6_K ? quant::Q6_K : quant::QNONE));
}

inline uint16_t f32_to_bf16_host(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);  // RNE (finite values)
    return static_cast<uint16_t>(u >> 16);
}
inline uint16_t f32_to_f16_host(float f) {
    _Float16 h = (_Float16)f;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}

struct Loader {
    std::vector<void*>& allocs;  // device allocations of the model being loaded (freed by its owner)
    size_t& weight_bytes;
    StFile st;
    GgufFile gg;
    bool gguf = false;
    std::string wdtype;  // dtype of the 16-bit 2-D weights (BF16 or F16)
    quant::QType qt = quant::QNONE;
    Loader(std::vector<void*>& a, size_t& wb) : allocs(a), weight_bytes(wb) {}

    template <typename T>
    T* upload(const void* host, size_t bytes) {
        void* d = nullptr;
        ACEMI_HIP(hipMalloc(&d, bytes));
        allocs.push_back(d);
        ACEMI_HIP(hipMemcpy(d, host, bytes, hipMemcpyHostToDevice));
        ACEMI_HIP(hipDeviceSynchronize());  // null-stream copy: done before any stream reads it
        weight_bytes += bytes;
        return static_cast<T*>(d);
    }
    // F32 / F16 / BF16 tensor -> f32 values (read_gguf_tensor_as_f32, acestep_dit_model.cpp:554-600)
    std::vector<float> gguf_f32(const GgufTensor& t) {
        auto raw = gg.read(t);
        int64_t n = 1;
        for (auto d : t.ne) n *= d;
        std::vector<float> v((size_t)n);
        if (t.type == GGML_F32) {
            std::memcpy(v.data(), raw.data(), (size_t)n * 4);
        } else if (t.type == GGML_F16 || t.type == GGML_BF16) {
            const uint16_t* p = reinterpret_cast<const uint16_t*>(raw.data());
            for (int64_t i = 0; i < n; ++i) {
                if (t.type == GGML_F16) {
                    v[(size_t)i] = half_to_f32(p[i]);
                } else {
                    uint32_t u = (uint32_t)p[i] << 16;
                    std::memcpy(&v[(size_t)i], &u, 4);
                }
            }
        } else {
            throw Unsupported("unsupported gguf tensor type for conversion: " + t.name);
        }
        return v;
    }
    // load_tensor_1d[_from_gguf] + cast_f32
    float* vec_f32(const std::string& name, int64_t expect) {
        std::vector<float> v;
        if (gguf) {
            const auto& t = gg.get(name);
            if (t.ne_at(1) != 1 || t.ne_at(2) != 1 || t.ne_at(3) != 1) throw IoError("invalid 1d tensor shape in gguf: " + name);
            v = gguf_f32(t);
        } else {
            const auto& t = st.get(name);
            v = to_f32(t, st.read(t));
        }
        if (expect >= 0 && (int64_t)v.size() != expect) throw IoError("invalid tensor shape for " + name);
        return upload<float>(v.data(), v.size() * 4);
    }
    // matrix [rows][cols] (2-D, or 3-D flattened over the last two dims)
    Mat mat(const std::string& name, int64_t rows, int64_t cols) {
        Mat out;
        out.rows = rows;
        out.cols = cols;
        if (gguf) {  // load_tensor_2d_from_gguf (:526-552): ne0 = in (cols), ne1 = out (rows), type kept
            const auto& t = gg.get(name);
            if (t.ne_at(2) != 1 || t.ne_at(3) != 1) throw IoError("invalid 2d tensor shape in gguf: " + name);
            if (t.ne_at(0) != cols || t.ne_at(1) != rows) throw IoError("invalid tensor shape for " + name);
            const quant::QType q = qtype_of_ggml(t.type);
            if (q != quant::QNONE) {
                out.dtype = "Q";
                out.qt = q;
                out.qblocks = gg.read(t);
                return out;
            }
            if (t.type == GGML_F16 || t.type == GGML_BF16) {
                out.dtype = t.type == GGML_F16 ? "F16" : "BF16";
                auto raw = gg.read(t);
                out.u16.resize((size_t)(rows * cols));
                std::memcpy(out.u16.data(), raw.data(), out.u16.size() * 2);
                return out;
            }
            if (t.type == GGML_F32) {
                out.dtype = "F32";
                out.f32 = gguf_f32(t);
                return out;
            }
            throw Unsupported(std::string("unsupported gguf tensor type ") + ggml_type_name(t.type) + ": " + name);
        }
        const auto& t = st.get(name);
        int64_t r = 1, c = 1;
        if (t.shape.size() == 2) {
            r = t.shape[0];
            c = t.shape[1];
        } else if (t.shape.size() == 3) {
            r = t.shape[0];
            c = t.shape[1] * t.shape[2];
        } else {
            throw IoError("invalid tensor shape for " + name);
        }
        if (r != rows || c != cols) throw IoError("invalid tensor shape for " + name);
        out.dtype = t.dtype;
        auto raw = st.read(t);
        if (t.dtype == "BF16" || t.dtype == "F16") {
            out.u16.resize(static_cast<size_t>(rows * cols));
            std::memcpy(out.u16.data(), raw.data(), out.u16.size() * 2);
        } else if (t.dtype == "F32") {
            out.f32 = to_f32(t, raw);
        } else {
            throw Unsupported("DiT 2-D weight " + name + " has dtype " + t.dtype + " (BF16/F16/F32 supported)");
        }
        return out;
    }
    bool has(const std::string& name) const { return gguf ? gg.has(name) : st.has(name); }
    // (rows, cols) of a 2-D weight as stored (torch [out][in]; GGUF ne1 x ne0)
    std::pair<int64_t, int64_t> shape2(const std::string& name) const {
        if (gguf) {
            const auto& t = gg.get(name);
            if (t.ne_at(2) != 1 || t.ne_at(3) != 1) throw IoError("invalid 2d tensor shape in gguf: " + name);
            return {t.ne_at(1), t.ne_at(0)};
        }
        const auto& t = st.get(name);
        if (t.shape.size() != 2) throw IoError("invalid tensor shape for " + name);
        return {t.shape[0], t.shape[1]};
    }
    // conv weights as f32 values (proj_in [H][Cin][P], proj_out [H][A][P]): the GGUF path converts them
    // to F32 (load_conv1d/convtranspose1d_weight_as_linear_from_gguf, :602-718)
    Mat conv_f32(const std::string& name, int64_t d0, int64_t d1, int64_t d2) {
        Mat out;
        out.rows = d0;
        out.cols = d1 * d2;
        out.dtype = "F32";
        if (gguf) {
            const auto& t = gg.get(name);
            if (t.ne_at(0) != d2 || t.ne_at(1) != d1 || t.ne_at(2) != d0 || t.ne_at(3) != 1)
                throw IoError("invalid conv1d tensor shape in gguf: " + name);
            out.f32 = gguf_f32(t);
            return out;
        }
        return mat(name, d0, d1 * d2);
    }
    // new matrix whose row r is row src_row(r) of `a`, with columns permuted by src_col(c)
    template <typename RowF, typename ColF>
    static Mat permute(const Mat& a, int64_t rows, int64_t cols, RowF src_row, ColF src_col) {
        Mat o;
        o.dtype = a.dtype;
        o.qt = a.qt;
        o.rows = rows;
        o.cols = cols;
        if (a.dtype == "Q") {  // whole block rows only (column order is fixed by the blocks)
            const size_t rb = quant::row_bytes(a.qt, a.cols);
            o.qblocks.resize((size_t)rows * rb);
            for (int64_t r = 0; r < rows; ++r)
                std::memcpy(&o.qblocks[(size_t)r * rb], &a.qblocks[(size_t)src_row(r) * rb], rb);
            return o;
        }
        if (a.dtype == "F32")
            o.f32.resize(static_cast<size_t>(rows * cols));
        else
            o.u16.resize(static_cast<size_t>(rows * cols));
        for (int64_t r = 0; r < rows; ++r)
            for (int64_t c = 0; c < cols; ++c) {
                const size_t si = static_cast<size_t>(src_row(r) * a.cols + src_col(c));
                const size_t di = static_cast<size_t>(r * cols + c);
                if (a.dtype == "F32")
                    o.f32[di] = a.f32[si];
                else
                    o.u16[di] = a.u16[si];
            }
        return o;
    }
    static Mat concat_rows(const std::vector<const Mat*>& parts) {
        Mat o;
        o.dtype = parts[0]->dtype;
        o.qt = parts[0]->qt;
        o.cols = parts[0]->cols;
        for (const Mat* p : parts) {
            if (p->dtype != o.dtype || p->qt != o.qt || p->cols != o.cols)
                throw Unsupported("fused weights must share one type");
            o.rows += p->rows;
            o.u16.insert(o.u16.end(), p->u16.begin(), p->u16.end());
            o.f32.insert(o.f32.end(), p->f32.begin(), p->f32.end());
            o.qblocks.insert(o.qblocks.end(), p->qblocks.begin(), p->qblocks.end());
        }
        return o;
    }
    std::vector<float> values(const Mat& a) {
        std::vector<float> v(static_cast<size_t>(a.rows * a.cols));
        if (a.dtype == "Q") {
            quant::dequantize_rows(a.qt, a.qblocks.data(), a.rows, a.cols, v.data());
            return v;
        }
        for (size_t i = 0; i < v.size(); ++i) v[i] = a.at(i);
        return v;
    }
    DevWeight from_blocks(quant::QType q, const uint8_t* blocks, int64_t rows, int64_t cols) {
        DevWeight w;
        w.rows = static_cast<int>(rows);
        w.cols = static_cast<int>(cols);
        std::vector<uint8_t> qp(quant::q_plane_bytes(q, rows, cols));
        std::vector<float> sp(quant::s_plane_floats(q, rows, cols));
        quant::to_planes(q, blocks, rows, cols, qp.data(), sp.data());
        w.fmt = q == quant::Q8_0 ? WF_Q8_0 : (q == quant::Q4_K ? WF_Q4_K : WF_Q6_K);
        w.q = upload<uint8_t>(qp.data(), qp.size());
        w.s = upload<float>(sp.data(), sp.size() * 4);
        return w;
    }
    // F32 weight kept at f32 precision (ggml: F32 mul_mat, activation not rounded): stored as the fp16
    // pair [hi | lo | hi] along K, multiplied with an activation written as [hi | hi | lo]
    // (Ah.Wh + Ah.Wl + Al.Wh, ~22-bit operands) by the ordinary fp16 GEMM with K' = 3K.
    DevWeight f32x3(const Mat& a) {
        DevWeight w;
        w.rows = static_cast<int>(a.rows);
        w.cols = static_cast<int>(a.cols);
        w.fmt = WF_F32X3;
        const auto v = values(a);
        std::vector<uint16_t> h((size_t)a.rows * 3 * a.cols);
        for (int64_t r = 0; r < a.rows; ++r)
            for (int64_t c = 0; c < a.cols; ++c) {
                const float x = v[(size_t)(r * a.cols + c)];
                const uint16_t hi = f32_to_f16_host(x);
                const uint16_t lo = f32_to_f16_host(x - half_to_f32(hi));
                uint16_t* row = &h[(size_t)r * 3 * a.cols];
                row[c] = hi;
                row[a.cols + c] = lo;
                row[2 * a.cols + c] = hi;
            }
        w.q = upload<uint16_t>(h.data(), h.size() * 2);
        return w;
    }
    // try_quantize_matrix (acestep_dit_model.cpp:156-192): quantize when requested and in-dim % block == 0
    DevWeight finish(const Mat& a, bool allow_f32 = false) {
        if (a.dtype == "Q") return from_blocks(a.qt, a.qblocks.data(), a.rows, a.cols);
        if (quant::applies(qt, a.cols)) {
            const auto v = values(a);
            std::vector<uint8_t> blocks(static_cast<size_t>(a.rows) * quant::row_bytes(qt, a.cols));
            quant::quantize_rows(qt, v.data(), a.rows, a.cols, blocks.data());
            return from_blocks(qt, blocks.data(), a.rows, a.cols);
        }
        if (a.dtype == "F32") {
            if (allow_f32) return f32x3(a);
            throw Unsupported("F32 2-D DiT weights are supported for proj_in/proj_out or with online quantization");
        }
        if (wdtype.empty()) wdtype = a.dtype;
        if (a.dtype != wdtype) throw Unsupported("mixed 16-bit 2-D weight dtypes are not supported");
        DevWeight w;
        w.rows = static_cast<int>(a.rows);
        w.cols = static_cast<int>(a.cols);
        w.fmt = a.dtype == "F16" ? WF_F16 : WF_BF16;
        w.q = upload<uint16_t>(a.u16.data(), a.u16.size() * 2);
        return w;
    }
    // dense 16-bit copy for the GEMV path: the file bits, or bf16(dequant(q)) for quantized weights
    uint16_t* finish16(const Mat& a, ActType& act) {
        if (a.dtype == "Q" || quant::applies(qt, a.cols) || a.dtype == "F32") {
            auto v = values(a);
            if (a.dtype != "Q" && quant::applies(qt, a.cols)) {
                std::vector<uint8_t> blocks(static_cast<size_t>(a.rows) * quant::row_bytes(qt, a.cols));
                quant::quantize_rows(qt, v.data(), a.rows, a.cols, blocks.data());
                quant::dequantize_rows(qt, blocks.data(), a.rows, a.cols, v.data());
            }
            std::vector<uint16_t> b(v.size());
            for (size_t i = 0; i < v.size(); ++i) b[i] = f32_to_bf16_host(v[i]);
            act = ActType::BF16;
            return upload<uint16_t>(b.data(), b.size() * 2);
        }
        act = a.dtype == "F16" ? ActType::F16 : ActType::BF16;
        return upload<uint16_t>(a.u16.data(), a.u16.size() * 2);
    }
    // mlp.gate_proj | mlp.up_proj as one [2I][H] weight, rows interleaved in groups of 16
    // ([g0..15, u0..15, g16..31, ...]) for the SwiGLU epilogue
    DevWeight gate_up(const std::string& p, int I, int H) {
        const Mat wg = mat(p + "mlp.gate_proj.weight", I, H);
        const Mat wu = mat(p + "mlp.up_proj.weight", I, H);
        const Mat gu = concat_rows({&wg, &wu});
        return finish(permute(
            gu, 2LL * I, H,
            [&](int64_t r) {
                const int64_t grp = r / 32, w = r % 32;
                return (w < 16 ? 0 : (int64_t)I) + grp * 16 + (w % 16);
            },
            [](int64_t col) { return col; }));
    }
    // cast_f32 of a table loaded by load_tensor_3d_as_2d: dequant(quant(t)) when it is quantized
    std::vector<float> table(const std::string& name, int64_t rows, int64_t cols) {
        if (gguf) {  // load_tensor_3d_as_2d_from_gguf (:554-585): ne = (cols, rows, 1)
            const auto& t = gg.get(name);
            if (t.ne_at(0) != cols || t.ne_at(1) != rows || t.ne_at(2) != 1) throw IoError("invalid 3d-as-2d tensor shape in gguf: " + name);
            const quant::QType q = qtype_of_ggml(t.type);
            if (q != quant::QNONE) {
                auto raw = gg.read(t);
                std::vector<float> v((size_t)(rows * cols));
                quant::dequantize_rows(q, raw.data(), rows, cols, v.data());
                return v;
            }
            return gguf_f32(t);
        }
        const auto& t = st.get(name);
        if (t.numel() != rows * cols) throw IoError("invalid tensor shape for " + name);
        auto v = to_f32(t, st.read(t));
        if (quant::applies(qt, cols)) {
            std::vector<uint8_t> blocks(static_cast<size_t>(rows) * quant::row_bytes(qt, cols));
            quant::quantize_rows(qt, v.data(), rows, cols, blocks.data());
            quant::dequantize_rows(qt, blocks.data(), rows, cols, v.data());
        }
        return v;
    }
};

}  // namespace acemi
