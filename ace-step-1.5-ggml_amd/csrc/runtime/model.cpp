// Weight ingestion: config.json + model.safetensors -> HBM (see model.h).
#include "model.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <sstream>

#include "json.h"
#include "gguf.h"
#include "quant.h"
#include "safetensors.h"

namespace acemi {
namespace {

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

quant::QType qtype_of_ggml(int t) {
    return t == GGML_Q8_0 ? quant::Q8_0 : (t == GGML_Q4_K ? quant::Q4_K : (t == GGML_Q6_K ? quant::Q6_K : quant::QNONE));
}

uint16_t f32_to_bf16_host(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    u += 0x7fffu + ((u >> 16) & 1u);  // RNE (finite values)
    return static_cast<uint16_t>(u >> 16);
}
uint16_t f32_to_f16_host(float f) {
    _Float16 h = (_Float16)f;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}

struct Loader {
    DitModel& m;
    StFile st;
    GgufFile gg;
    bool gguf = false;
    std::string wdtype;  // dtype of the 16-bit 2-D weights (BF16 or F16)
    quant::QType qt = quant::QNONE;
    explicit Loader(DitModel& mm) : m(mm) {}

    template <typename T>
    T* upload(const void* host, size_t bytes) {
        void* d = nullptr;
        ACEMI_HIP(hipMalloc(&d, bytes));
        m.allocs.push_back(d);
        ACEMI_HIP(hipMemcpy(d, host, bytes, hipMemcpyHostToDevice));
        m.weight_bytes += bytes;
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

}  // namespace

DitModel::~DitModel() {
    for (void* p : allocs) (void)hipFree(p);
}

void load_config(const std::string& path, DitConfig& c) {
    // acestep_dit_config.cpp:19-93 (required keys + optional ones)
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
        c.hidden = (int)o.at("hidden_size").as_int();
        c.intermediate = (int)o.at("intermediate_size").as_int();
        c.layers = (int)o.at("num_hidden_layers").as_int();
        c.hq = (int)o.at("num_attention_heads").as_int();
        c.hkv = (int)o.at("num_key_value_heads").as_int();
        c.head_dim = (int)o.at("head_dim").as_int();
        c.max_pos = (int)o.at("max_position_embeddings").as_int();
        c.eps = (float)o.at("rms_norm_eps").as_num();
        c.patch = (int)o.at("patch_size").as_int();
        c.in_channels = (int)o.at("in_channels").as_int();
        c.audio_dim = (int)o.at("audio_acoustic_hidden_dim").as_int();
        if (o.has("use_sliding_window")) c.use_sliding_window = o.at("use_sliding_window").as_bool();
        if (o.has("sliding_window") && o.at("sliding_window").kind == Json::Number)
            c.sliding_window = (int)o.at("sliding_window").as_int();
        if (o.has("rope_theta")) c.rope_theta = (float)o.at("rope_theta").as_num();
        auto opt_int = [&](const char* k, int& dst) {
            if (o.has(k) && o.at(k).kind == Json::Number) dst = (int)o.at(k).as_int();
        };
        opt_int("text_hidden_dim", c.text_hidden_dim);
        opt_int("num_lyric_encoder_hidden_layers", c.lyric_layers);
        opt_int("timbre_hidden_dim", c.timbre_hidden_dim);
        opt_int("num_timbre_encoder_hidden_layers", c.timbre_layers);
        opt_int("timbre_fix_frame", c.timbre_fix_frame);
        const auto& lt = o.at("layer_types");
        if (lt.kind != Json::Array) throw IoError("missing layer_types");
        c.layer_types.clear();
        for (const auto& v : lt.arr) c.layer_types.push_back(v.as_str());
    } catch (const IoError&) {
        throw;
    } catch (const std::exception& e) {
        throw IoError(std::string("config: ") + e.what());
    }
}

void load_dit_model(const std::string& dir, DitModel& m, int& status_hint) {
    status_hint = 3;
    try {
        namespace fs = std::filesystem;
        const fs::path p(dir);
        const fs::path root = p.extension() == ".gguf" ? p.parent_path() : p;
        // GGUF resolution order of resolve_gguf_path (acestep_dit_model.cpp:47-70)
        std::string gguf_path;
        for (const char* key : {"ACE_GGML_DIT_GGUF", "ACE_GGML_DIT_GGUF_PATH"}) {
            const char* v = std::getenv(key);
            if (gguf_path.empty() && v && v[0] && fs::exists(v)) gguf_path = v;
        }
        if (gguf_path.empty() && p.extension() == ".gguf" && fs::exists(p)) gguf_path = p.string();
        if (gguf_path.empty() && fs::is_directory(p) && fs::exists(p / "model.gguf")) gguf_path = (p / "model.gguf").string();
        // online quantization request (get_quant_type_from_env, acestep_dit_model.cpp:27-45); the GGUF
        // loaders keep the file's types and never quantize (:526-718)
        const quant::QType qt = gguf_path.empty() ? quant::from_env() : quant::QNONE;

        DitConfig& c = m.cfg;
        load_config((root / "config.json").string(), c);
        if (c.head_dim != 128) throw Unsupported("head_dim must be 128");
        if (c.hidden % 128 != 0 || c.intermediate % 128 != 0) throw Unsupported("hidden/intermediate must be multiples of 128");
        if (c.hkv <= 0 || c.hq % c.hkv != 0) throw Unsupported("num_attention_heads must be a multiple of num_key_value_heads");
        const int rep = c.hq / c.hkv;
        if (rep != 1 && rep != 2 && rep != 4) throw Unsupported("GQA ratio must be 1, 2 or 4");
        if ((c.patch * c.in_channels) % 64 != 0) throw Unsupported("patch*in_channels must be a multiple of 64");
        if ((c.patch * c.audio_dim) % 128 != 0) throw Unsupported("patch*audio_dim must be a multiple of 128");

        Loader L(m);
        L.qt = qt;
        m.qtype = qt;
        if (!gguf_path.empty()) {
            L.gguf = true;
            L.gg.open(gguf_path);
        } else {
            L.st.open((root / "model.safetensors").string());
        }
        const int H = c.hidden, I = c.intermediate, D = c.head_dim, P = c.patch, Cin = c.in_channels, A = c.audio_dim;
        const int qd = c.hq * D, kd = c.hkv * D;

        // proj_in: conv1d [H][Cin][P] -> [H][P*Cin] (load_conv1d_weight_as_linear :334-411; GGUF :602-637)
        {
            const Mat w = L.conv_f32("decoder.proj_in.1.weight", H, Cin, P);
            m.proj_in_w = L.finish(Loader::permute(
                                       w, H, (int64_t)P * Cin, [](int64_t r) { return r; },
                                       [&](int64_t col) { return (col % Cin) * P + col / Cin; }),
                                   true);
            m.proj_in_b = L.vec_f32("decoder.proj_in.1.bias", H);
        }
        // proj_out: convtranspose1d [H][A][P] -> [(o + k*A)][H] (load_convtranspose1d_weight_as_linear :413-490;
        // GGUF :639-677)
        {
            const Mat w = L.gguf ? L.conv_f32("decoder.proj_out.1.weight", H, A, P)
                                 : L.mat("decoder.proj_out.1.weight", H, (int64_t)A * P);
            // source element (i, o, k) sits at row i, column o*P + k; target (o + k*A, i)
            Mat wt;
            wt.dtype = w.dtype;
            wt.rows = (int64_t)A * P;
            wt.cols = H;
            if (w.dtype == "F32")
                wt.f32.resize((size_t)wt.rows * H);
            else
                wt.u16.resize((size_t)wt.rows * H);
            for (int i = 0; i < H; ++i)
                for (int o = 0; o < A; ++o)
                    for (int k = 0; k < P; ++k) {
                        const size_t si = ((size_t)i * A + o) * P + k, di = (size_t)(o + k * A) * H + i;
                        if (w.dtype == "F32")
                            wt.f32[di] = w.f32[si];
                        else
                            wt.u16[di] = w.u16[si];
                    }
            m.proj_out_w = L.finish(wt, true);
            m.proj_out_b = L.vec_f32("decoder.proj_out.1.bias", A);
        }
        m.cond_w = L.finish(L.mat("decoder.condition_embedder.weight", H, H));
        m.cond_b = L.vec_f32("decoder.condition_embedder.bias", H);
        m.norm_out = L.vec_f32("decoder.norm_out.weight", H);
        {
            auto ot = L.table("decoder.scale_shift_table", 2, H);
            m.out_table = L.upload<float>(ot.data(), ot.size() * 4);
        }
        const char* tags[2] = {"decoder.time_embed.", "decoder.time_embed_r."};
        for (int e = 0; e < 2; ++e) {
            const std::string p2 = tags[e];
            int64_t fin = 0;
            if (L.gguf) {
                const auto& t1 = L.gg.get(p2 + "linear_1.weight");
                if (t1.ne_at(1) != H || t1.ne_at(2) != 1) throw IoError("invalid tensor shape for " + p2 + "linear_1.weight");
                fin = t1.ne_at(0);
            } else {
                const auto& t1 = L.st.get(p2 + "linear_1.weight");
                if (t1.shape.size() != 2 || t1.shape[0] != H) throw IoError("invalid tensor shape for " + p2 + "linear_1.weight");
                fin = t1.shape[1];
            }
            if (fin != 256) throw Unsupported("timestep embedding input dim must be 256");
            ActType a1, a2, a3;
            m.te[e].w1 = L.finish16(L.mat(p2 + "linear_1.weight", H, fin), a1);
            m.te[e].b1 = L.vec_f32(p2 + "linear_1.bias", H);
            m.te[e].w2 = L.finish16(L.mat(p2 + "linear_2.weight", H, H), a2);
            m.te[e].b2 = L.vec_f32(p2 + "linear_2.bias", H);
            m.te[e].wp = L.finish16(L.mat(p2 + "time_proj.weight", 6LL * H, H), a3);
            m.te[e].bp = L.vec_f32(p2 + "time_proj.bias", 6LL * H);
            if (a1 != a2 || a2 != a3) throw Unsupported("mixed timestep weight types");
            m.te[e].act = a1;
        }
        std::vector<float> tables((size_t)c.layers * 6 * H);
        m.layers.resize(c.layers);
        for (int i = 0; i < c.layers; ++i) {
            const std::string p2 = "decoder.layers." + std::to_string(i) + ".";
            DevLayer& ly = m.layers[i];
            ly.self_norm = L.vec_f32(p2 + "self_attn_norm.weight", H);
            ly.cross_norm = L.vec_f32(p2 + "cross_attn_norm.weight", H);
            ly.mlp_norm = L.vec_f32(p2 + "mlp_norm.weight", H);
            ly.sq_norm = L.vec_f32(p2 + "self_attn.q_norm.weight", D);
            ly.sk_norm = L.vec_f32(p2 + "self_attn.k_norm.weight", D);
            ly.cq_norm = L.vec_f32(p2 + "cross_attn.q_norm.weight", D);
            ly.ck_norm = L.vec_f32(p2 + "cross_attn.k_norm.weight", D);
            {
                const Mat wq = L.mat(p2 + "self_attn.q_proj.weight", qd, H);
                const Mat wk = L.mat(p2 + "self_attn.k_proj.weight", kd, H);
                const Mat wv = L.mat(p2 + "self_attn.v_proj.weight", kd, H);
                ly.w_qkv = L.finish(Loader::concat_rows({&wq, &wk, &wv}));
            }
            ly.w_o = L.finish(L.mat(p2 + "self_attn.o_proj.weight", H, qd));
            ly.w_cq = L.finish(L.mat(p2 + "cross_attn.q_proj.weight", qd, H));
            {
                const Mat wk = L.mat(p2 + "cross_attn.k_proj.weight", kd, H);
                const Mat wv = L.mat(p2 + "cross_attn.v_proj.weight", kd, H);
                ly.w_ckv = L.finish(Loader::concat_rows({&wk, &wv}));
            }
            ly.w_co = L.finish(L.mat(p2 + "cross_attn.o_proj.weight", H, qd));
            ly.w_gu = L.gate_up(p2, I, H);
            ly.w_down = L.finish(L.mat(p2 + "mlp.down_proj.weight", H, I));
            {
                auto v = L.table(p2 + "scale_shift_table", 6, H);
                std::memcpy(&tables[(size_t)i * 6 * H], v.data(), v.size() * 4);
            }
            ly.sliding = i < (int)c.layer_types.size() && c.layer_types[i] == "sliding_attention";
        }
        m.tables = L.upload<float>(tables.data(), tables.size() * 4);

        // ---- condition encoders (optional; acestep_dit_model.cpp:885-996)
        if (L.has("encoder.text_projector.weight")) {
            const auto sh = L.shape2("encoder.text_projector.weight");
            if (sh.first != H) throw IoError("invalid tensor shape for encoder.text_projector.weight");
            m.text_proj = L.finish(L.mat("encoder.text_projector.weight", sh.first, sh.second));
        }
        auto load_encoder = [&](const std::string& pre, int n_layers, DevEncoder& e) {
            if (L.has(pre + "embed_tokens.weight")) {
                const auto sh = L.shape2(pre + "embed_tokens.weight");
                e.embed = L.finish(L.mat(pre + "embed_tokens.weight", sh.first, sh.second));
            }
            if (L.has(pre + "embed_tokens.bias")) e.embed_b = L.vec_f32(pre + "embed_tokens.bias", H);
            if (L.has(pre + "norm.weight")) e.norm = L.vec_f32(pre + "norm.weight", H);
            e.layers.resize(std::max(0, n_layers));
            if (n_layers > 0) {
                const auto sh = L.shape2(pre + "layers.0.mlp.gate_proj.weight");
                if (sh.second != H || sh.first <= 0 || sh.first % 128 != 0)
                    throw Unsupported("encoder MLP width must be a multiple of 128: " + pre);
                e.intermediate = (int)sh.first;
            }
            const int EI = e.intermediate;
            for (int i = 0; i < n_layers; ++i) {  // EncoderLayer (:903-937 / :960-994)
                const std::string p2 = pre + "layers." + std::to_string(i) + ".";
                DevLayer& ly = e.layers[i];
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
                ly.w_gu = L.gate_up(p2, EI, H);
                ly.w_down = L.finish(L.mat(p2 + "mlp.down_proj.weight", H, EI));
                ly.sliding = i < (int)c.layer_types.size() && c.layer_types[i] == "sliding_attention";
            }
            e.act = e.layers.empty() ? ActType::BF16 : e.layers[0].w_qkv.act();
            for (const DevLayer& ly : e.layers)
                for (const DevWeight* w : {&ly.w_qkv, &ly.w_o, &ly.w_gu, &ly.w_down})
                    if (w->act() != e.act) throw Unsupported("mixed encoder block weight types");
        };
        load_encoder("encoder.lyric_encoder.", c.lyric_layers, m.lyric);
        load_encoder("encoder.timbre_encoder.", c.timbre_layers, m.timbre);
        m.act = m.layers.empty() ? m.cond_w.act() : m.layers[0].w_qkv.act();
        for (const DevLayer& ly : m.layers)
            for (const DevWeight* w : {&ly.w_qkv, &ly.w_o, &ly.w_cq, &ly.w_ckv, &ly.w_co, &ly.w_gu, &ly.w_down})
                if (w->act() != m.act) throw Unsupported("mixed DiT block weight types");
        if (m.cond_w.act() != m.act) throw Unsupported("mixed DiT weight types");
        if (m.proj_out_w.fmt != WF_F32X3 && m.proj_out_w.act() != m.act) throw Unsupported("mixed DiT weight types");
    } catch (const Unsupported& e) {
        status_hint = 4;
        throw std::runtime_error(e.what());
    } catch (const HipError&) {
        status_hint = 1;
        throw;
    }
}

}  // namespace acemi
