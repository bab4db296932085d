// GGUF reader (see gguf.h).
#include "gguf.h"

#include <fstream>
#include <stdexcept>

namespace acemi {
namespace {

enum GgufValueType : uint32_t {
    GV_UINT8 = 0, GV_INT8 = 1, GV_UINT16 = 2, GV_INT16 = 3, GV_UINT32 = 4, GV_INT32 = 5, GV_FLOAT32 = 6,
    GV_BOOL = 7, GV_STRING = 8, GV_ARRAY = 9, GV_UINT64 = 10, GV_INT64 = 11, GV_FLOAT64 = 12,
};

struct Reader {
    std::ifstream in;
    std::string path;
    template <typename T>
    T get() {
        T v{};
        if (!in.read(reinterpret_cast<char*>(&v), sizeof(T))) throw std::runtime_error("gguf: truncated file " + path);
        return v;
    }
    std::string str() {
        const uint64_t n = get<uint64_t>();
        if (n > (1ull << 30)) throw std::runtime_error("gguf: invalid string length in " + path);
        std::string s(n, '\0');
        if (n && !in.read(s.data(), (std::streamsize)n)) throw std::runtime_error("gguf: truncated file " + path);
        return s;
    }
    void skip(uint64_t n) { in.seekg((std::streamoff)n, std::ios::cur); }
    size_t scalar_size(uint32_t t) {
        switch (t) {
            case GV_UINT8: case GV_INT8: case GV_BOOL: return 1;
            case GV_UINT16: case GV_INT16: return 2;
            case GV_UINT32: case GV_INT32: case GV_FLOAT32: return 4;
            case GV_UINT64: case GV_INT64: case GV_FLOAT64: return 8;
            default: return 0;
        }
    }
    // returns the value as uint64 for integer scalars (used for general.alignment), stores strings
    uint64_t value(uint32_t t, std::string* sval) {
        if (t == GV_STRING) {
            std::string s = str();
            if (sval) *sval = s;
            return 0;
        }
        if (t == GV_ARRAY) {
            const uint32_t et = get<uint32_t>();
            const uint64_t n = get<uint64_t>();
            if (et == GV_STRING) {
                for (uint64_t i = 0; i < n; ++i) (void)str();
            } else if (et == GV_ARRAY) {
                for (uint64_t i = 0; i < n; ++i) (void)value(GV_ARRAY, nullptr);
            } else {
                const size_t sz = scalar_size(et);
                if (!sz) throw std::runtime_error("gguf: bad array element type in " + path);
                skip(n * sz);
            }
            return 0;
        }
        switch (t) {
            case GV_UINT8: return get<uint8_t>();
            case GV_INT8: return (uint64_t)(int64_t)get<int8_t>();
            case GV_BOOL: return get<uint8_t>();
            case GV_UINT16: return get<uint16_t>();
            case GV_INT16: return (uint64_t)(int64_t)get<int16_t>();
            case GV_UINT32: return get<uint32_t>();
            case GV_INT32: return (uint64_t)(int64_t)get<int32_t>();
            case GV_FLOAT32: (void)get<float>(); return 0;
            case GV_UINT64: return get<uint64_t>();
            case GV_INT64: return (uint64_t)get<int64_t>();
            case GV_FLOAT64: (void)get<double>(); return 0;
            default: throw std::runtime_error("gguf: bad metadata value type in " + path);
        }
    }
};

}  // namespace

uint64_t ggml_row_bytes(int type, int64_t ne0) {
    switch (type) {
        case GGML_F32: return (uint64_t)ne0 * 4;
        case GGML_F16:
        case GGML_BF16: return (uint64_t)ne0 * 2;
        case GGML_Q8_0: return ne0 % 32 ? 0 : (uint64_t)(ne0 / 32) * 34;
        case GGML_Q4_K: return ne0 % 256 ? 0 : (uint64_t)(ne0 / 256) * 144;
        case GGML_Q6_K: return ne0 % 256 ? 0 : (uint64_t)(ne0 / 256) * 210;
        default: return 0;
    }
}

const char* ggml_type_name(int type) {
    switch (type) {
        case GGML_F32: return "f32";
        case GGML_F16: return "f16";
        case GGML_BF16: return "bf16";
        case GGML_Q8_0: return "q8_0";
        case GGML_Q4_K: return "q4_K";
        case GGML_Q6_K: return "q6_K";
        default: return "unsupported";
    }
}

void GgufFile::open(const std::string& p) {
    path = p;
    Reader r;
    r.path = p;
    r.in.open(p, std::ios::binary);
    if (!r.in) throw std::runtime_error("failed to load gguf file: " + p);
    char magic[4];
    if (!r.in.read(magic, 4) || magic[0] != 'G' || magic[1] != 'G' || magic[2] != 'U' || magic[3] != 'F')
        throw std::runtime_error("failed to load gguf file: " + p + " (bad magic)");
    version = r.get<uint32_t>();
    if (version < 2 || version > 3) throw std::runtime_error("failed to load gguf file: " + p + " (unsupported version)");
    const uint64_t n_tensors = r.get<uint64_t>();
    const uint64_t n_kv = r.get<uint64_t>();
    if (n_tensors > (1u << 24) || n_kv > (1u << 24)) throw std::runtime_error("gguf: implausible header in " + p);
    for (uint64_t i = 0; i < n_kv; ++i) {
        const std::string key = r.str();
        const uint32_t t = r.get<uint32_t>();
        std::string sval;
        const uint64_t v = r.value(t, &sval);
        if (t == GV_STRING) strings[key] = sval;
        if (key == "general.alignment" && t != GV_STRING && t != GV_ARRAY) {
            if (v == 0 || (v & (v - 1)) != 0) throw std::runtime_error("gguf: invalid alignment in " + p);
            alignment = (uint32_t)v;
        }
    }
    std::vector<GgufTensor> list;
    for (uint64_t i = 0; i < n_tensors; ++i) {
        GgufTensor t;
        t.name = r.str();
        const uint32_t nd = r.get<uint32_t>();
        if (nd > 4) throw std::runtime_error("gguf: tensor rank > 4 in " + p);
        int64_t n = 1;
        for (uint32_t d = 0; d < nd; ++d) {
            t.ne.push_back((int64_t)r.get<uint64_t>());
            if (t.ne.back() < 0) throw std::runtime_error("gguf: negative dim in " + p);
        }
        t.type = (int)r.get<uint32_t>();
        t.offset = r.get<uint64_t>();
        for (size_t d = 1; d < t.ne.size(); ++d) n *= t.ne[d];
        const uint64_t rb = ggml_row_bytes(t.type, t.ne_at(0));
        t.nbytes = rb * (uint64_t)n;  // 0 for unsupported types: rejected at use
        list.push_back(t);
    }
    const uint64_t pos = (uint64_t)r.in.tellg();
    data_offset = (pos + alignment - 1) / alignment * alignment;
    r.in.seekg(0, std::ios::end);
    const uint64_t fsize = (uint64_t)r.in.tellg();
    for (auto& t : list) {
        if (t.nbytes && data_offset + t.offset + t.nbytes > fsize)
            throw std::runtime_error("gguf: tensor data out of range: " + t.name);
        tensors[t.name] = t;
    }
}

const GgufTensor& GgufFile::get(const std::string& n) const {
    auto it = tensors.find(n);
    if (it == tensors.end()) throw std::runtime_error("missing tensor in gguf: " + n);
    return it->second;
}

std::vector<uint8_t> GgufFile::read(const GgufTensor& t) const {
    if (!t.nbytes) throw std::runtime_error(std::string("unsupported gguf tensor type ") + ggml_type_name(t.type) + ": " + t.name);
    std::vector<uint8_t> buf(t.nbytes);
    std::ifstream in(path, std::ios::binary);
    in.seekg((std::streamoff)(data_offset + t.offset));
    if (!in || !in.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)buf.size()))
        throw std::runtime_error("invalid tensor data size in gguf: " + t.name);
    return buf;
}

}  // namespace acemi
