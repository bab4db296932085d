// safetensors reader shared by the DiT and VAE loaders.
// Same contract as ace_safetensors::File (acestep_ggml/cpp/safetensors.cpp:46-171): u64 little-endian
// header length, JSON header {name: {dtype, shape, data_offsets}}, then the data.
#pragma once

#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "json.h"

namespace acemi {

struct IoError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct Unsupported : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline std::string read_file(const std::string& path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) throw IoError("failed to read " + path);
    std::ostringstream ss;
    ss << in.rdbuf();
    return ss.str();
}

// ------------------------------------------------------------ safetensors
// Format: u64 little-endian header length, JSON header {name: {dtype, shape, data_offsets}}, data.
// Same contract as ace_safetensors::File (acestep_ggml/cpp/safetensors.cpp:46-171).
struct StTensor {
    std::string dtype;
    std::vector<int64_t> shape;
    uint64_t begin = 0, end = 0;
    int64_t numel() const {
        int64_t n = 1;
        for (auto d : shape) n *= d;
        return n;
    }
    // bytes per element of the dtypes the loaders read; 0 for any other dtype (left to the caller,
    // which raises Unsupported for it)
    size_t elem_size() const {
        if (dtype == "F32" || dtype == "I32") return 4;
        if (dtype == "BF16" || dtype == "F16" || dtype == "I16") return 2;
        if (dtype == "I8" || dtype == "U8") return 1;
        if (dtype == "F64" || dtype == "I64") return 8;
        return 0;
    }
};

struct StFile {
    std::string path;
    uint64_t data_offset = 0;
    std::map<std::string, StTensor> tensors;

    void open(const std::string& p) {
        path = p;
        std::ifstream in(p, std::ios::binary);
        if (!in) throw IoError("failed to open " + p);
        in.seekg(0, std::ios::end);
        const uint64_t file_size = static_cast<uint64_t>(in.tellg());
        in.seekg(0, std::ios::beg);
        uint64_t hlen = 0;
        unsigned char b8[8];
        if (!in.read(reinterpret_cast<char*>(b8), 8)) throw IoError("failed to read header size");
        for (int i = 7; i >= 0; --i) hlen = (hlen << 8) | b8[i];
        if (hlen > (1ull << 31)) throw IoError("invalid safetensors header size");
        std::string header(hlen, '\0');
        if (!in.read(header.data(), static_cast<std::streamsize>(hlen))) throw IoError("failed to read header");
        data_offset = 8 + hlen;
        Json root;
        try {
            root = Json::parse(header);
        } catch (const std::exception& e) {
            throw IoError(std::string("invalid safetensors header: ") + e.what());
        }
        if (root.kind != Json::Object) throw IoError("invalid safetensors header");
        for (const auto& kv : root.obj) {
            if (kv.first == "__metadata__") continue;
            StTensor t;
            t.dtype = kv.second.at("dtype").as_str();
            for (const auto& d : kv.second.at("shape").arr) t.shape.push_back(d.as_int());
            const auto& off = kv.second.at("data_offsets").arr;
            if (off.size() != 2) throw IoError("data_offsets invalid");
            const int64_t b = off[0].as_int(), e = off[1].as_int();
            // the reference sizes every read from the shape and rejects a mismatch
            // (safetensors.cpp TensorInfo::nbytes / read_tensor); reject it here, at open, so no
            // later read or conversion can run past the tensor's bytes
            if (b < 0 || e < b) throw IoError("invalid data_offsets for tensor: " + kv.first);
            t.begin = static_cast<uint64_t>(b);
            t.end = static_cast<uint64_t>(e);
            if (data_offset + t.end > file_size) throw IoError("tensor data out of file bounds: " + kv.first);
            for (auto d : t.shape)
                if (d < 0) throw IoError("invalid shape for tensor: " + kv.first);
            const size_t es = t.elem_size();
            if (es != 0 && static_cast<uint64_t>(t.numel()) * es != t.end - t.begin)
                throw IoError("tensor byte size mismatch: " + kv.first);
            tensors[kv.first] = t;
        }
    }
    bool has(const std::string& n) const { return tensors.count(n) != 0; }
    const StTensor& get(const std::string& n) const {
        auto it = tensors.find(n);
        if (it == tensors.end()) throw IoError("missing tensor: " + n);
        return it->second;
    }
    std::vector<uint8_t> read(const StTensor& t) const {
        std::vector<uint8_t> buf(t.end - t.begin);
        std::ifstream in(path, std::ios::binary);
        in.seekg(static_cast<std::streamoff>(data_offset + t.begin));
        if (!in || !in.read(reinterpret_cast<char*>(buf.data()), static_cast<std::streamsize>(buf.size())))
            throw IoError("read failed");
        return buf;
    }
};

inline float half_to_f32(uint16_t h) {
    const uint32_t s = (h >> 15) & 1u, e = (h >> 10) & 31u, f = h & 1023u;
    uint32_t out;
    if (e == 0) {
        if (f == 0) {
            out = s << 31;
        } else {  // subnormal
            int ee = -1;
            uint32_t ff = f;
            do {
                ++ee;
                ff <<= 1;
            } while ((ff & 1024u) == 0);
            out = (s << 31) | ((127 - 15 - ee) << 23) | ((ff & 1023u) << 13);
        }
    } else if (e == 31) {
        out = (s << 31) | 0x7f800000u | (f << 13);
    } else {
        out = (s << 31) | ((e - 15 + 127) << 23) | (f << 13);
    }
    float r;
    std::memcpy(&r, &out, 4);
    return r;
}

inline std::vector<float> to_f32(const StTensor& t, const std::vector<uint8_t>& raw) {
    const int64_t n = t.numel();
    std::vector<float> out(static_cast<size_t>(n));
    if (t.dtype == "F32") {
        std::memcpy(out.data(), raw.data(), static_cast<size_t>(n) * 4);
    } else if (t.dtype == "BF16") {
        const uint16_t* s = reinterpret_cast<const uint16_t*>(raw.data());
        for (int64_t i = 0; i < n; ++i) {
            uint32_t u = static_cast<uint32_t>(s[i]) << 16;
            std::memcpy(&out[static_cast<size_t>(i)], &u, 4);
        }
    } else if (t.dtype == "F16") {
        const uint16_t* s = reinterpret_cast<const uint16_t*>(raw.data());
        for (int64_t i = 0; i < n; ++i) out[static_cast<size_t>(i)] = half_to_f32(s[i]);
    } else {
        throw Unsupported("unsupported dtype: " + t.dtype);
    }
    return out;
}

}  // namespace acemi
