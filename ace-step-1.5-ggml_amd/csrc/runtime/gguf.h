// Minimal GGUF (v2/v3) reader for the DiT loader: tensor directory + raw tensor bytes.
//
// Replaces the reference's gguf_init_from_file use in acestep_dit_model.cpp:71-97 (files written by
// acestep_ggml/tools/export_safetensors_to_gguf.py:154-281 with llama.cpp's GGUFWriter).  Layout:
// "GGUF", u32 version, u64 n_tensors, u64 n_kv, n_kv x {string key, u32 type, value}, n_tensors x
// {string name, u32 n_dims, u64 ne[n_dims], u32 ggml_type, u64 offset}, padding to
// general.alignment (default 32), tensor data (offsets relative to the data start).
// Strings are u64 length + bytes.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace acemi {

enum GgmlType : int {
    GGML_F32 = 0,
    GGML_F16 = 1,
    GGML_Q8_0 = 8,
    GGML_Q4_K = 12,
    GGML_Q6_K = 14,
    GGML_BF16 = 30,
};

struct GgufTensor {
    std::string name;
    std::vector<int64_t> ne;  // ggml order: ne[0] = innermost (row length)
    int type = 0;
    uint64_t offset = 0;      // from the data section start
    uint64_t nbytes = 0;
    int64_t ne_at(int i) const { return i < (int)ne.size() ? ne[i] : 1; }
};

struct GgufFile {
    std::string path;
    uint32_t version = 0;
    uint64_t data_offset = 0;
    uint32_t alignment = 32;
    std::map<std::string, GgufTensor> tensors;
    std::map<std::string, std::string> strings;  // string-valued metadata (e.g. general.architecture)

    void open(const std::string& path);  // throws std::runtime_error
    bool has(const std::string& n) const { return tensors.count(n) != 0; }
    const GgufTensor& get(const std::string& n) const;
    std::vector<uint8_t> read(const GgufTensor& t) const;
};

// bytes of one row of `ne0` values (block formats: ne0 % block == 0); 0 for unsupported types
uint64_t ggml_row_bytes(int type, int64_t ne0);
const char* ggml_type_name(int type);

}  // namespace acemi
