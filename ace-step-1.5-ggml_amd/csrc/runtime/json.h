// Minimal JSON value + recursive-descent parser (config.json and safetensors headers).
// Plays the role of the reference's ace_json (acestep_ggml/cpp/json_min.{h,cpp}).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace acemi {

struct Json {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0.0;
    std::string str;
    std::vector<Json> arr;
    std::map<std::string, Json> obj;

    static Json parse(const std::string& text);  // throws std::runtime_error

    bool has(const std::string& k) const { return kind == Object && obj.count(k) != 0; }
    const Json& at(const std::string& k) const;
    int64_t as_int() const;
    double as_num() const;
    const std::string& as_str() const;
    bool as_bool() const;
};

}  // namespace acemi
