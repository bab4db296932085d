#include "json.h"

#include <cctype>
#include <cstdlib>
#include <stdexcept>

namespace acemi {
namespace {

struct Parser {
    const std::string& s;
    size_t i = 0;
    explicit Parser(const std::string& t) : s(t) {}

    [[noreturn]] void fail(const char* what) const {
        throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i));
    }
    void ws() {
        while (i < s.size() && std::isspace(static_cast<unsigned char>(s[i]))) ++i;
    }
    bool eat(char c) {
        ws();
        if (i < s.size() && s[i] == c) {
            ++i;
            return true;
        }
        return false;
    }
    void expect(char c) {
        if (!eat(c)) fail("unexpected character");
    }
    static void put_utf8(std::string& o, uint32_t cp) {
        if (cp < 0x80) {
            o += static_cast<char>(cp);
        } else if (cp < 0x800) {
            o += static_cast<char>(0xC0 | (cp >> 6));
            o += static_cast<char>(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
            o += static_cast<char>(0xE0 | (cp >> 12));
            o += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
            o += static_cast<char>(0x80 | (cp & 0x3F));
        } else {
            o += static_cast<char>(0xF0 | (cp >> 18));
            o += static_cast<char>(0x80 | ((cp >> 12) & 0x3F));
            o += static_cast<char>(0x80 | ((cp >> 6) & 0x3F));
            o += static_cast<char>(0x80 | (cp & 0x3F));
        }
    }
    std::string string_body() {
        std::string o;
        while (true) {
            if (i >= s.size()) fail("unterminated string");
            char c = s[i++];
            if (c == '"') break;
            if (c != '\\') {
                o += c;
                continue;
            }
            if (i >= s.size()) fail("bad escape");
            char e = s[i++];
            switch (e) {
                case '"': o += '"'; break;
                case '\\': o += '\\'; break;
                case '/': o += '/'; break;
                case 'b': o += '\b'; break;
                case 'f': o += '\f'; break;
                case 'n': o += '\n'; break;
                case 'r': o += '\r'; break;
                case 't': o += '\t'; break;
                case 'u': {
                    if (i + 4 > s.size()) fail("bad \\u escape");
                    uint32_t cp = static_cast<uint32_t>(std::strtoul(s.substr(i, 4).c_str(), nullptr, 16));
                    i += 4;
                    put_utf8(o, cp);
                    break;
                }
                default: fail("bad escape");
            }
        }
        return o;
    }
    Json value() {
        ws();
        if (i >= s.size()) fail("unexpected end");
        Json v;
        char c = s[i];
        if (c == '{') {
            ++i;
            v.kind = Json::Object;
            if (eat('}')) return v;
            do {
                ws();
                expect('"');
                std::string k = string_body();
                expect(':');
                v.obj[k] = value();
            } while (eat(','));
            expect('}');
        } else if (c == '[') {
            ++i;
            v.kind = Json::Array;
            if (eat(']')) return v;
            do {
                v.arr.push_back(value());
            } while (eat(','));
            expect(']');
        } else if (c == '"') {
            ++i;
            v.kind = Json::String;
            v.str = string_body();
        } else if (s.compare(i, 4, "true") == 0) {
            i += 4;
            v.kind = Json::Bool;
            v.b = true;
        } else if (s.compare(i, 5, "false") == 0) {
            i += 5;
            v.kind = Json::Bool;
        } else if (s.compare(i, 4, "null") == 0) {
            i += 4;
        } else {
            const char* start = s.c_str() + i;
            char* end = nullptr;
            v.num = std::strtod(start, &end);
            if (end == start) fail("bad number");
            i += static_cast<size_t>(end - start);
            v.kind = Json::Number;
        }
        return v;
    }
};

}  // namespace

Json Json::parse(const std::string& text) {
    Parser p(text);
    Json v = p.value();
    p.ws();
    if (p.i != text.size()) p.fail("trailing characters");
    return v;
}

const Json& Json::at(const std::string& k) const {
    auto it = obj.find(k);
    if (kind != Object || it == obj.end()) throw std::runtime_error("json: missing key " + k);
    return it->second;
}

int64_t Json::as_int() const {
    if (kind == Number) return static_cast<int64_t>(num);
    if (kind == Bool) return b ? 1 : 0;
    throw std::runtime_error("json: not a number");
}

double Json::as_num() const {
    if (kind == Number) return num;
    throw std::runtime_error("json: not a number");
}

const std::string& Json::as_str() const {
    if (kind != String) throw std::runtime_error("json: not a string");
    return str;
}

bool Json::as_bool() const {
    if (kind == Bool) return b;
    if (kind == Number) return num != 0.0;
    throw std::runtime_error("json: not a bool");
}

}  // namespace acemi
