// json.h — minimal JSON reader for the .xalm header (the reference vendors nlohmann/json,
// 3rdparty/json.hpp; the header written by convert.py uses objects, arrays, strings,
// integers and floats only).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace xalm {

struct Json {
    enum Kind { Null, Bool, Number, String, Array, Object } kind = Null;
    bool b = false;
    double num = 0;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;  // insertion order kept

    const Json* find(const std::string& k) const {
        for (auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    const Json& at(const std::string& k) const {
        const Json* j = find(k);
        if (!j) throw std::out_of_range("json: missing key '" + k + "'");
        return *j;
    }
    bool contains(const std::string& k) const { return find(k) != nullptr; }
    const std::string& as_string() const {
        if (kind != String) throw std::invalid_argument("json: not a string");
        return str;
    }
    long long as_int() const {
        if (kind != Number) throw std::invalid_argument("json: not a number");
        return (long long)num;
    }

    static Json parse(const std::string& s) {
        size_t i = 0;
        Json j = parse_value(s, i);
        skip_ws(s, i);
        if (i != s.size()) throw std::invalid_argument("json: trailing characters");
        return j;
    }

private:
    static void skip_ws(const std::string& s, size_t& i) {
        while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\r' || s[i] == '\t')) i++;
    }
    static void expect(const std::string& s, size_t& i, char c) {
        skip_ws(s, i);
        if (i >= s.size() || s[i] != c) throw std::invalid_argument(std::string("json: expected '") + c + "'");
        i++;
    }
    static void put_utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) out += (char)cp;
        else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
        else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
        } else {
            out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
            out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
        }
    }
    static uint32_t hex4(const std::string& s, size_t& i) {
        if (i + 4 > s.size()) throw std::invalid_argument("json: bad \\u escape");
        uint32_t v = (uint32_t)std::stoul(s.substr(i, 4), nullptr, 16);
        i += 4;
        return v;
    }
    static std::string parse_string(const std::string& s, size_t& i) {
        expect(s, i, '"');
        std::string out;
        while (i < s.size() && s[i] != '"') {
            char c = s[i++];
            if (c != '\\') { out += c; continue; }
            if (i >= s.size()) break;
            char e = s[i++];
            switch (e) {
                case 'n': out += '\n'; break;
                case 't': out += '\t'; break;
                case 'r': out += '\r'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'u': {
                    uint32_t cp = hex4(s, i);
                    if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
                        i += 2;
                        uint32_t lo = hex4(s, i);
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    put_utf8(out, cp);
                    break;
                }
                default: out += e; break;
            }
        }
        if (i >= s.size()) throw std::invalid_argument("json: unterminated string");
        i++;
        return out;
    }
    static Json parse_value(const std::string& s, size_t& i) {
        skip_ws(s, i);
        if (i >= s.size()) throw std::invalid_argument("json: unexpected end");
        Json j;
        const char c = s[i];
        if (c == '{') {
            j.kind = Object;
            i++;
            skip_ws(s, i);
            if (i < s.size() && s[i] == '}') { i++; return j; }
            for (;;) {
                std::string k = parse_string(s, i);
                expect(s, i, ':');
                j.obj.emplace_back(std::move(k), parse_value(s, i));
                skip_ws(s, i);
                if (i < s.size() && s[i] == ',') { i++; continue; }
                expect(s, i, '}');
                return j;
            }
        }
        if (c == '[') {
            j.kind = Array;
            i++;
            skip_ws(s, i);
            if (i < s.size() && s[i] == ']') { i++; return j; }
            for (;;) {
                j.arr.push_back(parse_value(s, i));
                skip_ws(s, i);
                if (i < s.size() && s[i] == ',') { i++; continue; }
                expect(s, i, ']');
                return j;
            }
        }
        if (c == '"') { j.kind = String; j.str = parse_string(s, i); return j; }
        if (s.compare(i, 4, "true") == 0) { j.kind = Bool; j.b = true; i += 4; return j; }
        if (s.compare(i, 5, "false") == 0) { j.kind = Bool; i += 5; return j; }
        if (s.compare(i, 4, "null") == 0) { i += 4; return j; }
        size_t end = i;
        while (end < s.size() && (isdigit((unsigned char)s[end]) || s[end] == '-' || s[end] == '+' || s[end] == '.' ||
                                  s[end] == 'e' || s[end] == 'E'))
            end++;
        if (end == i) throw std::invalid_argument("json: bad value");
        j.kind = Number;
        j.num = std::stod(s.substr(i, end - i));
        i = end;
        return j;
    }
};

}  // namespace xalm
