// Minimal JSON DOM + recursive-descent parser for scene files.
// Stand-in for rapidjson, which the reference parser uses
// (src/runtime/loader/Parser.cpp); accepts the subset scene files use,
// plus '//' line comments which Ignis scene files sometimes carry.
#pragma once

#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace igx::json {

struct Value {
    enum Type { Null, Bool, Number, String, Array, Object } type = Null;
    bool b = false;
    double num = 0;
    std::string str;
    std::vector<Value> arr;
    std::vector<std::pair<std::string, Value>> obj; // keeps file order

    bool is_null() const { return type == Null; }
    bool is_number() const { return type == Number; }
    bool is_string() const { return type == String; }
    bool is_array() const { return type == Array; }
    bool is_object() const { return type == Object; }
    bool is_bool() const { return type == Bool; }

    const Value* find(const std::string& key) const {
        if (type != Object) return nullptr;
        for (auto& kv : obj)
            if (kv.first == key) return &kv.second;
        return nullptr;
    }
};

class Parser {
public:
    explicit Parser(const std::string& s) : s_(s) {}
    Value parse() {
        skip();
        Value v = value();
        skip();
        if (p_ != s_.size()) fail("trailing characters");
        return v;
    }

private:
    const std::string& s_;
    size_t p_ = 0;

    [[noreturn]] void fail(const std::string& what) {
        size_t line = 1;
        for (size_t i = 0; i < p_ && i < s_.size(); ++i)
            if (s_[i] == '\n') ++line;
        throw std::runtime_error("JSON parse error at line " + std::to_string(line) + ": " + what);
    }
    void skip() {
        while (p_ < s_.size()) {
            char c = s_[p_];
            if (c == ' ' || c == '\t' || c == '\n' || c == '\r') {
                ++p_;
            } else if (c == '/' && p_ + 1 < s_.size() && s_[p_ + 1] == '/') {
                while (p_ < s_.size() && s_[p_] != '\n') ++p_;
            } else if (c == '/' && p_ + 1 < s_.size() && s_[p_ + 1] == '*') {
                p_ += 2;
                while (p_ + 1 < s_.size() && !(s_[p_] == '*' && s_[p_ + 1] == '/')) ++p_;
                p_ += 2;
            } else {
                break;
            }
        }
    }
    Value value() {
        if (p_ >= s_.size()) fail("unexpected end");
        char c = s_[p_];
        if (c == '{') return object();
        if (c == '[') return array();
        if (c == '"') { Value v; v.type = Value::String; v.str = string(); return v; }
        if (c == 't' || c == 'f') return boolean();
        if (c == 'n') { expect("null"); return Value(); }
        return number();
    }
    void expect(const char* lit) {
        for (const char* q = lit; *q; ++q, ++p_)
            if (p_ >= s_.size() || s_[p_] != *q) fail(std::string("expected ") + lit);
    }
    Value boolean() {
        Value v; v.type = Value::Bool;
        if (s_[p_] == 't') { expect("true"); v.b = true; } else { expect("false"); v.b = false; }
        return v;
    }
    Value number() {
        const char* start = s_.c_str() + p_;
        char* end = nullptr;
        double d = std::strtod(start, &end);
        if (end == start) fail("invalid value");
        p_ += (size_t)(end - start);
        Value v; v.type = Value::Number; v.num = d;
        return v;
    }
    std::string string() {
        ++p_; // opening quote
        std::string out;
        while (p_ < s_.size() && s_[p_] != '"') {
            char c = s_[p_++];
            if (c == '\\') {
                if (p_ >= s_.size()) fail("bad escape");
                char e = s_[p_++];
                switch (e) {
                case 'n': out += '\n'; break;
                case 't': out += '\t'; break;
                case 'r': out += '\r'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'u': {
                    unsigned cp = (unsigned)std::strtoul(s_.substr(p_, 4).c_str(), nullptr, 16);
                    p_ += 4;
                    if (cp < 0x80) out += (char)cp;
                    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
                    else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
                    break;
                }
                default: out += e;
                }
            } else {
                out += c;
            }
        }
        if (p_ >= s_.size()) fail("unterminated string");
        ++p_;
        return out;
    }
    Value array() {
        Value v; v.type = Value::Array;
        ++p_;
        skip();
        if (p_ < s_.size() && s_[p_] == ']') { ++p_; return v; }
        for (;;) {
            skip();
            v.arr.push_back(value());
            skip();
            if (p_ >= s_.size()) fail("unterminated array");
            if (s_[p_] == ',') { ++p_; skip(); if (p_ < s_.size() && s_[p_] == ']') { ++p_; return v; } continue; }
            if (s_[p_] == ']') { ++p_; return v; }
            fail("expected , or ]");
        }
    }
    Value object() {
        Value v; v.type = Value::Object;
        ++p_;
        skip();
        if (p_ < s_.size() && s_[p_] == '}') { ++p_; return v; }
        for (;;) {
            skip();
            if (p_ >= s_.size() || s_[p_] != '"') fail("expected key");
            std::string key = string();
            skip();
            if (p_ >= s_.size() || s_[p_] != ':') fail("expected :");
            ++p_;
            skip();
            v.obj.emplace_back(std::move(key), value());
            skip();
            if (p_ >= s_.size()) fail("unterminated object");
            if (s_[p_] == ',') { ++p_; skip(); if (p_ < s_.size() && s_[p_] == '}') { ++p_; return v; } continue; }
            if (s_[p_] == '}') { ++p_; return v; }
            fail("expected , or }");
        }
    }
};

inline Value parse(const std::string& s) { return Parser(s).parse(); }

} // namespace igx::json
