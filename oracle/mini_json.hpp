// oracle/mini_json.hpp -- TEST INFRASTRUCTURE (oracle). Not part of the product.
//
// Minimal JSON DOM with the conversion semantics the reference relies on from its vendored
// nlohmann/json 3.12.0 (/root/reference/Code/json.hpp):
//   * integer tokens -> int64 (leading '-') / uint64, overflow falls back to double
//     (lexer, json.hpp:7987-7989, 8357 -- numbers go through strtoll/strtoull/strtod);
//   * get<float>/get<int> = static_cast of the stored int64/uint64/double/bool
//     (from_json for arithmetic types, json.hpp:5229-5262): decimal -> double -> float,
//     never strtof, and 36.0 -> 36 for int;
//   * get<array<float,3>> reads .at(0..2) (json.hpp:5166-5181), so short arrays and
//     non-arrays throw; value(key, def) throws on non-objects (json.hpp:22357-22373);
//   * duplicate object keys: the last one wins (DOM parser operator[] assignment).
#pragma once
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace oj {

struct error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct Value {
  enum Kind { Null, Bool, Int, Uint, Dbl, Str, Arr, Obj } kind = Null;
  bool b = false;
  int64_t i = 0;
  uint64_t u = 0;
  double d = 0;
  std::string s;
  std::vector<Value> a;
  std::map<std::string, Value> o;

  bool is_object() const { return kind == Obj; }
  bool is_array() const { return kind == Arr; }
  bool is_number() const { return kind == Int || kind == Uint || kind == Dbl; }
  bool contains(const std::string& k) const { return kind == Obj && o.count(k) != 0; }
  size_t size() const { return kind == Arr ? a.size() : kind == Obj ? o.size() : (kind == Null ? 0 : 1); }
  // nlohmann empty(): null -> true, array/object -> no elements, scalars -> false
  bool empty() const { return kind == Null || (kind == Arr && a.empty()) || (kind == Obj && o.empty()); }

  const Value& at(size_t idx) const {
    if (kind != Arr) throw error("type_error.304: cannot use at() with non-array");
    if (idx >= a.size()) throw error("out_of_range.401: array index out of range");
    return a[idx];
  }
  const Value& at(const std::string& k) const {
    if (kind != Obj) throw error("type_error.304: cannot use at() with non-object");
    auto it = o.find(k);
    if (it == o.end()) throw error("out_of_range.403: key not found");
    return it->second;
  }
  template <class T>
  T num() const {
    switch (kind) {
      case Uint: return static_cast<T>(u);
      case Int: return static_cast<T>(i);
      case Dbl: return static_cast<T>(d);
      case Bool: return static_cast<T>(b);
      default: throw error("type_error.302: type must be number");
    }
  }
  float get_float() const { return num<float>(); }
  int get_int() const { return num<int>(); }
  void get_vec3(float out[3]) const {
    for (int k = 0; k < 3; ++k) out[k] = at((size_t)k).get_float();
  }
  std::string get_string() const {
    if (kind != Str) throw error("type_error.302: type must be string");
    return s;
  }
  float value_float(const std::string& k, float def) const {
    if (kind != Obj) throw error("type_error.306: cannot use value() with non-object");
    auto it = o.find(k);
    return it == o.end() ? def : it->second.get_float();
  }
};

class Parser {
 public:
  explicit Parser(const std::string& text) : t_(text) {}
  Value parse() {
    Value v = value();
    ws();
    if (p_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  const std::string& t_;
  size_t p_ = 0;
  [[noreturn]] void fail(const char* m) { throw error(std::string("parse_error: ") + m + " at byte " + std::to_string(p_)); }
  void ws() {
    while (p_ < t_.size() && (t_[p_] == ' ' || t_[p_] == '\t' || t_[p_] == '\n' || t_[p_] == '\r')) ++p_;
  }
  bool lit(const char* w) {
    size_t n = 0;
    while (w[n]) ++n;
    if (t_.compare(p_, n, w) == 0) { p_ += n; return true; }
    return false;
  }
  Value value() {
    ws();
    if (p_ >= t_.size()) fail("unexpected end");
    char c = t_[p_];
    Value v;
    if (c == '{') {
      ++p_;
      v.kind = Value::Obj;
      ws();
      if (p_ < t_.size() && t_[p_] == '}') { ++p_; return v; }
      for (;;) {
        ws();
        if (p_ >= t_.size() || t_[p_] != '"') fail("expected key");
        std::string k = str();
        ws();
        if (p_ >= t_.size() || t_[p_] != ':') fail("expected ':'");
        ++p_;
        v.o[k] = value();
        ws();
        if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
        if (p_ < t_.size() && t_[p_] == '}') { ++p_; return v; }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++p_;
      v.kind = Value::Arr;
      ws();
      if (p_ < t_.size() && t_[p_] == ']') { ++p_; return v; }
      for (;;) {
        v.a.push_back(value());
        ws();
        if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
        if (p_ < t_.size() && t_[p_] == ']') { ++p_; return v; }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') { v.kind = Value::Str; v.s = str(); return v; }
    if (lit("true")) { v.kind = Value::Bool; v.b = true; return v; }
    if (lit("false")) { v.kind = Value::Bool; v.b = false; return v; }
    if (lit("null")) return v;
    return number();
  }
  std::string str() {
    ++p_;  // opening quote
    std::string out;
    while (p_ < t_.size() && t_[p_] != '"') {
      char c = t_[p_++];
      if (c == '\\') {
        if (p_ >= t_.size()) fail("bad escape");
        char e = t_[p_++];
        switch (e) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            if (p_ + 4 > t_.size()) fail("bad \\u");
            unsigned cp = (unsigned)std::strtoul(t_.substr(p_, 4).c_str(), nullptr, 16);
            p_ += 4;
            if (cp < 0x80) out += (char)cp;
            else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
            else { out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F)); }
            break;
          }
          default: fail("bad escape");
        }
      } else {
        out += c;
      }
    }
    if (p_ >= t_.size()) fail("unterminated string");
    ++p_;
    return out;
  }
  Value number() {
    size_t b = p_;
    bool is_float = false;
    if (t_[p_] == '-') ++p_;
    if (p_ >= t_.size()) fail("bad number");
    if (t_[p_] == '0') ++p_;
    else if (t_[p_] >= '1' && t_[p_] <= '9') { while (p_ < t_.size() && isdig(t_[p_])) ++p_; }
    else fail("bad number");
    if (p_ < t_.size() && t_[p_] == '.') {
      is_float = true; ++p_;
      if (p_ >= t_.size() || !isdig(t_[p_])) fail("bad fraction");
      while (p_ < t_.size() && isdig(t_[p_])) ++p_;
    }
    if (p_ < t_.size() && (t_[p_] == 'e' || t_[p_] == 'E')) {
      is_float = true; ++p_;
      if (p_ < t_.size() && (t_[p_] == '+' || t_[p_] == '-')) ++p_;
      if (p_ >= t_.size() || !isdig(t_[p_])) fail("bad exponent");
      while (p_ < t_.size() && isdig(t_[p_])) ++p_;
    }
    std::string tok = t_.substr(b, p_ - b);
    Value v;
    if (!is_float) {
      errno = 0;
      if (tok[0] == '-') {
        long long x = std::strtoll(tok.c_str(), nullptr, 10);
        if (errno == 0) { v.kind = Value::Int; v.i = x; return v; }
      } else {
        unsigned long long x = std::strtoull(tok.c_str(), nullptr, 10);
        if (errno == 0) { v.kind = Value::Uint; v.u = x; return v; }
      }
    }
    v.kind = Value::Dbl;
    v.d = std::strtod(tok.c_str(), nullptr);
    return v;
  }
  static bool isdig(char c) { return c >= '0' && c <= '9'; }
};

inline Value parse(const std::string& text) { return Parser(text).parse(); }

}  // namespace oj
