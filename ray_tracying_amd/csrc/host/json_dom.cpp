// json_dom.cpp -- see json_dom.hpp.
#include "json_dom.hpp"

#include <charconv>
#include <cstring>

namespace rth {

class JsonParser {
 public:
  JsonParser(JsonDoc& d, std::string_view t) : d_(d), t_(t) {}
  uint32_t run() {
    uint32_t v = value();
    ws();
    if (p_ != t_.size()) fail("trailing characters");
    return v;
  }

 private:
  JsonDoc& d_;
  std::string_view t_;
  size_t p_ = 0;
  std::vector<uint32_t> tmp_;

  [[noreturn]] void fail(const char* m) {
    throw JsonError(std::string("parse_error: ") + m + " at byte " + std::to_string(p_));
  }
  void ws() {
    while (p_ < t_.size()) {
      char c = t_[p_];
      if (c == ' ' || c == '\n' || c == '\t' || c == '\r') ++p_;
      else break;
    }
  }
  uint32_t push(JsonDoc::Kind k, uint32_t n, uint64_t pay) {
    d_.nodes_.push_back(JsonDoc::Node{(uint8_t)k, n, pay});
    return (uint32_t)(d_.nodes_.size() - 1);
  }
  bool lit(const char* w, size_t n) {
    if (t_.size() - p_ >= n && std::memcmp(t_.data() + p_, w, n) == 0) { p_ += n; return true; }
    return false;
  }
  uint32_t value() {
    ws();
    if (p_ >= t_.size()) fail("unexpected end of input");
    char c = t_[p_];
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') return string_node();
    if (lit("true", 4)) return push(JsonDoc::Bool, 0, 1);
    if (lit("false", 5)) return push(JsonDoc::Bool, 0, 0);
    if (lit("null", 4)) return push(JsonDoc::Null, 0, 0);
    return number();
  }
  uint32_t array() {
    ++p_;
    size_t mark = tmp_.size();
    ws();
    if (p_ < t_.size() && t_[p_] == ']') {
      ++p_;
    } else {
      for (;;) {
        tmp_.push_back(value());
        ws();
        if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
        if (p_ < t_.size() && t_[p_] == ']') { ++p_; break; }
        fail("expected ',' or ']'");
      }
    }
    uint32_t n = (uint32_t)(tmp_.size() - mark);
    uint64_t start = d_.kids_.size();
    d_.kids_.insert(d_.kids_.end(), tmp_.begin() + mark, tmp_.end());
    tmp_.resize(mark);
    return push(JsonDoc::Arr, n, start);
  }
  uint32_t object() {
    ++p_;
    size_t mark = tmp_.size();
    ws();
    if (p_ < t_.size() && t_[p_] == '}') {
      ++p_;
    } else {
      for (;;) {
        ws();
        if (p_ >= t_.size() || t_[p_] != '"') fail("expected string key");
        uint32_t k = string_node();
        ws();
        if (p_ >= t_.size() || t_[p_] != ':') fail("expected ':'");
        ++p_;
        uint32_t v = value();
        tmp_.push_back(k);
        tmp_.push_back(v);
        ws();
        if (p_ < t_.size() && t_[p_] == ',') { ++p_; continue; }
        if (p_ < t_.size() && t_[p_] == '}') { ++p_; break; }
        fail("expected ',' or '}'");
      }
    }
    uint32_t n = (uint32_t)((tmp_.size() - mark) / 2);
    uint64_t start = d_.kids_.size();
    d_.kids_.insert(d_.kids_.end(), tmp_.begin() + mark, tmp_.end());
    tmp_.resize(mark);
    return push(JsonDoc::Obj, n, start);
  }
  static void utf8(std::string& o, unsigned cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  }
  unsigned hex4() {
    if (t_.size() - p_ < 4) fail("bad \\u escape");
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = t_[p_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (unsigned)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (unsigned)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (unsigned)(c - 'A' + 10);
      else fail("bad \\u escape");
    }
    return v;
  }
  uint32_t string_node() {
    ++p_;
    size_t off = d_.pool_.size();
    std::string& o = d_.pool_;
    for (;;) {
      if (p_ >= t_.size()) fail("unterminated string");
      char c = t_[p_++];
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (c != '\\') { o += c; continue; }
      if (p_ >= t_.size()) fail("bad escape");
      char e = t_[p_++];
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
          unsigned cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (!lit("\\u", 2)) fail("missing low surrogate");
            unsigned lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return push(JsonDoc::Str, (uint32_t)(o.size() - off), off);
  }
  uint32_t number() {
    const size_t b = p_;
    bool is_float = false;
    auto dig = [&](size_t i) { return i < t_.size() && t_[i] >= '0' && t_[i] <= '9'; };
    if (t_[p_] == '-') ++p_;
    if (p_ < t_.size() && t_[p_] == '0') ++p_;
    else if (dig(p_)) { while (dig(p_)) ++p_; }
    else fail("invalid literal");
    if (p_ < t_.size() && t_[p_] == '.') {
      is_float = true;
      ++p_;
      if (!dig(p_)) fail("invalid fraction");
      while (dig(p_)) ++p_;
    }
    if (p_ < t_.size() && (t_[p_] == 'e' || t_[p_] == 'E')) {
      is_float = true;
      ++p_;
      if (p_ < t_.size() && (t_[p_] == '+' || t_[p_] == '-')) ++p_;
      if (!dig(p_)) fail("invalid exponent");
      while (dig(p_)) ++p_;
    }
    const char* first = t_.data() + b;
    const char* last = t_.data() + p_;
    if (!is_float) {
      if (*first == '-') {
        int64_t v;
        auto r = std::from_chars(first, last, v);
        if (r.ec == std::errc()) { uint64_t u; std::memcpy(&u, &v, 8); return push(JsonDoc::Int, 0, u); }
      } else {
        uint64_t v;
        auto r = std::from_chars(first, last, v);
        if (r.ec == std::errc()) return push(JsonDoc::Uint, 0, v);
      }
    }
    double dv = 0;
    auto r = std::from_chars(first, last, dv);  // correctly rounded, == strtod
    if (r.ec == std::errc::result_out_of_range) dv = std::strtod(std::string(first, last).c_str(), nullptr);
    uint64_t bits;
    std::memcpy(&bits, &dv, 8);
    return push(JsonDoc::Dbl, 0, bits);
  }
};

JsonDoc::JsonDoc(std::string_view text) {
  nodes_.reserve(text.size() / 8 + 16);
  kids_.reserve(text.size() / 8 + 16);
  JsonParser p(*this, text);
  root_ = p.run();
}

uint32_t JsonDoc::at(uint32_t v, uint32_t i) const {
  if (kind(v) != Arr) throw JsonError("type_error.304: cannot use at() with " + std::to_string(kind(v)));
  if (i >= nodes_[v].n) throw JsonError("out_of_range.401: array index " + std::to_string(i) + " is out of range");
  return kids_[nodes_[v].pay + i];
}

std::string_view JsonDoc::key(uint32_t v, uint32_t i) const {
  const Node& k = nodes_[kids_[nodes_[v].pay + 2 * (uint64_t)i]];
  return std::string_view(pool_.data() + k.pay, k.n);
}

uint32_t JsonDoc::find(uint32_t v, std::string_view key_) const {
  if (kind(v) != Obj) return kNone;
  const Node& o = nodes_[v];
  uint32_t found = kNone;
  for (uint32_t i = 0; i < o.n; ++i) {
    const Node& k = nodes_[kids_[o.pay + 2 * (uint64_t)i]];
    if (k.n == key_.size() && std::memcmp(pool_.data() + k.pay, key_.data(), k.n) == 0) found = kids_[o.pay + 2 * (uint64_t)i + 1];
  }
  return found;
}

double JsonDoc::as_double(uint32_t v) const {
  const Node& n = nodes_[v];
  switch ((Kind)n.kind) {
    case Uint: return (double)n.pay;
    case Int: { int64_t x; std::memcpy(&x, &n.pay, 8); return (double)x; }
    case Dbl: { double x; std::memcpy(&x, &n.pay, 8); return x; }
    case Bool: return n.pay ? 1.0 : 0.0;
    default: throw JsonError("type_error.302: type must be number");
  }
}

float JsonDoc::get_float(uint32_t v) const {
  const Node& n = nodes_[v];
  switch ((Kind)n.kind) {
    case Uint: return (float)n.pay;  // static_cast<float>(uint64) -- one rounding
    case Int: { int64_t x; std::memcpy(&x, &n.pay, 8); return (float)x; }
    case Dbl: { double x; std::memcpy(&x, &n.pay, 8); return (float)x; }
    case Bool: return n.pay ? 1.0f : 0.0f;
    default: throw JsonError("type_error.302: type must be number");
  }
}

int JsonDoc::get_int(uint32_t v) const {
  const Node& n = nodes_[v];
  switch ((Kind)n.kind) {
    case Uint: return (int)n.pay;
    case Int: { int64_t x; std::memcpy(&x, &n.pay, 8); return (int)x; }
    case Dbl: { double x; std::memcpy(&x, &n.pay, 8); return (int)x; }
    case Bool: return n.pay ? 1 : 0;
    default: throw JsonError("type_error.302: type must be number");
  }
}

void JsonDoc::get_vec3(uint32_t v, float out[3]) const {
  for (uint32_t i = 0; i < 3; ++i) out[i] = get_float(at(v, i));
}

std::string JsonDoc::get_string(uint32_t v) const {
  if (kind(v) != Str) throw JsonError("type_error.302: type must be string");
  return std::string(pool_.data() + nodes_[v].pay, nodes_[v].n);
}

float JsonDoc::value_float(uint32_t v, std::string_view k, float def) const {
  if (kind(v) != Obj) throw JsonError("type_error.306: cannot use value() with non-object");
  uint32_t f = find(v, k);
  return f == kNone ? def : get_float(f);
}

}  // namespace rth
