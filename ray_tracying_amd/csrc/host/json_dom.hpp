// json_dom.hpp -- compact JSON DOM for the scene loader (host C++).
//
// Semantics follow what the reference takes from nlohmann/json 3.12.0
// (/root/reference/Code/json.hpp): integer tokens are int64 (leading '-') or uint64 and fall
// back to double on overflow; other numbers are decimal -> double (correctly rounded, like
// strtod, json.hpp:7987-7989, 8357) and get<float>() narrows double -> float
// (json.hpp:5229-5262); booleans convert to 0/1 in numeric gets; get<int>() truncates;
// duplicate keys: the last one wins.  Built for 10^8-byte scene files (1M-triangle soups):
// 16-byte nodes, children stored contiguously, numbers parsed with std::from_chars.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

namespace rth {

struct JsonError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class JsonDoc {
 public:
  enum Kind : uint8_t { Null, Bool, Int, Uint, Dbl, Str, Arr, Obj };
  struct Node {
    uint8_t kind;
    uint32_t n;     // Arr/Obj: child count; Str: length
    uint64_t pay;   // Int/Uint/Dbl bits; Bool; Str: offset into pool; Arr/Obj: first slot in kids_
  };
  // Parses `text`; throws JsonError("parse_error...") on malformed input.
  explicit JsonDoc(std::string_view text);

  uint32_t root() const { return root_; }
  Kind kind(uint32_t v) const { return (Kind)nodes_[v].kind; }
  bool is_array(uint32_t v) const { return kind(v) == Arr; }
  bool is_object(uint32_t v) const { return kind(v) == Obj; }
  bool is_number(uint32_t v) const { Kind k = kind(v); return k == Int || k == Uint || k == Dbl; }
  uint32_t size(uint32_t v) const { Kind k = kind(v); return (k == Arr || k == Obj) ? nodes_[v].n : (k == Null ? 0 : 1); }
  bool empty(uint32_t v) const { Kind k = kind(v); return k == Null || ((k == Arr || k == Obj) && nodes_[v].n == 0); }
  // array element (throws like json::at)
  uint32_t at(uint32_t v, uint32_t i) const;
  // object member lookup; returns kNone if absent (last duplicate wins)
  static constexpr uint32_t kNone = 0xFFFFFFFFu;
  uint32_t find(uint32_t v, std::string_view key) const;
  bool contains(uint32_t v, std::string_view key) const { return is_object(v) && find(v, key) != kNone; }
  // conversions with nlohmann's rules
  double as_double(uint32_t v) const;  // numbers and bools, else type_error.302
  float get_float(uint32_t v) const;
  int get_int(uint32_t v) const;
  void get_vec3(uint32_t v, float out[3]) const;  // .at(0..2).get<float>()
  std::string get_string(uint32_t v) const;
  // object.value(key, default) -- throws type_error.306 on non-objects
  float value_float(uint32_t v, std::string_view key, float def) const;
  uint32_t child(uint32_t v, uint32_t i) const { return kids_[nodes_[v].pay + i]; }
  std::string_view key(uint32_t v, uint32_t i) const;  // object member i's key

 private:
  std::vector<Node> nodes_;
  std::vector<uint32_t> kids_;   // Arr: child ids; Obj: (key node id, value node id) pairs
  std::string pool_;
  uint32_t root_ = 0;
  friend class JsonParser;
};

}  // namespace rth
