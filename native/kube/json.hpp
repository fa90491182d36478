// Small JSON DOM for the Kubernetes wire format (RFC 8259): parser, compact serializer,
// structural hash and RFC 7386 merge patch. Shared by the scheduler's native transport
// (watch-event projection, native/kube/transport.cpp) and the native fake apiserver
// (native/kube/fakeapi.cpp).
//
// Numbers keep their source text, so a re-serialised object is byte-identical in its
// numeric fields (resourceVersions, quantities and int64 priorities never pass through
// a double).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace yk {

struct Value;
using Member = std::pair<std::string, Value>;

struct Value {
  enum Type : uint8_t { Null, Bool, Num, Str, Arr, Obj };
  Type t = Null;
  bool b = false;
  std::string s;              // Str: unescaped text; Num: source text
  std::vector<Value> arr;
  std::vector<Member> obj;

  Value() = default;
  static Value str(std::string v) { Value x; x.t = Str; x.s = std::move(v); return x; }
  static Value num(std::string v) { Value x; x.t = Num; x.s = std::move(v); return x; }
  static Value num(int64_t v) { return num(std::to_string(v)); }
  static Value boolean(bool v) { Value x; x.t = Bool; x.b = v; return x; }
  static Value object() { Value x; x.t = Obj; return x; }
  static Value array() { Value x; x.t = Arr; return x; }

  bool is_obj() const { return t == Obj; }
  bool is_arr() const { return t == Arr; }
  bool is_str() const { return t == Str; }
  bool is_null() const { return t == Null; }

  // object lookup (linear: Kubernetes objects have small maps); nullptr when absent
  const Value* get(std::string_view k) const;
  Value* get(std::string_view k);
  // nested lookup "a", "b", "c"
  const Value* path(std::initializer_list<std::string_view> keys) const;
  // string value of a member ("" when absent or not a string)
  std::string_view sv(std::string_view k) const;
  // member by key, inserted (as null) when absent; *this becomes an object if it was null
  Value& at(std::string_view k);
  bool erase(std::string_view k);
  // truthiness the way Python's `if x:` reads decoded JSON
  bool truthy() const;
  // integer value of a Num (or a numeric Str); `ok` false when not an integer
  int64_t as_int(bool* ok = nullptr) const;
};

struct ParseError {
  size_t pos;
  const char* what;
};

// Parses one JSON value spanning the whole of `text` (surrounding whitespace allowed).
// Throws ParseError.
Value parse(std::string_view text);
// Parses one JSON value starting at text[*pos]; advances *pos past it.
Value parse_prefix(std::string_view text, size_t* pos);

void dump(const Value& v, std::string& out);
std::string dump(const Value& v);
void dump_string(std::string_view s, std::string& out);   // quoted + escaped

// 64-bit structural hash (member order sensitive, as the apiserver preserves order)
uint64_t hash(const Value& v, uint64_t seed = 0x9e3779b97f4a7c15ull);

// RFC 7386 JSON merge patch: applies `patch` onto `target` in place
void merge_patch(Value& target, const Value& patch);
// Kubernetes strategic merge patch (the subset the core/v1 Pod needs): like a merge patch, but
// lists with a patch merge key (status.conditions by type, containers / volumes / env by name,
// ports by containerPort, ownerReferences by uid) merge element-wise by that key, an element
// with "$patch": "delete" removes its match, and $setElementOrder / $retainKeys directives are
// accepted and ignored
void strategic_merge_patch(Value& target, const Value& patch);

bool equal(const Value& a, const Value& b);

// the hash's building blocks (shared with flatjson.hpp so both hashes agree)
uint64_t hash_mix(uint64_t h, uint64_t x);
uint64_t hash_text(std::string_view s, uint64_t h);

}  // namespace yk
