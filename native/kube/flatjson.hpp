// Flat JSON document for the hot decode path: one pass over the text into a vector of nodes
// that point back into it (no per-value allocation; only strings with escapes are decoded
// into a side buffer). The watch stream decodes three events per scheduled pod (ADDED, the
// Binding's echo, DELETED), so this replaces the allocating DOM (json.hpp) there; semantics
// (string unescaping, number text, truthiness, integer reading, structural hash) are the
// DOM's, so a projection over either agrees field for field
// (tests/test_native_kube.py::test_flat_projection_equals_dom_projection).
#pragma once

#include <cstdint>
#include <string>
#include <string_view>
#include <vector>

namespace yk {

class FlatDoc {
 public:
  enum Type : uint8_t { Null, Bool, Num, Str, Arr, Obj };
  struct Node {
    uint8_t t = Null;
    bool b = false;
    bool esc = false;          // Str: decoded text lives in the side buffer
    uint32_t off = 0, len = 0; // Str/Num: text span (source, or side buffer when esc); Arr/Obj: child count in len
    uint32_t koff = 0, klen = 0;
    bool kesc = false;
    uint32_t next = 0;         // index of the next sibling (0 = none)
    uint32_t first = 0;        // Arr/Obj: first child (0 = none)
    uint32_t beg = 0, end = 0; // source span of the whole value
  };

  // Parses `text` (one JSON value, surrounding whitespace allowed). False on malformed input.
  bool parse(std::string_view text);

  class View {
   public:
    View() = default;
    View(const FlatDoc* d, uint32_t i) : d_(d), i_(i) {}
    explicit operator bool() const { return d_ != nullptr; }
    Type t() const { return Type(node().t); }
    bool is(Type x) const { return d_ && node().t == x; }
    View get(std::string_view k) const;           // object member (first match), empty when absent
    std::string_view sv(std::string_view k) const;  // string member, "" when absent / not a string
    std::string_view str() const;                 // Str: unescaped text; Num: source text
    std::string_view key() const;                 // member key (unescaped)
    std::string_view raw() const;                 // source text of the value
    bool truthy() const;
    bool b() const { return node().b; }
    int64_t as_int(bool* ok) const;
    size_t size() const { return node().len; }    // Arr/Obj: number of children
    View first() const;                           // first child
    View next() const;                            // next sibling
    uint64_t hash(uint64_t seed) const;           // == yk::hash of the equivalent DOM Value

   private:
    const Node& node() const { return d_->nodes_[i_]; }
    const FlatDoc* d_ = nullptr;
    uint32_t i_ = 0;
  };

  View root() const { return nodes_.empty() ? View() : View(this, 0); }

 private:
  friend class View;
  std::string_view text_;
  std::vector<Node> nodes_;
  std::string side_;           // unescaped strings
};

// the DOM hash helpers (json.cpp), shared so the flat hash is bit-identical
uint64_t hash_mix(uint64_t h, uint64_t x);
uint64_t hash_text(std::string_view s, uint64_t h);

}  // namespace yk
