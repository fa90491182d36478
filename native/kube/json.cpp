// JSON DOM implementation (see json.hpp).
#include "json.hpp"

#include <cstring>

namespace yk {

namespace {

struct Parser {
  const char* p;
  const char* beg;
  const char* end;
  int depth = 0;

  [[noreturn]] void fail(const char* what) const { throw ParseError{size_t(p - beg), what}; }

  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }

  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  uint32_t hex4() {
    if (end - p < 4) fail("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      int h = hexv(p[i]);
      if (h < 0) fail("bad \\u escape");
      v = v * 16 + uint32_t(h);
    }
    p += 4;
    return v;
  }

  static void utf8(uint32_t cp, std::string& out) {
    if (cp < 0x80) {
      out.push_back(char(cp));
    } else if (cp < 0x800) {
      out.push_back(char(0xC0 | (cp >> 6)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out.push_back(char(0xE0 | (cp >> 12)));
      out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    } else {
      out.push_back(char(0xF0 | (cp >> 18)));
      out.push_back(char(0x80 | ((cp >> 12) & 0x3F)));
      out.push_back(char(0x80 | ((cp >> 6) & 0x3F)));
      out.push_back(char(0x80 | (cp & 0x3F)));
    }
  }

  void string(std::string& out) {
    // p at the opening quote
    ++p;
    const char* run = p;
    // fast path: no escapes
    while (p < end) {
      char c = *p;
      if (c == '"') {
        out.assign(run, size_t(p - run));
        ++p;
        return;
      }
      if (c == '\\') break;
      if (static_cast<unsigned char>(c) < 0x20) fail("control character in string");
      ++p;
    }
    out.assign(run, size_t(p - run));
    while (p < end) {
      char c = *p++;
      if (c == '"') return;
      if (c != '\\') {
        if (static_cast<unsigned char>(c) < 0x20) fail("control character in string");
        out.push_back(c);
        continue;
      }
      if (p >= end) break;
      char e = *p++;
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              uint32_t lo = hex4();
              if (lo >= 0xDC00 && lo <= 0xDFFF) {
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              } else {
                utf8(0xFFFD, out);
                cp = lo;
              }
            } else {
              cp = 0xFFFD;
            }
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            cp = 0xFFFD;
          }
          utf8(cp, out);
          break;
        }
        default: fail("bad escape");
      }
    }
    fail("unterminated string");
  }

  void number(Value& v) {
    const char* s = p;
    if (p < end && *p == '-') ++p;
    if (p >= end) fail("bad number");
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') ++p;
    } else {
      fail("bad number");
    }
    if (p < end && *p == '.') {
      ++p;
      if (p >= end || *p < '0' || *p > '9') fail("bad fraction");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || *p < '0' || *p > '9') fail("bad exponent");
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    v.t = Value::Num;
    v.s.assign(s, size_t(p - s));
  }

  void lit(const char* w, size_t n) {
    if (size_t(end - p) < n || std::memcmp(p, w, n) != 0) fail("bad literal");
    p += n;
  }

  void value(Value& v) {
    ws();
    if (p >= end) fail("unexpected end");
    char c = *p;
    switch (c) {
      case '{': {
        if (++depth > 512) fail("nesting too deep");
        ++p;
        v.t = Value::Obj;
        ws();
        if (p < end && *p == '}') { ++p; --depth; return; }
        while (true) {
          ws();
          if (p >= end || *p != '"') fail("expected key");
          v.obj.emplace_back();
          Member& m = v.obj.back();
          string(m.first);
          ws();
          if (p >= end || *p != ':') fail("expected ':'");
          ++p;
          value(m.second);
          ws();
          if (p < end && *p == ',') { ++p; continue; }
          if (p < end && *p == '}') { ++p; break; }
          fail("expected ',' or '}'");
        }
        --depth;
        return;
      }
      case '[': {
        if (++depth > 512) fail("nesting too deep");
        ++p;
        v.t = Value::Arr;
        ws();
        if (p < end && *p == ']') { ++p; --depth; return; }
        while (true) {
          v.arr.emplace_back();
          value(v.arr.back());
          ws();
          if (p < end && *p == ',') { ++p; continue; }
          if (p < end && *p == ']') { ++p; break; }
          fail("expected ',' or ']'");
        }
        --depth;
        return;
      }
      case '"':
        v.t = Value::Str;
        string(v.s);
        return;
      case 't': lit("true", 4); v.t = Value::Bool; v.b = true; return;
      case 'f': lit("false", 5); v.t = Value::Bool; v.b = false; return;
      case 'n': lit("null", 4); v.t = Value::Null; return;
      default: number(v); return;
    }
  }
};

const char kHex[] = "0123456789abcdef";

inline uint64_t mix(uint64_t h, uint64_t x) {
  h ^= x + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  h *= 0xff51afd7ed558ccdull;
  return h ^ (h >> 33);
}

uint64_t hash_bytes(std::string_view s, uint64_t h) {
  // 8 bytes per step (multiply-xorshift over little-endian words), folded into the running
  // hash; the watch stream hashes every pod's spec + metadata three times per scheduled pod
  uint64_t f = 0xcbf29ce484222325ull ^ (s.size() * 0x9e3779b97f4a7c15ull);
  const char* p = s.data();
  size_t n = s.size();
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    f = (f ^ w) * 0x100000001b3ull;
    f ^= f >> 29;
    p += 8;
    n -= 8;
  }
  if (n) {
    uint64_t w = 0;
    std::memcpy(&w, p, n);
    f = (f ^ w) * 0x100000001b3ull;
    f ^= f >> 29;
  }
  return mix(h, f);
}

}  // namespace

uint64_t hash_mix(uint64_t h, uint64_t x) { return mix(h, x); }
uint64_t hash_text(std::string_view s, uint64_t h) { return hash_bytes(s, h); }

const Value* Value::get(std::string_view k) const {
  if (t != Obj) return nullptr;
  for (const auto& m : obj)
    if (m.first == k) return &m.second;
  return nullptr;
}

Value* Value::get(std::string_view k) {
  if (t != Obj) return nullptr;
  for (auto& m : obj)
    if (m.first == k) return &m.second;
  return nullptr;
}

const Value* Value::path(std::initializer_list<std::string_view> keys) const {
  const Value* v = this;
  for (auto k : keys) {
    v = v->get(k);
    if (!v) return nullptr;
  }
  return v;
}

std::string_view Value::sv(std::string_view k) const {
  const Value* v = get(k);
  return (v && v->t == Str) ? std::string_view(v->s) : std::string_view();
}

Value& Value::at(std::string_view k) {
  if (t == Null) t = Obj;
  for (auto& m : obj)
    if (m.first == k) return m.second;
  obj.emplace_back(std::string(k), Value());
  return obj.back().second;
}

bool Value::erase(std::string_view k) {
  if (t != Obj) return false;
  for (auto it = obj.begin(); it != obj.end(); ++it) {
    if (it->first == k) {
      obj.erase(it);
      return true;
    }
  }
  return false;
}

bool Value::truthy() const {
  switch (t) {
    case Null: return false;
    case Bool: return b;
    case Num: {
      for (char c : s)
        if (c >= '1' && c <= '9') return true;
      return false;
    }
    case Str: return !s.empty();
    case Arr: return !arr.empty();
    case Obj: return !obj.empty();
  }
  return false;
}

int64_t Value::as_int(bool* ok) const {
  if (ok) *ok = false;
  if (t != Num && t != Str) return 0;
  const std::string& x = s;
  size_t i = 0;
  bool neg = false;
  if (i < x.size() && (x[i] == '-' || x[i] == '+')) neg = x[i++] == '-';
  if (i >= x.size()) return 0;
  __int128 v = 0;
  for (; i < x.size(); ++i) {
    if (x[i] < '0' || x[i] > '9') return 0;
    v = v * 10 + (x[i] - '0');
    if (v > (__int128)INT64_MAX + 1) return 0;
  }
  if (neg) v = -v;
  if (v > INT64_MAX || v < INT64_MIN) return 0;
  if (ok) *ok = true;
  return int64_t(v);
}

Value parse(std::string_view text) {
  Parser ps{text.data(), text.data(), text.data() + text.size()};
  Value v;
  ps.value(v);
  ps.ws();
  if (ps.p != ps.end) ps.fail("trailing data");
  return v;
}

Value parse_prefix(std::string_view text, size_t* pos) {
  Parser ps{text.data() + *pos, text.data(), text.data() + text.size()};
  Value v;
  ps.value(v);
  *pos = size_t(ps.p - text.data());
  return v;
}

namespace {
// any byte of w that is '"', '\\' or a control character (< 0x20): SWAR zero-byte tests
inline bool word_needs_escape(uint64_t w) {
  constexpr uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
  const uint64_t q = w ^ (ones * '"'), b = w ^ (ones * '\\');
  const uint64_t zq = (q - ones) & ~q & highs, zb = (b - ones) & ~b & highs;
  const uint64_t lt = (w - ones * 0x20) & ~w & highs;   // bytes < 0x20 (ASCII-exact with the & ~w)
  return (zq | zb | lt) != 0;
}
}  // namespace

void dump_string(std::string_view s, std::string& out) {
  out.push_back('"');
  // clean 8-byte words (the common case: names, labels, timestamps) are copied in one append
  size_t i0 = 0;
  while (i0 + 8 <= s.size()) {
    uint64_t w;
    std::memcpy(&w, s.data() + i0, 8);
    if (word_needs_escape(w)) break;
    i0 += 8;
  }
  size_t run = 0;
  for (size_t i = i0; i < s.size(); ++i) {
    unsigned char c = static_cast<unsigned char>(s[i]);
    const char* rep = nullptr;
    char buf[7];
    if (c == '"') rep = "\\\"";
    else if (c == '\\') rep = "\\\\";
    else if (c == '\n') rep = "\\n";
    else if (c == '\r') rep = "\\r";
    else if (c == '\t') rep = "\\t";
    else if (c < 0x20) {
      buf[0] = '\\'; buf[1] = 'u'; buf[2] = '0'; buf[3] = '0';
      buf[4] = kHex[c >> 4]; buf[5] = kHex[c & 15]; buf[6] = 0;
      rep = buf;
    }
    if (rep) {
      out.append(s.data() + run, i - run);
      out.append(rep);
      run = i + 1;
    }
  }
  out.append(s.data() + run, s.size() - run);
  out.push_back('"');
}

void dump(const Value& v, std::string& out) {
  switch (v.t) {
    case Value::Null: out.append("null"); return;
    case Value::Bool: out.append(v.b ? "true" : "false"); return;
    case Value::Num: out.append(v.s); return;
    case Value::Str: dump_string(v.s, out); return;
    case Value::Arr: {
      out.push_back('[');
      bool first = true;
      for (const auto& x : v.arr) {
        if (!first) out.push_back(',');
        first = false;
        dump(x, out);
      }
      out.push_back(']');
      return;
    }
    case Value::Obj: {
      out.push_back('{');
      bool first = true;
      for (const auto& m : v.obj) {
        if (!first) out.push_back(',');
        first = false;
        dump_string(m.first, out);
        out.push_back(':');
        dump(m.second, out);
      }
      out.push_back('}');
      return;
    }
  }
}

std::string dump(const Value& v) {
  std::string out;
  out.reserve(256);
  dump(v, out);
  return out;
}

uint64_t hash(const Value& v, uint64_t h) {
  h = mix(h, v.t);
  switch (v.t) {
    case Value::Null: return h;
    case Value::Bool: return mix(h, v.b);
    case Value::Num:
    case Value::Str: return hash_bytes(v.s, h);
    case Value::Arr:
      for (const auto& x : v.arr) h = hash(x, h);
      return mix(h, v.arr.size());
    case Value::Obj:
      for (const auto& m : v.obj) h = hash(m.second, hash_bytes(m.first, h));
      return mix(h, v.obj.size());
  }
  return h;
}

void merge_patch(Value& target, const Value& patch) {
  if (patch.t != Value::Obj) {
    target = patch;
    return;
  }
  if (target.t != Value::Obj) {
    target = Value::object();
  }
  for (const auto& m : patch.obj) {
    if (m.second.t == Value::Null) {
      target.erase(m.first);
    } else {
      merge_patch(target.at(m.first), m.second);
    }
  }
}

namespace {
const char* merge_key_of(std::string_view field) {
  static const std::pair<const char*, const char*> kKeys[] = {
      {"conditions", "type"},     {"containers", "name"}, {"initContainers", "name"},
      {"ephemeralContainers", "name"}, {"volumes", "name"}, {"env", "name"},
      {"ports", "containerPort"}, {"ownerReferences", "uid"}, {"volumeMounts", "mountPath"},
      {"imagePullSecrets", "name"}};
  for (const auto& k : kKeys)
    if (field == k.first) return k.second;
  return nullptr;
}
}  // namespace

void strategic_merge_patch(Value& target, const Value& patch) {
  if (patch.t != Value::Obj) {
    target = patch;
    return;
  }
  if (target.t != Value::Obj) target = Value::object();
  for (const auto& m : patch.obj) {
    const std::string& k = m.first;
    if (!k.empty() && k[0] == '$') continue;                 // $setElementOrder/..., $retainKeys, $patch
    if (m.second.t == Value::Null) {
      target.erase(k);
      continue;
    }
    const char* mk = merge_key_of(k);
    Value* cur = target.get(k);
    if (mk && m.second.t == Value::Arr && cur && cur->t == Value::Arr) {
      for (const Value& item : m.second.arr) {
        const Value* key = item.t == Value::Obj ? item.get(mk) : nullptr;
        if (!key) {
          cur->arr.push_back(item);
          continue;
        }
        auto it = cur->arr.begin();
        for (; it != cur->arr.end(); ++it) {
          const Value* ck = it->t == Value::Obj ? it->get(mk) : nullptr;
          if (ck && equal(*ck, *key)) break;
        }
        const bool del = item.sv("$patch") == "delete";
        if (it == cur->arr.end()) {
          if (!del) {
            Value fresh = Value::object();
            strategic_merge_patch(fresh, item);
            cur->arr.push_back(std::move(fresh));
          }
        } else if (del) {
          cur->arr.erase(it);
        } else {
          strategic_merge_patch(*it, item);
        }
      }
      continue;
    }
    if (m.second.t == Value::Arr) {
      // a list without a merge key is replaced, its elements' directives dropped
      Value repl = Value::array();
      for (const Value& item : m.second.arr) {
        if (item.t == Value::Obj) {
          Value fresh = Value::object();
          strategic_merge_patch(fresh, item);
          repl.arr.push_back(std::move(fresh));
        } else {
          repl.arr.push_back(item);
        }
      }
      target.at(k) = std::move(repl);
      continue;
    }
    strategic_merge_patch(target.at(k), m.second);
  }
}

bool equal(const Value& a, const Value& b) {
  if (a.t != b.t) return false;
  switch (a.t) {
    case Value::Null: return true;
    case Value::Bool: return a.b == b.b;
    case Value::Num:
    case Value::Str: return a.s == b.s;
    case Value::Arr:
      if (a.arr.size() != b.arr.size()) return false;
      for (size_t i = 0; i < a.arr.size(); ++i)
        if (!equal(a.arr[i], b.arr[i])) return false;
      return true;
    case Value::Obj:
      if (a.obj.size() != b.obj.size()) return false;
      for (size_t i = 0; i < a.obj.size(); ++i)
        if (a.obj[i].first != b.obj[i].first || !equal(a.obj[i].second, b.obj[i].second)) return false;
      return true;
  }
  return false;
}

}  // namespace yk
