// Flat JSON document (see flatjson.hpp). Grammar and unescaping follow json.cpp's parser.
#include "flatjson.hpp"

#include <cstring>

namespace yk {

namespace {

struct FlatParser {
  const char* p;
  const char* base;
  const char* end;
  std::vector<FlatDoc::Node>& nodes;
  std::string& side;
  int depth = 0;
  bool bad = false;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }

  static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }

  bool hex4(uint32_t* out) {
    if (end - p < 4) return false;
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      int h = hexv(p[i]);
      if (h < 0) return false;
      v = v * 16 + uint32_t(h);
    }
    p += 4;
    *out = v;
    return true;
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

  // any byte that is '"', '\\' or < 0x20 in an 8-byte word
  static bool special(uint64_t w) {
    constexpr uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
    const uint64_t q = w ^ (ones * '"'), b = w ^ (ones * '\\');
    const uint64_t zq = (q - ones) & ~q & highs, zb = (b - ones) & ~b & highs;
    const uint64_t lt = (w - ones * 0x20) & ~w & highs;
    return (zq | zb | lt) != 0;
  }

  // p at the opening quote; (off, len, esc) of the string's text
  bool string(uint32_t* off, uint32_t* len, bool* esc) {
    ++p;
    const char* run = p;
    while (end - p >= 8) {
      uint64_t w;
      std::memcpy(&w, p, 8);
      if (special(w)) break;
      p += 8;
    }
    while (p < end) {
      const char c = *p;
      if (c == '"') {
        *off = uint32_t(run - base);
        *len = uint32_t(p - run);
        *esc = false;
        ++p;
        return true;
      }
      if (c == '\\') break;
      if (static_cast<unsigned char>(c) < 0x20) return false;
      ++p;
    }
    // escapes: decode into the side buffer
    const size_t s0 = side.size();
    side.append(run, size_t(p - run));
    while (p < end) {
      const char c = *p++;
      if (c == '"') {
        *off = uint32_t(s0);
        *len = uint32_t(side.size() - s0);
        *esc = true;
        return true;
      }
      if (c != '\\') {
        if (static_cast<unsigned char>(c) < 0x20) return false;
        side.push_back(c);
        continue;
      }
      if (p >= end) return false;
      const char e = *p++;
      switch (e) {
        case '"': side.push_back('"'); break;
        case '\\': side.push_back('\\'); break;
        case '/': side.push_back('/'); break;
        case 'b': side.push_back('\b'); break;
        case 'f': side.push_back('\f'); break;
        case 'n': side.push_back('\n'); break;
        case 'r': side.push_back('\r'); break;
        case 't': side.push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xD800 && cp <= 0xDBFF) {
            if (end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              uint32_t lo;
              if (!hex4(&lo)) return false;
              if (lo >= 0xDC00 && lo <= 0xDFFF) {
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              } else {
                utf8(0xFFFD, side);
                cp = lo;
              }
            } else {
              cp = 0xFFFD;
            }
          } else if (cp >= 0xDC00 && cp <= 0xDFFF) {
            cp = 0xFFFD;
          }
          utf8(cp, side);
          break;
        }
        default: return false;
      }
    }
    return false;
  }

  bool number(FlatDoc::Node& n) {
    const char* s = p;
    if (p < end && *p == '-') ++p;
    if (p >= end) return false;
    if (*p == '0') {
      ++p;
    } else if (*p >= '1' && *p <= '9') {
      while (p < end && *p >= '0' && *p <= '9') ++p;
    } else {
      return false;
    }
    if (p < end && *p == '.') {
      ++p;
      if (p >= end || *p < '0' || *p > '9') return false;
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    if (p < end && (*p == 'e' || *p == 'E')) {
      ++p;
      if (p < end && (*p == '+' || *p == '-')) ++p;
      if (p >= end || *p < '0' || *p > '9') return false;
      while (p < end && *p >= '0' && *p <= '9') ++p;
    }
    n.t = FlatDoc::Num;
    n.off = uint32_t(s - base);
    n.len = uint32_t(p - s);
    return true;
  }

  bool lit(const char* w, size_t k) {
    if (size_t(end - p) < k || std::memcmp(p, w, k) != 0) return false;
    p += k;
    return true;
  }

  // parses one value into a new node; returns its index (0 with bad=true on error)
  uint32_t value() {
    ws();
    if (p >= end) return fail();
    const uint32_t idx = uint32_t(nodes.size());
    nodes.emplace_back();
    nodes[idx].beg = uint32_t(p - base);
    switch (*p) {
      case '{':
      case '[': {
        const bool obj = *p == '{';
        const char close = obj ? '}' : ']';
        if (++depth > 512) return fail();
        ++p;
        nodes[idx].t = obj ? FlatDoc::Obj : FlatDoc::Arr;
        ws();
        if (p < end && *p == close) {
          ++p;
          --depth;
          break;
        }
        uint32_t prev = 0, cnt = 0;
        while (true) {
          uint32_t koff = 0, klen = 0;
          bool kesc = false;
          if (obj) {
            ws();
            if (p >= end || *p != '"' || !string(&koff, &klen, &kesc)) return fail();
            ws();
            if (p >= end || *p != ':') return fail();
            ++p;
          }
          const uint32_t c = value();
          if (bad) return 0;
          if (obj) {
            nodes[c].koff = koff;
            nodes[c].klen = klen;
            nodes[c].kesc = kesc;
          }
          if (cnt == 0) nodes[idx].first = c;
          else nodes[prev].next = c;
          prev = c;
          ++cnt;
          ws();
          if (p < end && *p == ',') {
            ++p;
            continue;
          }
          if (p < end && *p == close) {
            ++p;
            break;
          }
          return fail();
        }
        nodes[idx].len = cnt;
        --depth;
        break;
      }
      case '"': {
        uint32_t off, len;
        bool esc;
        if (!string(&off, &len, &esc)) return fail();
        nodes[idx].t = FlatDoc::Str;
        nodes[idx].off = off;
        nodes[idx].len = len;
        nodes[idx].esc = esc;
        break;
      }
      case 't':
        if (!lit("true", 4)) return fail();
        nodes[idx].t = FlatDoc::Bool;
        nodes[idx].b = true;
        break;
      case 'f':
        if (!lit("false", 5)) return fail();
        nodes[idx].t = FlatDoc::Bool;
        break;
      case 'n':
        if (!lit("null", 4)) return fail();
        break;
      default:
        if (!number(nodes[idx])) return fail();
    }
    nodes[idx].end = uint32_t(p - base);
    return idx;
  }

  uint32_t fail() {
    bad = true;
    return 0;
  }
};

}  // namespace

bool FlatDoc::parse(std::string_view text) {
  text_ = text;
  nodes_.clear();
  side_.clear();
  if (text.size() >= (1ull << 32)) return false;
  nodes_.reserve(64);
  FlatParser ps{text.data(), text.data(), text.data() + text.size(), nodes_, side_};
  ps.value();
  if (ps.bad) {
    nodes_.clear();
    return false;
  }
  ps.ws();
  if (ps.p != ps.end) {
    nodes_.clear();
    return false;
  }
  return true;
}

FlatDoc::View FlatDoc::View::get(std::string_view k) const {
  if (!d_ || node().t != Obj) return View();
  for (uint32_t c = node().first; c; c = d_->nodes_[c].next) {
    const Node& n = d_->nodes_[c];
    const std::string_view key = n.kesc ? std::string_view(d_->side_).substr(n.koff, n.klen)
                                        : d_->text_.substr(n.koff, n.klen);
    if (key == k) return View(d_, c);
  }
  return View();
}

std::string_view FlatDoc::View::sv(std::string_view k) const {
  View v = get(k);
  return v && v.t() == Str ? v.str() : std::string_view();
}

std::string_view FlatDoc::View::str() const {
  const Node& n = node();
  if (n.t != Str && n.t != Num) return std::string_view();
  return n.esc ? std::string_view(d_->side_).substr(n.off, n.len) : d_->text_.substr(n.off, n.len);
}

std::string_view FlatDoc::View::key() const {
  const Node& n = node();
  return n.kesc ? std::string_view(d_->side_).substr(n.koff, n.klen) : d_->text_.substr(n.koff, n.klen);
}

std::string_view FlatDoc::View::raw() const {
  const Node& n = node();
  return d_->text_.substr(n.beg, n.end - n.beg);
}

bool FlatDoc::View::truthy() const {
  if (!d_) return false;
  const Node& n = node();
  switch (n.t) {
    case Null: return false;
    case Bool: return n.b;
    case Num: {
      for (char c : str())
        if (c >= '1' && c <= '9') return true;
      return false;
    }
    case Str: return n.len != 0;
    case Arr:
    case Obj: return n.len != 0;
  }
  return false;
}

int64_t FlatDoc::View::as_int(bool* ok) const {
  if (ok) *ok = false;
  if (!d_ || (node().t != Num && node().t != Str)) return 0;
  const std::string_view x = str();
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

FlatDoc::View FlatDoc::View::first() const {
  if (!d_) return View();
  const Node& n = node();
  return (n.t == Arr || n.t == Obj) && n.first ? View(d_, n.first) : View();
}

FlatDoc::View FlatDoc::View::next() const {
  if (!d_) return View();
  return node().next ? View(d_, node().next) : View();
}

uint64_t FlatDoc::View::hash(uint64_t h) const {
  // yk::hash (json.cpp) over the equivalent DOM value
  const Node& n = node();
  h = hash_mix(h, n.t);
  switch (n.t) {
    case Null: return h;
    case Bool: return hash_mix(h, n.b);
    case Num:
    case Str: return hash_text(str(), h);
    case Arr:
      for (View c = first(); c; c = c.next()) h = c.hash(h);
      return hash_mix(h, n.len);
    case Obj:
      for (View c = first(); c; c = c.next()) h = c.hash(hash_text(c.key(), h));
      return hash_mix(h, n.len);
  }
  return h;
}

}  // namespace yk
