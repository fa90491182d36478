// Incremental HTTP/1.1 message parsers (header-only): responses for the scheduler's
// native client (pipelined keep-alive requests, chunked watch streams) and requests for
// the native fake apiserver. Both consume bytes as they arrive and never block.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace yk {

inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? char(c + 32) : c; }

inline bool iequals(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i)
    if (lower(a[i]) != lower(b[i])) return false;
  return true;
}

inline std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.remove_suffix(1);
  return s;
}

struct Headers {
  std::vector<std::pair<std::string, std::string>> h;   // names lower-cased
  std::string_view get(std::string_view name) const {
    for (const auto& kv : h)
      if (kv.first == name) return kv.second;
    return {};
  }
  bool has(std::string_view name) const {
    for (const auto& kv : h)
      if (kv.first == name) return true;
    return false;
  }
};

// Parses one header line "Name: value" into `hs`; false on a malformed line.
inline bool parse_header_line(std::string_view line, Headers& hs) {
  size_t c = line.find(':');
  if (c == std::string_view::npos || c == 0) return false;
  std::string name(line.substr(0, c));
  for (auto& ch : name) ch = lower(ch);
  hs.h.emplace_back(std::move(name), std::string(trim(line.substr(c + 1))));
  return true;
}

// Response parser. Body bytes are handed to `on_body` as they arrive (streaming), and the
// message end is reported by feed()'s return. Supports Content-Length, chunked and
// read-until-close bodies, plus HEAD-less responses without a body (1xx/204/304).
class ResponseParser {
 public:
  enum State { kStatus, kHeaders, kLen, kChunkSize, kChunkData, kChunkCrlf, kTrailers, kClose, kDone };

  int status = 0;
  Headers headers;
  bool keep_alive = true;

  void reset() {
    st_ = kStatus;
    status = 0;
    headers.h.clear();
    keep_alive = true;
    remaining_ = 0;
    line_.clear();
  }

  // Consumes bytes from data[0..n). Returns the number consumed; sets *done when the
  // message completed (the caller resets and feeds the rest to the next response).
  // Body bytes go to on_body(const char*, size_t). Returns -1 on a protocol error.
  template <class OnBody>
  long feed(const char* data, size_t n, bool* done, OnBody&& on_body) {
    size_t i = 0;
    *done = false;
    while (i < n) {
      switch (st_) {
        case kStatus:
        case kHeaders:
        case kChunkSize:
        case kChunkCrlf:
        case kTrailers: {
          const char* nl = static_cast<const char*>(std::memchr(data + i, '\n', n - i));
          if (!nl) {
            line_.append(data + i, n - i);
            if (line_.size() > 65536) return -1;
            return long(n);
          }
          line_.append(data + i, size_t(nl - (data + i)));
          i = size_t(nl - data) + 1;
          std::string_view line(line_);
          if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
          if (!line_step(line, done)) return -1;
          line_.clear();
          if (*done) return long(i);
          break;
        }
        case kLen:
        case kChunkData: {
          size_t take = std::min<uint64_t>(remaining_, n - i);
          if (take) on_body(data + i, take);
          i += take;
          remaining_ -= take;
          if (remaining_ == 0) {
            if (st_ == kLen) {
              st_ = kDone;
              *done = true;
              return long(i);
            }
            st_ = kChunkCrlf;
          }
          break;
        }
        case kClose:
          on_body(data + i, n - i);
          return long(n);
        case kDone:
          *done = true;
          return long(i);
      }
    }
    return long(i);
  }

  // the peer closed: a read-until-close body completes, anything else is truncated
  bool finish_on_close() {
    if (st_ == kClose) {
      st_ = kDone;
      return true;
    }
    return false;
  }

  bool in_body() const { return st_ == kLen || st_ == kChunkSize || st_ == kChunkData || st_ == kChunkCrlf || st_ == kClose; }

 private:
  bool line_step(std::string_view line, bool* done) {
    switch (st_) {
      case kStatus: {
        if (line.empty()) return true;          // tolerate stray CRLF between messages
        if (line.size() < 12 || line.substr(0, 5) != "HTTP/") return false;
        status = 0;
        for (size_t k = 9; k < 12; ++k) {
          if (line[k] < '0' || line[k] > '9') return false;
          status = status * 10 + (line[k] - '0');
        }
        keep_alive = line.substr(5, 3) != "1.0";
        st_ = kHeaders;
        return true;
      }
      case kHeaders: {
        if (!line.empty()) return parse_header_line(line, headers);
        auto conn = headers.get("connection");
        if (iequals(conn, "close")) keep_alive = false;
        else if (iequals(conn, "keep-alive")) keep_alive = true;
        if (status / 100 == 1 || status == 204 || status == 304) {
          st_ = kDone;
          *done = true;
          return true;
        }
        if (iequals(headers.get("transfer-encoding"), "chunked")) {
          st_ = kChunkSize;
          return true;
        }
        auto cl = headers.get("content-length");
        if (!cl.empty()) {
          uint64_t v = 0;
          for (char c : cl) {
            if (c < '0' || c > '9') return false;
            v = v * 10 + uint64_t(c - '0');
          }
          remaining_ = v;
          if (v == 0) {
            st_ = kDone;
            *done = true;
          } else {
            st_ = kLen;
          }
          return true;
        }
        keep_alive = false;
        st_ = kClose;
        return true;
      }
      case kChunkSize: {
        uint64_t v = 0;
        size_t k = 0;
        for (; k < line.size(); ++k) {
          char c = line[k];
          int d = (c >= '0' && c <= '9') ? c - '0' : (c >= 'a' && c <= 'f') ? c - 'a' + 10
                  : (c >= 'A' && c <= 'F') ? c - 'A' + 10 : -1;
          if (d < 0) break;
          v = v * 16 + uint64_t(d);
        }
        if (k == 0) return false;
        if (v == 0) {
          st_ = kTrailers;
        } else {
          remaining_ = v;
          st_ = kChunkData;
        }
        return true;
      }
      case kChunkCrlf:
        st_ = kChunkSize;
        return line.empty();
      case kTrailers:
        if (line.empty()) {
          st_ = kDone;
          *done = true;
        }
        return true;
      default:
        return false;
    }
  }

  State st_ = kStatus;
  uint64_t remaining_ = 0;
  std::string line_;
};

// Request parser for the fake apiserver: request line, headers, Content-Length body.
struct Request {
  std::string method, target, path, query;
  Headers headers;
  std::string body;
  bool keep_alive = true;
};

class RequestParser {
 public:
  // Returns bytes consumed, sets *done when `req` is complete; -1 on a malformed request.
  long feed(const char* data, size_t n, bool* done, Request& req) {
    size_t i = 0;
    *done = false;
    while (i < n) {
      if (st_ == 2) {
        size_t take = std::min<uint64_t>(remaining_, n - i);
        req.body.append(data + i, take);
        i += take;
        remaining_ -= take;
        if (remaining_ == 0) {
          st_ = 0;
          *done = true;
          return long(i);
        }
        continue;
      }
      const char* nl = static_cast<const char*>(std::memchr(data + i, '\n', n - i));
      if (!nl) {
        line_.append(data + i, n - i);
        if (line_.size() > 65536) return -1;
        return long(n);
      }
      line_.append(data + i, size_t(nl - (data + i)));
      i = size_t(nl - data) + 1;
      std::string_view line(line_);
      if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
      if (st_ == 0) {
        if (line.empty()) {
          line_.clear();
          continue;
        }
        size_t a = line.find(' '), b = line.rfind(' ');
        if (a == std::string_view::npos || b == a) return -1;
        req = Request();
        req.method = std::string(line.substr(0, a));
        req.target = std::string(line.substr(a + 1, b - a - 1));
        req.keep_alive = line.substr(b + 1) != "HTTP/1.0";
        size_t q = req.target.find('?');
        req.path = req.target.substr(0, q);
        if (q != std::string::npos) req.query = req.target.substr(q + 1);
        st_ = 1;
      } else {
        if (!line.empty()) {
          if (!parse_header_line(line, req.headers)) return -1;
        } else {
          auto conn = req.headers.get("connection");
          if (iequals(conn, "close")) req.keep_alive = false;
          else if (iequals(conn, "keep-alive")) req.keep_alive = true;
          if (iequals(req.headers.get("transfer-encoding"), "chunked")) return -1;   // unsupported
          uint64_t v = 0;
          for (char c : req.headers.get("content-length")) {
            if (c < '0' || c > '9') return -1;
            v = v * 10 + uint64_t(c - '0');
          }
          line_.clear();
          if (v == 0) {
            st_ = 0;
            *done = true;
            return long(i);
          }
          if (v > (256u << 20)) return -1;
          remaining_ = v;
          req.body.reserve(v);
          st_ = 2;
          continue;
        }
      }
      line_.clear();
    }
    return long(i);
  }

 private:
  int st_ = 0;          // 0 request line, 1 headers, 2 body
  uint64_t remaining_ = 0;
  std::string line_;
};

inline int unhex(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

inline std::string url_decode(std::string_view s) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    char c = s[i];
    if (c == '+') {
      out.push_back(' ');
    } else if (c == '%' && i + 2 < s.size() && unhex(s[i + 1]) >= 0 && unhex(s[i + 2]) >= 0) {
      out.push_back(char(unhex(s[i + 1]) * 16 + unhex(s[i + 2])));
      i += 2;
    } else {
      out.push_back(c);
    }
  }
  return out;
}

inline void url_encode_into(std::string_view s, std::string& out) {
  static const char hx[] = "0123456789ABCDEF";
  for (unsigned char c : s) {
    if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '-' || c == '_' ||
        c == '.' || c == '~') {
      out.push_back(char(c));
    } else {
      out.push_back('%');
      out.push_back(hx[c >> 4]);
      out.push_back(hx[c & 15]);
    }
  }
}

inline std::string url_encode(std::string_view s) {
  std::string out;
  url_encode_into(s, out);
  return out;
}

// query "a=1&b=x%2Cy" → value of `key` (decoded), or `dflt`
inline std::string query_param(std::string_view q, std::string_view key, std::string_view dflt = {}) {
  while (!q.empty()) {
    size_t amp = q.find('&');
    std::string_view kv = q.substr(0, amp);
    size_t eq = kv.find('=');
    std::string_view k = kv.substr(0, eq);
    if (k == key) return eq == std::string_view::npos ? std::string() : url_decode(kv.substr(eq + 1));
    if (amp == std::string_view::npos) break;
    q.remove_prefix(amp + 1);
  }
  return std::string(dflt);
}

}  // namespace yk
