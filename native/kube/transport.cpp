// Native Kubernetes API transport (see transport.hpp).
#include "transport.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <pthread.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>

#include "flatjson.hpp"
#include "http.hpp"
#include "json.hpp"

namespace yk {

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void efd_signal(int fd) {
  uint64_t one = 1;
  ssize_t r = ::write(fd, &one, sizeof(one));
  (void)r;
}

void efd_clear(int fd) {
  uint64_t v;
  ssize_t r = ::read(fd, &v, sizeof(v));
  (void)r;
}

std::string ssl_error_text() {
  unsigned long e = ERR_get_error();
  if (!e) return "tls error";
  char buf[256];
  ERR_error_string_n(e, buf, sizeof(buf));
  return buf;
}

bool is_ip_literal(const std::string& h) {
  unsigned char buf[16];
  return inet_pton(AF_INET, h.c_str(), buf) == 1 || inet_pton(AF_INET6, h.c_str(), buf) == 1;
}

}  // namespace

struct Transport::Req {
  uint64_t id = 0;
  std::string wire;
  bool limited = false;
  bool watch = false;
  bool pods = false;
  PodSink* sink = nullptr;  // native lane request: answered through sink->on_answer(tag)
  uint64_t tag = 0;
  bool expired = false;     // completed by timeout; the late response is dropped
  double deadline = 0.0;
  double idle_timeout = 0.0;  // watch: close when nothing arrived for this long (0 = never)
  double t_submit = 0.0;      // lane Bindings: handed to the transport / written to a connection
  double t_sent = 0.0;
};

struct Transport::Conn {
  int fd = -1;
  SSL* ssl = nullptr;
  enum State { kConnecting, kHandshake, kOpen, kDead } st = kConnecting;
  bool watch = false;
  bool pods = false;
  uint64_t watch_id = 0;
  bool watch_cancelled = false;
  std::string wbuf;
  size_t woff = 0;
  std::deque<std::unique_ptr<Req>> inflight;
  ResponseParser rp;
  std::string body;          // current response body (or a watch's error body)
  std::string lines;         // watch: undecoded stream bytes
  std::vector<WatchEvent> evs;
  uint32_t interest = 0;
  bool registered = false;
  double last_rx = 0.0;      // last time bytes arrived (watch idle timeout)
  std::string last_rv;       // watch: resourceVersion of the last event handed to the pod sink
  double idle_timeout = 0.0;
};

Transport::Transport(ClientConfig cfg) : cfg_(std::move(cfg)) {
  if (cfg_.conns < 1) cfg_.conns = 1;
  if (cfg_.max_inflight < 1) cfg_.max_inflight = 1;
  token_ = cfg_.token;
  // resolve once (the apiserver address does not move under a running scheduler)
  addrinfo hints{};
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_family = AF_UNSPEC;
  addrinfo* res = nullptr;
  std::string port = std::to_string(cfg_.port);
  std::string host = cfg_.host;
  if (host.size() > 2 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  cfg_.host = host;
  int rc = getaddrinfo(host.c_str(), port.c_str(), &hints, &res);
  if (rc != 0 || !res) throw std::runtime_error("resolve " + host + ": " + gai_strerror(rc));
  addr_.assign(reinterpret_cast<uint8_t*>(res->ai_addr), reinterpret_cast<uint8_t*>(res->ai_addr) + res->ai_addrlen);
  family_ = res->ai_family;
  freeaddrinfo(res);

  if (cfg_.tls) {
    ssl_ctx_ = SSL_CTX_new(TLS_client_method());
    if (!ssl_ctx_) throw std::runtime_error("SSL_CTX_new: " + ssl_error_text());
    SSL_CTX_set_min_proto_version(ssl_ctx_, TLS1_2_VERSION);
    SSL_CTX_set_mode(ssl_ctx_, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
    if (cfg_.insecure) {
      SSL_CTX_set_verify(ssl_ctx_, SSL_VERIFY_NONE, nullptr);
    } else {
      SSL_CTX_set_verify(ssl_ctx_, SSL_VERIFY_PEER, nullptr);
      if (!cfg_.ca_file.empty()) {
        if (SSL_CTX_load_verify_locations(ssl_ctx_, cfg_.ca_file.c_str(), nullptr) != 1)
          throw std::runtime_error("CA " + cfg_.ca_file + ": " + ssl_error_text());
      } else {
        SSL_CTX_set_default_verify_paths(ssl_ctx_);
      }
    }
    if (!cfg_.cert_file.empty() && !cfg_.key_file.empty()) {
      if (SSL_CTX_use_certificate_chain_file(ssl_ctx_, cfg_.cert_file.c_str()) != 1 ||
          SSL_CTX_use_PrivateKey_file(ssl_ctx_, cfg_.key_file.c_str(), SSL_FILETYPE_PEM) != 1)
        throw std::runtime_error("client certificate: " + ssl_error_text());
    }
  }
  ep_ = epoll_create1(EPOLL_CLOEXEC);
  wake_efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  out_efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (ep_ < 0 || wake_efd_ < 0 || out_efd_ < 0) throw std::runtime_error("epoll/eventfd setup failed");
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.ptr = nullptr;
  epoll_ctl(ep_, EPOLL_CTL_ADD, wake_efd_, &ev);
  qps_ = cfg_.qps;
  burst_ = cfg_.burst;
  tokens_ = cfg_.burst > 0 ? cfg_.burst : 1;
  last_refill_ = now_s();
  th_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "yoda-io");   // per-thread CPU in bench / top -H
    run();
  });
}

Transport::~Transport() { close(); }

void Transport::close() {
  if (!stop_.exchange(true)) {
    efd_signal(wake_efd_);
    if (th_.joinable()) th_.join();
    for (auto& c : pool_) {
      if (c->ssl) SSL_free(c->ssl);
      if (c->fd >= 0) ::close(c->fd);
    }
    pool_.clear();
    for (auto& kv : watches_) {
      if (kv.second->ssl) SSL_free(kv.second->ssl);
      if (kv.second->fd >= 0) ::close(kv.second->fd);
    }
    watches_.clear();
    if (ssl_ctx_) SSL_CTX_free(ssl_ctx_);
    ssl_ctx_ = nullptr;
    ::close(ep_);
    ::close(wake_efd_);
    ::close(out_efd_);
  }
}

std::string Transport::head(const std::string& method, const std::string& path, size_t body_len,
                            const std::string& content_type) {
  std::string h;
  h.reserve(256 + path.size());
  h.append(method).append(" ").append(cfg_.prefix).append(path).append(" HTTP/1.1\r\nHost: ");
  if (cfg_.host.find(':') != std::string::npos) h.append("[").append(cfg_.host).append("]");
  else h.append(cfg_.host);
  h.append(":").append(std::to_string(cfg_.port)).append("\r\nUser-Agent: ").append(cfg_.user_agent);
  h.append("\r\nAccept: application/json\r\n");
  {
    std::lock_guard<std::mutex> g(in_mu_);
    if (!token_.empty()) h.append("Authorization: Bearer ").append(token_).append("\r\n");
  }
  if (body_len || method == "POST" || method == "PUT" || method == "PATCH") {
    h.append("Content-Type: ").append(content_type.empty() ? "application/json" : content_type);
    h.append("\r\nContent-Length: ").append(std::to_string(body_len)).append("\r\n");
  }
  h.append("\r\n");
  return h;
}

void Transport::submit(std::unique_ptr<Req> r) {
  bool was_empty;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    was_empty = incoming_.empty() && cancels_.empty();
    incoming_.push_back(std::move(r));
  }
  if (was_empty) efd_signal(wake_efd_);
}

uint64_t Transport::request(const std::string& method, const std::string& path, const std::string& body,
                            const std::string& content_type, bool limited, double timeout_s) {
  auto r = std::make_unique<Req>();
  r->id = next_id_++;
  r->wire = head(method, path, body.size(), content_type);
  r->wire.append(body);
  r->limited = limited;
  r->deadline = timeout_s > 0 ? now_s() + timeout_s : 0.0;
  uint64_t id = r->id;
  submit(std::move(r));
  return id;
}

std::string Transport::bind_body(const std::string& ns, const std::string& name, const std::string& uid,
                                 const std::string& node, const std::vector<KV>& annotations) {
  std::string b;
  b.reserve(256);
  append_bind_body(b, ns, name, uid, node, annotations);
  return b;
}

void Transport::append_bind_body(std::string& b, const std::string& ns, const std::string& name,
                                 const std::string& uid, const std::string& node,
                                 const std::vector<KV>& annotations, std::string_view ann_json) {
  b.append("{\"apiVersion\":\"v1\",\"kind\":\"Binding\",\"metadata\":{\"name\":");
  dump_string(name, b);
  b.append(",\"namespace\":");
  dump_string(ns, b);
  b.append(",\"uid\":");
  dump_string(uid, b);
  b.append(",\"annotations\":{");
  b.append(ann_json);
  for (size_t i = 0; ann_json.empty() && i < annotations.size(); ++i) {
    if (i) b.push_back(',');
    dump_string(annotations[i].first, b);
    b.push_back(':');
    dump_string(annotations[i].second, b);
  }
  b.append("}},\"target\":{\"apiVersion\":\"v1\",\"kind\":\"Node\",\"name\":");
  dump_string(node, b);
  b.append("}}");
}

// A Binding POST in one buffer: request line, headers, body. The body goes into a per-thread
// scratch first (its length is a header); the header lines that do not change between
// requests (head()'s, for a POST of application/json) are built once per token.
void Transport::bind_wire(const BindSpec& s, std::string& wire) {
  thread_local std::string body;
  body.clear();
  append_bind_body(body, s.ns, s.name, s.uid, s.node, s.annotations, s.ann_json);
  char len[32];
  char* le = std::to_chars(len, len + 20, body.size()).ptr;
  memcpy(le, "\r\n\r\n", 4);
  const int nl = int(le + 4 - len);
  wire.reserve(320 + cfg_.prefix.size() + s.ns.size() + s.name.size() + body.size());
  wire.append("POST ").append(cfg_.prefix).append("/api/v1/namespaces/");
  url_encode_into(s.ns, wire);
  wire.append("/pods/");
  url_encode_into(s.name, wire);
  wire.append("/binding HTTP/1.1\r\n");
  {
    std::lock_guard<std::mutex> g(in_mu_);
    if (bind_hdr_.empty() || bind_hdr_token_ != token_) {
      std::string& h = bind_hdr_;
      h.clear();
      h.append("Host: ");
      if (cfg_.host.find(':') != std::string::npos) h.append("[").append(cfg_.host).append("]");
      else h.append(cfg_.host);
      h.append(":").append(std::to_string(cfg_.port)).append("\r\nUser-Agent: ").append(cfg_.user_agent);
      h.append("\r\nAccept: application/json\r\n");
      if (!token_.empty()) h.append("Authorization: Bearer ").append(token_).append("\r\n");
      h.append("Content-Type: application/json\r\nContent-Length: ");
      bind_hdr_token_ = token_;
    }
    wire.append(bind_hdr_);
  }
  wire.append(len, size_t(nl)).append(body);
}

uint64_t Transport::bind(const std::string& ns, const std::string& name, const std::string& uid,
                         const std::string& node, const std::vector<KV>& annotations, double timeout_s) {
  std::string b = bind_body(ns, name, uid, node, annotations);
  std::string path = "/api/v1/namespaces/" + url_encode(ns) + "/pods/" + url_encode(name) + "/binding";
  return request("POST", path, b, "application/json", true, timeout_s);
}

uint64_t Transport::bind_many(const std::vector<BindSpec>& binds, double timeout_s) {
  if (binds.empty()) return 0;
  const uint64_t first = next_id_.fetch_add(binds.size());
  const double deadline = timeout_s > 0 ? now_s() + timeout_s : 0.0;
  std::vector<std::unique_ptr<Req>> rs;
  rs.reserve(binds.size());
  for (size_t k = 0; k < binds.size(); ++k) {
    const BindSpec& s = binds[k];
    auto r = std::make_unique<Req>();
    r->id = first + k;
    bind_wire(s, r->wire);
    r->limited = true;
    r->deadline = deadline;
    rs.push_back(std::move(r));
  }
  bool was_empty;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    was_empty = incoming_.empty() && cancels_.empty();
    for (auto& r : rs) incoming_.push_back(std::move(r));
  }
  if (was_empty) efd_signal(wake_efd_);
  return first;
}

void Transport::recycle(std::vector<std::shared_ptr<PodEv>>&& dead) {
  if (dead.empty()) return;
  bool wake;
  {
    std::lock_guard<std::mutex> g(recycle_mu_);
    if (recycle_.empty()) {
      recycle_.swap(dead);
    } else {
      recycle_.reserve(recycle_.size() + dead.size());
      for (auto& d : dead) recycle_.push_back(std::move(d));
    }
    wake = recycle_.size() >= 16384;      // an idle I/O thread would otherwise hold them a while
  }
  dead.clear();
  if (wake) efd_signal(wake_efd_);
}

void Transport::bind_native(std::vector<BindSpec>&& binds, const std::vector<uint64_t>& tags, double timeout_s,
                            PodSink* sink) {
  if (binds.empty()) return;
  const double t_submit = now_s();
  const double deadline = timeout_s > 0 ? t_submit + timeout_s : 0.0;
  std::vector<std::unique_ptr<Req>> rs;
  rs.reserve(binds.size());
  for (size_t k = 0; k < binds.size(); ++k) {
    const BindSpec& s = binds[k];
    auto r = std::make_unique<Req>();
    r->id = next_id_++;
    bind_wire(s, r->wire);
    r->limited = true;
    r->deadline = deadline;
    r->sink = sink;
    r->tag = k < tags.size() ? tags[k] : 0;
    r->t_submit = t_submit;
    rs.push_back(std::move(r));
  }
  bool was_empty;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    was_empty = incoming_.empty() && cancels_.empty();
    for (auto& r : rs) incoming_.push_back(std::move(r));
  }
  if (was_empty) efd_signal(wake_efd_);
}

void Transport::request_native(const std::string& method, const std::string& path, std::string&& body,
                               bool limited, double timeout_s, uint64_t tag, PodSink* sink, const char* content_type) {
  auto r = std::make_unique<Req>();
  r->id = next_id_++;
  // PATCH bodies are JSON merge patches (an event's series) unless the caller names the type
  // (the PodScheduled condition is a strategic merge patch, conditions merged by type)
  r->wire = head(method, path, body.size(),
                 content_type ? content_type : method == "PATCH" ? "application/merge-patch+json" : "application/json");
  r->wire.append(body);
  r->limited = limited;
  r->deadline = timeout_s > 0 ? now_s() + timeout_s : 0.0;
  r->sink = sink;
  r->tag = tag;
  submit(std::move(r));
}

void Transport::set_pod_sink(PodSink* sink) {
  std::lock_guard<std::mutex> g(sink_mu_);
  pod_sink_ = sink;
  light_pods_.store(sink != nullptr, std::memory_order_relaxed);
}

void complete_pod_ev(PodEv* e) {
  e->materialize();
  PodProj full;
  FlatDoc d;
  if (d.parse(e->raw)) project_pod(d.root(), full);
  if (e->p.ident_partial) {            // a deletion scanned to metadata only
    e->p.sched = full.sched.empty() ? "default-scheduler" : full.sched;
    e->p.node = full.node;
    e->p.phase = full.phase;
    e->p.ident_partial = false;
  }
  merge_non_identity(e->p, std::move(full));
}

void Transport::answer(Req& r, int status, std::string&& body) {
  if (r.sink) {
    if (r.t_sent > 0) {
      const double rtt = now_s() - r.t_sent;
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.sink_rtt_s += rtt;
      stats_.sink_rtt_max_s = std::max(stats_.sink_rtt_max_s, rtt);
      stats_.sink_answered++;
    }
    // delivered at flush(), in one batch per loop turn, if the sink is still attached
    if (answers_for_ != r.sink && !sink_answers_.empty()) flush_answers();
    answers_for_ = r.sink;
    sink_answers_.push_back(PodSink::Answer{r.tag, status, std::move(body), now_s()});
    return;
  }
  Completion e;
  e.kind = Completion::kResponse;
  e.id = r.id;
  e.status = status;
  e.body = std::move(body);
  complete(std::move(e));
}

void Transport::flush_answers() {
  if (sink_answers_.empty()) return;
  {
    std::lock_guard<std::mutex> g(sink_mu_);
    if (answers_for_ == pod_sink_ && pod_sink_) pod_sink_->on_answers(sink_answers_);
  }
  sink_answers_.clear();
  answers_for_ = nullptr;
}

void Transport::offer_pod_events(Conn* c) {
  if (!c->pods || c->evs.empty()) return;
  std::lock_guard<std::mutex> g(sink_mu_);
  if (!pod_sink_) return;
  // the reflector resumes from the stream's last resourceVersion, which the sink's events
  // no longer show it: the watch-end completion carries it (Completion::rv)
  for (auto it = c->evs.rbegin(); it != c->evs.rend(); ++it)
    if (!it->rv.empty()) {
      c->last_rv = it->rv;
      break;
    }
  pod_sink_->on_pod_events(c->watch_id, c->evs);
}

uint64_t Transport::watch(const std::string& path, bool pods, double idle_timeout_s) {
  auto r = std::make_unique<Req>();
  r->id = next_id_++;
  r->wire = head("GET", path, 0, "");
  r->watch = true;
  r->pods = pods;
  r->idle_timeout = idle_timeout_s;
  uint64_t id = r->id;
  submit(std::move(r));
  return id;
}

void Transport::cancel(uint64_t id) {
  bool was_empty;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    was_empty = incoming_.empty() && cancels_.empty();
    cancels_.push_back(id);
  }
  if (was_empty) efd_signal(wake_efd_);
}

void Transport::set_rate(double qps, int burst) {
  qps_ = qps;
  burst_ = burst;
  refill_ = true;          // a (re)configured bucket starts full, like a new client-go limiter
  efd_signal(wake_efd_);
}

void Transport::set_token(const std::string& token) {
  std::lock_guard<std::mutex> g(in_mu_);
  token_ = token;
}

std::vector<Completion> Transport::drain() {
  efd_clear(out_efd_);
  std::vector<Completion> v;
  std::lock_guard<std::mutex> g(out_mu_);
  v.swap(out_);
  return v;
}

TransportStats Transport::stats() {
  std::lock_guard<std::mutex> g(stats_mu_);
  return stats_;
}

void Transport::complete(Completion&& c) { local_out_.push_back(std::move(c)); }

void Transport::flush() {
  flush_answers();
  if (local_out_.empty()) return;
  bool was_empty;
  {
    std::lock_guard<std::mutex> g(out_mu_);
    was_empty = out_.empty();
    if (was_empty) {
      out_.swap(local_out_);
    } else {
      for (auto& c : local_out_) out_.push_back(std::move(c));
    }
  }
  local_out_.clear();
  if (was_empty) efd_signal(out_efd_);
}

// ------------------------------------------------------------------ connections
std::unique_ptr<Transport::Conn> Transport::open_conn(bool watch) {
  int fd = ::socket(family_, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return nullptr;
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  setsockopt(fd, SOL_SOCKET, SO_KEEPALIVE, &one, sizeof(one));
  // a black-holed peer (LB / apiserver failover) is detected in ~60 s like Go's dialer
  // (30 s keep-alive), not after the kernel's 2 h default
  int idle = 30, intvl = 10, cnt = 3;
  setsockopt(fd, IPPROTO_TCP, TCP_KEEPIDLE, &idle, sizeof(idle));
  setsockopt(fd, IPPROTO_TCP, TCP_KEEPINTVL, &intvl, sizeof(intvl));
  setsockopt(fd, IPPROTO_TCP, TCP_KEEPCNT, &cnt, sizeof(cnt));
  int rc = ::connect(fd, reinterpret_cast<const sockaddr*>(addr_.data()), socklen_t(addr_.size()));
  if (rc != 0 && errno != EINPROGRESS) {
    ::close(fd);
    return nullptr;
  }
  auto c = std::make_unique<Conn>();
  c->fd = fd;
  c->watch = watch;
  c->st = Conn::kConnecting;
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.connects++;
  }
  update_interest(c.get());
  return c;
}

void Transport::update_interest(Conn* c) {
  uint32_t want = EPOLLIN | EPOLLRDHUP;
  if (c->st == Conn::kConnecting || (c->woff < c->wbuf.size())) want |= EPOLLOUT;
  if (c->st == Conn::kHandshake) want = EPOLLIN | EPOLLOUT;
  if (c->registered && want == c->interest) return;
  epoll_event ev{};
  ev.events = want;
  ev.data.ptr = c;
  epoll_ctl(ep_, c->registered ? EPOLL_CTL_MOD : EPOLL_CTL_ADD, c->fd, &ev);
  c->registered = true;
  c->interest = want;
}

void Transport::close_conn(Conn* c, int status, const std::string& why) {
  if (c->st == Conn::kDead) return;
  c->st = Conn::kDead;
  if (c->registered) epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
  if (c->ssl) {
    SSL_free(c->ssl);
    c->ssl = nullptr;
  }
  ::close(c->fd);
  c->fd = -1;
  if (c->watch) {
    if (!c->watch_cancelled) {
      offer_pod_events(c);
      if (!c->evs.empty()) {
        Completion ce;
        ce.kind = Completion::kEvents;
        ce.id = c->watch_id;
        ce.events.swap(c->evs);
        complete(std::move(ce));
      }
      Completion e;
      e.kind = Completion::kWatchEnd;
      e.id = c->watch_id;
      e.status = status;
      e.body = why;
      e.rv = c->last_rv;
      complete(std::move(e));
    }
    return;
  }
  uint64_t failed = 0;
  for (auto& r : c->inflight) {
    if (r->expired) continue;
    answer(*r, status, std::string(why));
    failed++;
  }
  c->inflight.clear();
  if (failed) {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.errors += failed;
  }
}

void Transport::do_handshake(Conn* c) {
  int r = SSL_connect(c->ssl);
  if (r == 1) {
    c->st = Conn::kOpen;
    update_interest(c);
    do_write(c);
    return;
  }
  int e = SSL_get_error(c->ssl, r);
  if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return;
  close_conn(c, -1, "tls handshake: " + ssl_error_text());
}

void Transport::do_write(Conn* c) {
  if (c->st != Conn::kOpen) return;
  size_t sent = 0;
  while (c->woff < c->wbuf.size()) {
    const char* p = c->wbuf.data() + c->woff;
    size_t n = c->wbuf.size() - c->woff;
    long w;
    if (c->ssl) {
      w = SSL_write(c->ssl, p, int(std::min<size_t>(n, 1 << 20)));
      if (w <= 0) {
        int e = SSL_get_error(c->ssl, int(w));
        if (e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) break;
        close_conn(c, -1, "tls write: " + ssl_error_text());
        return;
      }
    } else {
      w = ::send(c->fd, p, n, MSG_NOSIGNAL);
      if (w < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        close_conn(c, -1, std::string("write: ") + strerror(errno));
        return;
      }
    }
    c->woff += size_t(w);
    sent += size_t(w);
  }
  if (c->woff >= c->wbuf.size()) {
    c->wbuf.clear();
    c->woff = 0;
  } else if (c->woff > (1u << 20)) {
    c->wbuf.erase(0, c->woff);
    c->woff = 0;
  }
  if (sent) {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.bytes_out += sent;
  }
  update_interest(c);
}

void Transport::on_body(Conn* c, const char* data, size_t n) {
  if (c->watch && c->rp.status == 200) {
    c->lines.append(data, n);
    watch_lines(c);
  } else {
    c->body.append(data, n);
  }
}


namespace {
// time inside the decoder (it never blocks, so this is its CPU time bar preemption): the
// monotonic clock is read in the vDSO, while CLOCK_THREAD_CPUTIME_ID is a system call —
// two per read turn cost the I/O thread 10-20 % of its time when the scheduler keeps up and
// each turn decodes one or two events (native sampler, profiles/bench/r6/natprof/)
double decode_clock_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + ts.tv_nsec * 1e-9;
}
}  // namespace

void Transport::watch_lines(Conn* c) {
  // one flat parse per event line ({"type":..., "object":{...}}): no per-value allocation;
  // pods are projected from the same document (project.hpp)
  const double cpu0 = decode_clock_s();
  size_t start = 0;
  uint64_t nev = 0, nerr = 0, nslab = 0;
  FlatDoc doc;
  // the read buffer as a view: deletions may take the buffer itself over as their shared slab
  // (PodEv::slab), after which the unconsumed tail is copied back into c->lines
  std::string_view buf(c->lines);
  std::shared_ptr<const std::string> slab;
  while (true) {
    size_t nl = buf.find('\n', start);
    if (nl == std::string::npos) break;
    std::string_view line(buf.data() + start, nl - start);
    start = nl + 1;
    bool blank = true;
    for (char ch : line)
      if (ch != ' ' && ch != '\r' && ch != '\t') {
        blank = false;
        break;
      }
    if (blank) continue;
    std::shared_ptr<PodEv> pe;
    if (c->pods && light_pods_.load(std::memory_order_relaxed)) {
      // echoes and deletions with a lane attached: the identity fields by one skipping scan,
      // the rest of the pod on demand (PodEv::full); other types stop at the type member
      char t = 0;
      std::string_view obj;
      pe = std::make_shared<PodEv>();
      static const bool scan_all = getenv("YODA_WATCH_SCAN_ALL") != nullptr;   // A/B: the old full scan
      static const bool copy_del = getenv("YODA_WATCH_COPY_DELETIONS") != nullptr;   // A/B: copy every text
      if (scan_watch_identity(line, &t, &obj, pe->p, !scan_all) && (t == 'M' || t == 'D')) {
        WatchEvent ev;
        ev.type = t;
        ev.rv = pe->p.rv;
        pe->light = true;
        pe->complete = &complete_pod_ev;
        if (t == 'D' && !copy_del && (slab || c->lines.size() >= 4096)) {
          if (!slab) {
            // moving a heap-held string keeps its buffer: `buf` and `line` stay valid
            auto own = std::make_shared<std::string>(std::move(c->lines));
            c->lines.clear();
            slab = std::move(own);
          }
          pe->slab = slab;
          pe->slab_off = uint32_t(obj.data() - slab->data());
          pe->slab_len = uint32_t(obj.size());
          nslab++;
        } else {
          pe->raw.assign(obj.data(), obj.size());
        }
        ev.pod = std::move(pe);
        c->evs.push_back(std::move(ev));
        nev++;
        continue;
      }
    }
    if (!doc.parse(line) || !doc.root().is(FlatDoc::Obj)) {
      nerr++;
      continue;
    }
    const FlatDoc::View root = doc.root();
    const FlatDoc::View tv = root.get("type");
    const FlatDoc::View obj = root.get("object");
    if (!tv || !tv.is(FlatDoc::Str) || !obj) {
      nerr++;
      continue;
    }
    const std::string_view type = tv.str();
    WatchEvent ev;
    ev.type = type == "ADDED" ? 'A' : type == "MODIFIED" ? 'M' : type == "DELETED" ? 'D'
              : type == "BOOKMARK" ? 'B' : type == "ERROR" ? 'E' : '?';
    if (ev.type == '?') {
      nerr++;
      continue;
    }
    if (const FlatDoc::View m = obj.get("metadata")) ev.rv = std::string(m.sv("resourceVersion"));
    const std::string_view raw = obj.raw();
    if (c->pods && ev.type != 'B' && ev.type != 'E') {
      if (pe) pe->p = PodProj();
      else pe = std::make_shared<PodEv>();
      if (ev.type != 'A' && light_pods_.load(std::memory_order_relaxed)) {
        // echoes and deletions: the lane reads identity fields only; the rest on demand
        project_identity(obj, pe->p);
        pe->light = true;
        pe->complete = &complete_pod_ev;
      } else if (light_pods_.load(std::memory_order_relaxed)) {
        // with a lane attached the spec / metadata hash is computed only if something compares
        // it (PodEv::hash: Python's update check of a forwarded pod, the lane's of a queued one)
        project_pod_nohash(obj, pe->p);
        pe->hash_of = &spec_meta_hash_of;
      } else {
        project_pod(obj, pe->p);
      }
      pe->raw.assign(raw.data(), raw.size());
      ev.pod = std::move(pe);
    } else if (ev.type != 'B') {
      ev.raw.assign(raw.data(), raw.size());
    }
    c->evs.push_back(std::move(ev));
    nev++;
  }
  if (slab) c->lines.assign(buf.data() + start, buf.size() - start);
  else if (start) c->lines.erase(0, start);
  if (nev || nerr) {
    const double dc = decode_clock_s() - cpu0;
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.watch_events += nev;
    stats_.slab_deletions += nslab;
    stats_.parse_errors += nerr;
    stats_.watch_cpu_s += dc;
  }
}

void Transport::on_message_done(Conn* c) {
  if (c->watch) {
    // server ended the watch (timeoutSeconds) or refused it: the reflector re-watches or relists
    int st = c->rp.status;
    std::string body = st == 200 ? std::string() : std::move(c->body);
    c->body.clear();
    close_conn(c, st, body);
    return;
  }
  if (c->inflight.empty()) {
    close_conn(c, -1, "unsolicited response");
    return;
  }
  std::unique_ptr<Req> r = std::move(c->inflight.front());
  c->inflight.pop_front();
  if (!r->expired) answer(*r, c->rp.status, std::move(c->body));
  c->body.clear();
  {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.responses++;
  }
  bool ka = c->rp.keep_alive;
  c->rp.reset();
  if (!ka) close_conn(c, -1, "connection closed by server");
}

// bytes of a watch stream decoded per I/O loop turn before requests get their turn
// (YODA_WATCH_READ_SLICE overrides; 0 = read until the socket is drained)
static size_t watch_read_slice() {
  static const size_t v = [] {
    const char* e = getenv("YODA_WATCH_READ_SLICE");
    if (!e || !*e) return size_t(32) << 10;
    const long long x = atoll(e);
    return x > 0 ? size_t(x) : ~size_t(0);
  }();
  return v;
}

void Transport::do_read(Conn* c) {
  char buf[65536];
  size_t got_total = 0;
  while (c->st == Conn::kOpen) {
    long n;
    if (c->ssl) {
      n = SSL_read(c->ssl, buf, sizeof(buf));
      if (n <= 0) {
        int e = SSL_get_error(c->ssl, int(n));
        if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) break;
        if (e == SSL_ERROR_ZERO_RETURN) n = 0;
        else {
          close_conn(c, -1, "tls read: " + ssl_error_text());
          return;
        }
      }
    } else {
      n = ::recv(c->fd, buf, sizeof(buf), 0);
      if (n < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK) break;
        close_conn(c, -1, std::string("read: ") + strerror(errno));
        return;
      }
    }
    if (n == 0) {
      if (c->rp.finish_on_close()) {
        on_message_done(c);
        if (c->st == Conn::kDead) return;
      }
      close_conn(c, c->watch ? 200 : -1, c->watch ? "" : "connection closed by server");
      return;
    }
    got_total += size_t(n);
    c->last_rx = now_s();
    size_t off = 0;
    while (off < size_t(n) && c->st == Conn::kOpen) {
      bool done = false;
      long used = c->rp.feed(buf + off, size_t(n) - off, &done,
                             [&](const char* d, size_t k) { on_body(c, d, k); });
      if (used < 0) {
        close_conn(c, -1, "malformed HTTP response");
        return;
      }
      off += size_t(used);
      if (done) {
        on_message_done(c);
      }
    }
    if (c->watch && !c->evs.empty() && c->st == Conn::kOpen) offer_pod_events(c);
    if (c->watch && !c->evs.empty() && c->st == Conn::kOpen) {
      Completion ce;
      ce.kind = Completion::kEvents;
      ce.id = c->watch_id;
      ce.events.swap(c->evs);
      complete(std::move(ce));
    }
    // a watch stream with a backlog (a burst's ADDED events) would keep this thread here until
    // it drains, while the lane's Bindings wait to be written and their answers to be read:
    // hand back to the loop after a slice (epoll is level-triggered, the rest is read next
    // turn). TLS keeps reading: bytes OpenSSL already buffered raise no further epoll event.
    if (c->watch && !c->ssl && got_total >= watch_read_slice()) break;
  }
  if (got_total) {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.bytes_in += got_total;
    if (c->watch) stats_.watch_bytes += got_total;
  }
}

void Transport::on_event(Conn* c, uint32_t ev) {
  if (c->st == Conn::kDead) return;
  if (c->st == Conn::kConnecting) {
    if (ev & (EPOLLOUT | EPOLLERR | EPOLLHUP)) {
      int err = 0;
      socklen_t len = sizeof(err);
      getsockopt(c->fd, SOL_SOCKET, SO_ERROR, &err, &len);
      if (err) {
        close_conn(c, -1, std::string("connect: ") + strerror(err));
        return;
      }
      if (ssl_ctx_) {
        c->ssl = SSL_new(ssl_ctx_);
        SSL_set_fd(c->ssl, c->fd);
        if (!is_ip_literal(cfg_.host)) SSL_set_tlsext_host_name(c->ssl, cfg_.host.c_str());
        if (!cfg_.insecure) {
          X509_VERIFY_PARAM* vp = SSL_get0_param(c->ssl);
          if (is_ip_literal(cfg_.host)) X509_VERIFY_PARAM_set1_ip_asc(vp, cfg_.host.c_str());
          else X509_VERIFY_PARAM_set1_host(vp, cfg_.host.c_str(), 0);
        }
        c->st = Conn::kHandshake;
        update_interest(c);
        do_handshake(c);
      } else {
        c->st = Conn::kOpen;
        update_interest(c);
        do_write(c);
      }
    }
    return;
  }
  if (c->st == Conn::kHandshake) {
    do_handshake(c);
    return;
  }
  if (ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) do_read(c);
  if (c->st == Conn::kOpen && (ev & EPOLLOUT)) do_write(c);
}

// ------------------------------------------------------------------ scheduling of requests
void Transport::dispatch() {
  double now = now_s();
  const double qps = qps_.load();
  if (refill_.exchange(false)) tokens_ = burst_.load() > 0 ? burst_.load() : 1;
  if (qps > 0) {
    double cap = burst_.load() > 0 ? burst_.load() : 1;
    tokens_ = std::min(cap, tokens_ + (now - last_refill_) * qps);
    last_refill_ = now;
    while (!throttled_.empty() && tokens_ >= 1.0) {
      tokens_ -= 1.0;
      ready_.push_back(std::move(throttled_.front()));
      throttled_.pop_front();
    }
  } else {
    while (!throttled_.empty()) {
      ready_.push_back(std::move(throttled_.front()));
      throttled_.pop_front();
    }
  }
  // drop dead pooled connections
  pool_.erase(std::remove_if(pool_.begin(), pool_.end(), [](const std::unique_ptr<Conn>& c) { return c->st == Conn::kDead; }),
              pool_.end());
  std::vector<Conn*> touched;
  while (!ready_.empty()) {
    Conn* best = nullptr;
    for (auto& c : pool_) {
      if (c->st == Conn::kDead) continue;
      if (int(c->inflight.size()) >= cfg_.max_inflight) continue;
      if (!best || c->inflight.size() < best->inflight.size()) best = c.get();
    }
    if ((!best || !best->inflight.empty()) && int(pool_.size()) < cfg_.conns) {
      if (auto n = open_conn(false)) {
        best = n.get();
        pool_.push_back(std::move(n));
      }
    }
    if (!best) break;          // every connection is full: wait for responses
    std::unique_ptr<Req> r = std::move(ready_.front());
    ready_.pop_front();
    best->wbuf.append(r->wire);
    if (r->t_submit > 0) {
      r->t_sent = now;
      const double q = now - r->t_submit;
      std::lock_guard<std::mutex> g(stats_mu_);
      stats_.sink_queue_s += q;
      stats_.sink_queue_max_s = std::max(stats_.sink_queue_max_s, q);
      stats_.sink_sent++;
    }
    r->wire.clear();
    r->wire.shrink_to_fit();
    best->inflight.push_back(std::move(r));
    if (std::find(touched.begin(), touched.end(), best) == touched.end()) touched.push_back(best);
  }
  for (Conn* c : touched) {
    if (c->st == Conn::kOpen) do_write(c);
    else update_interest(c);
  }
}

void Transport::check_timeouts(double now) {
  uint64_t n = 0;
  auto expire = [&](Req& r) {
    answer(r, -2, std::string("request timed out"));
    r.expired = true;
    n++;
  };
  for (auto* q : {&throttled_, &ready_}) {
    for (auto it = q->begin(); it != q->end();) {
      if ((*it)->deadline > 0 && now > (*it)->deadline) {
        expire(**it);
        it = q->erase(it);
      } else {
        ++it;
      }
    }
  }
  for (auto& c : pool_) {
    if (c->st == Conn::kDead || c->inflight.empty()) continue;
    bool oldest_expired = false;
    for (auto& r : c->inflight)
      if (!r->expired && r->deadline > 0 && now > r->deadline) {
        if (&r == &c->inflight.front()) oldest_expired = true;
        expire(*r);
      }
    // the connection's oldest request got no answer in time: responses are ordered, so
    // everything pipelined behind it is stuck too — close it, failing those requests now
    // (their callers retry), and let dispatch() open a fresh connection for the slot
    if (oldest_expired) close_conn(c.get(), -1, "connection closed: an earlier request on it timed out");
  }
  for (auto& kv : watches_) {
    Conn* c = kv.second.get();
    if (c->st != Conn::kDead && c->idle_timeout > 0 && now - c->last_rx > c->idle_timeout)
      close_conn(c, -1, "watch idle timeout");     // the reflector re-watches / relists
  }
  if (n) {
    std::lock_guard<std::mutex> g(stats_mu_);
    stats_.timeouts += n;
  }
}

void Transport::run() {
  epoll_event evs[128];
  while (!stop_.load()) {
    int timeout_ms = 200;
    const double qps = qps_.load();
    if (!throttled_.empty() && qps > 0) {
      double wait = (1.0 - tokens_) / qps;
      timeout_ms = std::max(0, std::min(timeout_ms, int(wait * 1000.0) + 1));
    }
    if (!local_out_.empty()) timeout_ms = 0;
    int n = epoll_wait(ep_, evs, 128, timeout_ms);
    if (n < 0 && errno != EINTR) break;
    {
      // pod events the lane finished with: freed here, before this turn decodes new ones
      std::vector<std::shared_ptr<PodEv>> dead;
      {
        std::lock_guard<std::mutex> g(recycle_mu_);
        dead.swap(recycle_);
      }
      if (!dead.empty()) {
        std::lock_guard<std::mutex> g(stats_mu_);
        stats_.recycled += dead.size();
      }
    }
    bool woke = false;
    for (int i = 0; i < n; ++i) {
      if (evs[i].data.ptr == nullptr) {
        woke = true;
        continue;
      }
      on_event(static_cast<Conn*>(evs[i].data.ptr), evs[i].events);
    }
    if (woke) {
      efd_clear(wake_efd_);
      // the rate read before epoll_wait may predate a set_rate() that came with this wake-up
      const double qps = qps_.load();
      std::vector<std::unique_ptr<Req>> in;
      std::vector<uint64_t> cancels;
      {
        std::lock_guard<std::mutex> g(in_mu_);
        in.swap(incoming_);
        cancels.swap(cancels_);
      }
      for (auto& r : in) {
        {
          std::lock_guard<std::mutex> g(stats_mu_);
          stats_.requests++;
          if (r->limited && qps > 0 && (!throttled_.empty() || tokens_ < 1.0)) stats_.throttled++;
        }
        if (r->watch) {
          auto c = open_conn(true);
          if (!c) {
            Completion e;
            e.kind = Completion::kWatchEnd;
            e.id = r->id;
            e.status = -1;
            e.body = std::string("connect: ") + strerror(errno);
            complete(std::move(e));
            continue;
          }
          c->watch_id = r->id;
          c->pods = r->pods;
          c->idle_timeout = r->idle_timeout;
          c->last_rx = now_s();
          c->wbuf = std::move(r->wire);
          watches_[r->id] = std::move(c);
          continue;
        }
        if (r->limited && qps > 0) throttled_.push_back(std::move(r));
        else ready_.push_back(std::move(r));
      }
      for (uint64_t id : cancels) {
        auto it = watches_.find(id);
        if (it != watches_.end()) {
          it->second->watch_cancelled = true;
          close_conn(it->second.get(), 0, "cancelled");
        }
      }
    }
    dispatch();
    // reap finished watch connections
    for (auto it = watches_.begin(); it != watches_.end();) {
      if (it->second->st == Conn::kDead) it = watches_.erase(it);
      else ++it;
    }
    double now = now_s();
    if (now >= next_timeout_check_) {
      check_timeouts(now);
      next_timeout_check_ = now + 0.05;
    }
    flush();
  }
  // fail everything still pending
  for (auto* q : {&throttled_, &ready_}) {
    for (auto& r : *q) answer(*r, -1, std::string("transport closed"));
    q->clear();
  }
  for (auto& c : pool_) close_conn(c.get(), -1, "transport closed");
  for (auto& kv : watches_) close_conn(kv.second.get(), -1, "transport closed");
  flush();
}

}  // namespace yk
