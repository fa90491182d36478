// Native Kubernetes API transport for the scheduler's hot path.
//
// One epoll I/O thread owns every socket: a pool of keep-alive connections carrying
// pipelined requests (binding POSTs, event writes, any other verb) and one dedicated
// connection per watch stream. Watch events are framed (chunked encoding → lines), parsed
// and — for pods — projected (project.hpp) on the I/O thread, so the Python event loop
// receives ready-to-use records in batches. Completions are handed over through a
// mutex-protected queue plus an eventfd the asyncio loop watches (`add_reader`).
//
// Replaces, for the hot path, the two client-go stacks the reference process runs
// (kube-scheduler's informers + binder and the controller-runtime cache;
// reference pkg/yoda/scheduler.go:53-73). HTTPS via OpenSSL (in-cluster CA, client
// certificates, insecure-skip-tls-verify), bearer token (rotatable), client-side QPS/burst
// token bucket with the semantics of client-go's flowcontrol limiter.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "lane_port.hpp"
#include "project.hpp"

struct ssl_ctx_st;

namespace yk {

struct ClientConfig {
  std::string host = "127.0.0.1";
  int port = 80;
  bool tls = false;
  std::string prefix;          // path prefix of the server URL ("" normally)
  std::string ca_file, cert_file, key_file;
  bool insecure = false;
  std::string token;
  int conns = 8;               // pooled request connections
  int max_inflight = 64;       // pipelined requests per connection
  double qps = 0.0;            // <= 0: unlimited
  int burst = 0;
  std::string user_agent = "yoda-scheduler/0.2 (MI355X)";
};

struct Completion {
  enum Kind : uint8_t { kResponse = 0, kEvents = 1, kWatchEnd = 2 };
  Kind kind = kResponse;
  uint64_t id = 0;
  int status = 0;              // HTTP status; -1 connection error, -2 timeout
  std::string body;
  std::string rv;              // kWatchEnd: resourceVersion of the stream's last event
  std::vector<WatchEvent> events;
};

struct TransportStats {
  uint64_t requests = 0, responses = 0, errors = 0, timeouts = 0, connects = 0;
  uint64_t watch_events = 0, watch_bytes = 0, parse_errors = 0, bytes_out = 0, bytes_in = 0;
  uint64_t throttled = 0;
  uint64_t slab_deletions = 0;
  uint64_t recycled = 0;         // pod events a sink handed back, freed on this (I/O) thread   // deletions left in their read buffer (PodEv::slab), not copied
  double watch_cpu_s = 0;     // I/O thread time decoding watch lines (parse + projection; monotonic clock, the decoder does not block)
  // lane Bindings: hand-off → written to a connection (queue), written → answer read (rtt)
  uint64_t sink_sent = 0, sink_answered = 0;
  double sink_queue_s = 0, sink_queue_max_s = 0, sink_rtt_s = 0, sink_rtt_max_s = 0;
};

// PodEv::complete for light events (flat re-parse of `raw`, full projection)
void complete_pod_ev(PodEv* e);

class Transport : public PodPort {
 public:
  explicit Transport(ClientConfig cfg);
  ~Transport();
  Transport(const Transport&) = delete;
  Transport& operator=(const Transport&) = delete;

  int fd() const { return out_efd_; }
  // Generic request. `limited`: goes through the QPS token bucket. timeout_s <= 0: none.
  uint64_t request(const std::string& method, const std::string& path, const std::string& body,
                   const std::string& content_type, bool limited, double timeout_s);
  // POST pods/{name}/binding with the body formatted here (rate-limited).
  uint64_t bind(const std::string& ns, const std::string& name, const std::string& uid, const std::string& node,
                const std::vector<KV>& annotations, double timeout_s);
  using BindSpec = yk::BindSpec;
  // A run of Bindings in one hand-off to the I/O thread (one lock, one wake-up); their
  // ids are consecutive: the first is returned.
  uint64_t bind_many(const std::vector<BindSpec>& binds, double timeout_s);
  // Streaming GET (watch=1 in `path`); `pods` selects the pod projection. The stream is
  // closed (kWatchEnd, status -1) when no byte arrived for idle_timeout_s (0 = never).
  uint64_t watch(const std::string& path, bool pods, double idle_timeout_s = 0.0);
  void cancel(uint64_t id);
  // Native pod lane (lane_port.hpp): every pod watch event goes to `sink` first; nullptr
  // detaches it (waits for a sink call in progress). Answers of requests submitted for a
  // sink that is no longer attached are dropped.
  void set_pod_sink(PodSink* sink);
  void recycle(std::vector<std::shared_ptr<PodEv>>&& dead) override;
  void bind_native(std::vector<BindSpec>&& binds, const std::vector<uint64_t>& tags, double timeout_s,
                   PodSink* sink) override;
  void request_native(const std::string& method, const std::string& path, std::string&& body, bool limited,
                      double timeout_s, uint64_t tag, PodSink* sink, const char* content_type = nullptr) override;
  std::vector<Completion> drain();
  void set_token(const std::string& token);
  // client QPS / burst (clientConnection); qps <= 0 disables limiting
  void set_rate(double qps, int burst);
  TransportStats stats();
  void close();

  struct Conn;
  struct Req;

 private:
  void run();
  void submit(std::unique_ptr<Req> r);
  void append_bind_body(std::string& b, const std::string& ns, const std::string& name, const std::string& uid,
                        const std::string& node, const std::vector<KV>& annotations,
                        std::string_view ann_json = {});
  void bind_wire(const BindSpec& s, std::string& wire);
  std::string bind_body(const std::string& ns, const std::string& name, const std::string& uid,
                        const std::string& node, const std::vector<KV>& annotations);
  std::string head(const std::string& method, const std::string& path, size_t body_len,
                   const std::string& content_type);
  std::unique_ptr<Conn> open_conn(bool watch);
  void close_conn(Conn* c, int status, const std::string& why);
  void on_event(Conn* c, uint32_t ev);
  void do_handshake(Conn* c);
  void do_read(Conn* c);
  void do_write(Conn* c);
  void update_interest(Conn* c);
  void on_body(Conn* c, const char* data, size_t n);
  void on_message_done(Conn* c);
  void watch_lines(Conn* c);
  void dispatch();
  void check_timeouts(double now);
  void complete(Completion&& c);
  void answer(Req& r, int status, std::string&& body);   // completion or sink answer
  void offer_pod_events(Conn* c);
  void flush_answers();
  void flush();

  ClientConfig cfg_;
  ssl_ctx_st* ssl_ctx_ = nullptr;
  std::vector<uint8_t> addr_;              // resolved sockaddr
  int family_ = 0;
  int ep_ = -1, wake_efd_ = -1, out_efd_ = -1;
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::atomic<uint64_t> next_id_{1};

  std::mutex in_mu_;
  std::vector<std::unique_ptr<Req>> incoming_;
  std::vector<uint64_t> cancels_;
  std::mutex recycle_mu_;
  std::vector<std::shared_ptr<PodEv>> recycle_;   // dropped on the I/O thread (recycle())
  std::string bind_hdr_, bind_hdr_token_;   // bind_wire's constant header lines (in_mu_)
  std::string token_;

  std::mutex out_mu_;
  std::vector<Completion> out_;
  std::vector<Completion> local_out_;      // I/O thread: batched before the handover

  // I/O-thread state
  std::deque<std::unique_ptr<Req>> throttled_, ready_;
  std::vector<std::unique_ptr<Conn>> pool_;
  std::unordered_map<uint64_t, std::unique_ptr<Conn>> watches_;
  std::atomic<double> qps_{0.0};
  std::atomic<int> burst_{0};
  std::atomic<bool> refill_{false};
  double tokens_ = 0.0, last_refill_ = 0.0;
  double next_timeout_check_ = 0.0;

  std::mutex stats_mu_;
  TransportStats stats_;

  std::mutex sink_mu_;                     // held around every sink call (I/O thread)
  PodSink* pod_sink_ = nullptr;
  std::atomic<bool> light_pods_{false};    // a sink is attached: MODIFIED/DELETED decoded light
  std::vector<PodSink::Answer> sink_answers_;   // I/O thread: answers for the sink, per loop turn
  PodSink* answers_for_ = nullptr;
};

}  // namespace yk
