// The seam between the native transport (module _yoda_kube) and the native pod lane (module
// _yoda_core). Header-only abstract interfaces: each side calls the other through a vtable,
// so neither module links the other's code, and Python only hands raw pointers across
// (Transport.port_ptr() → Lane, Lane.sink_ptr() → Transport.set_pod_sink()).
//
//   transport I/O thread ──on_pod_events──► lane (takes every pod watch event)
//   lane thread ──bind_native / request_native──► transport (Bindings, Scheduled events)
//   transport I/O thread ──on_answers──► lane (the apiserver's answers, by tag, per loop turn)
//
// Both callbacks run on the transport's I/O thread with the transport's sink lock held;
// they must only enqueue (never block, never call back into the transport).
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "project.hpp"

namespace yk {

struct PodEv {
  PodProj p;
  std::string raw;             // the pod object's JSON text
  // A deletion's text stays in the watch read buffer it arrived in (shared by the deletions
  // of that read) instead of being copied out: the lane drops a lane-owned pod's deletion
  // unread. materialize() copies it into `raw` — the lane does before handing the event to
  // Python, and complete() (full()) does before projecting. Lane thread / under `once` only.
  std::shared_ptr<const std::string> slab;
  uint32_t slab_off = 0, slab_len = 0;
  void materialize() {
    if (slab) {
      raw.assign(slab->data() + slab_off, slab_len);
      slab.reset();
    }
  }
  std::string_view raw_view() const {
    return slab ? std::string_view(slab->data() + slab_off, slab_len) : std::string_view(raw);
  }
  // A "light" event carries only the identity fields (ns, name, uid, rv, node, scheduler,
  // phase, deletion, creation) — what the lane reads of a Binding's echo or a deletion. The
  // rest (labels, requests, selectors, flags, spec/metadata hash, ok) is projected from `raw`
  // on first use through full(), once, thread-safely; identity fields are never rewritten.
  bool light = false;
  void (*complete)(PodEv*) = nullptr;
  mutable std::once_flag once;
  const PodProj& full() const {
    if (light && complete) std::call_once(once, [this] { complete(const_cast<PodEv*>(this)); });
    return p;
  }
  // spec_meta_hash, computed from `raw` on first use when the decode skipped it (hash_pending);
  // the decoder (the transport, in the kube module) sets the function, as it does `complete`
  uint64_t (*hash_of)(std::string_view raw) = nullptr;
  mutable std::once_flag hash_once;
  uint64_t hash() const {
    const PodProj& f = full();
    std::call_once(hash_once, [this, &f] {
      if (f.hash_pending && hash_of) {
        PodProj& m = const_cast<PodProj&>(f);
        m.spec_meta_hash = hash_of(raw);
        m.hash_pending = false;
      }
    });
    return f.spec_meta_hash;
  }
};

struct WatchEvent {
  char type = 0;               // 'A' ADDED, 'M' MODIFIED, 'D' DELETED, 'B' BOOKMARK, 'E' ERROR
  std::string rv;
  std::string raw;             // object JSON (non-pod watches; ERROR status for pods too)
  std::shared_ptr<PodEv> pod;  // pod watches
};

struct BindSpec {
  std::string ns, name, uid, node;
  std::vector<KV> annotations;
  // the annotations as serialised JSON object members (`"k":"v",...`), used instead of
  // `annotations` when set: the lane writes them in one buffer (no per-key allocations)
  std::string ann_json;
};

class PodSink {
 public:
  virtual ~PodSink() = default;
  // A decoded batch of a pod watch. The sink moves the pod events it wants out of `evs`
  // (erasing them); what is left (bookmarks, errors, and any pod event it declines) goes
  // to the Python informer as before, in order.
  virtual void on_pod_events(uint64_t watch_id, std::vector<WatchEvent>& evs) = 0;
  // Answers to requests submitted through PodPort with this sink, batched per I/O loop turn
  // (one hand-off and at most one wake-up of the consumer per turn, not one per response):
  // HTTP status, or -1 (connection failed / closed) / -2 (timed out) with a reason in `body`.
  struct Answer {
    uint64_t tag;
    int status;
    std::string body;
    double t = 0;              // steady-clock seconds when the I/O thread read the answer (0: unknown)
  };
  virtual void on_answers(std::vector<Answer>& answers) = 0;
};

class PodPort {
 public:
  virtual ~PodPort() = default;
  // Binding POSTs (client rate limit applies), answered through sink->on_answers (tags[k]).
  virtual void bind_native(std::vector<BindSpec>&& binds, const std::vector<uint64_t>& tags, double timeout_s,
                           PodSink* sink) = 0;
  // Any other request (events, pod status); answered through sink->on_answers (tag). A PATCH
  // body is a JSON merge patch unless `content_type` names another patch type.
  virtual void request_native(const std::string& method, const std::string& path, std::string&& body,
                              bool limited, double timeout_s, uint64_t tag, PodSink* sink,
                              const char* content_type = nullptr) = 0;
  // Pod events the sink is done with, handed back so that their last reference drops on the
  // thread that allocated them (the I/O thread): freed there, their memory returns to that
  // thread's malloc cache instead of contending for its arena from the sink's thread.
  virtual void recycle(std::vector<std::shared_ptr<PodEv>>&& dead) { dead.clear(); }
};

}  // namespace yk
