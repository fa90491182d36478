// Native pod lane: the per-pod scheduling lifecycle in C++.
//
// What upstream kube-scheduler does in compiled Go for the reference plugin — informer →
// activeQ → scheduleOne → assume → async bind → confirm on the watch echo → forget on
// delete (the reference only supplies Filter/Score, /root/reference/pkg/yoda/scheduler.go:76-130)
// — runs here for every pod of an all-native profile without a Python call per pod:
//
//   transport I/O thread ── every pod watch event ──► Lane inbox
//   lane thread: store update → admission → priority queue → Engine::schedule_batch (assume)
//                → Binding POSTs straight to the transport → answers / echo / delete
//   Python event loop: only what the lane forwards — pods of other profiles or with features
//                a Python plugin handles, unschedulable pods a PostFilter (preemption) may
//                help, bind failures — pulled in batches through an eventfd.
//
// Unschedulable pods no PostFilter can help (the profile has none, or DefaultPreemption and the
// pod's priority cannot preempt) stay in the lane, as upstream's queue keeps them in compiled Go
// (/root/reference/pkg/yoda/scheduler.go:85-92 → FitError; deploy/yoda-scheduler.yaml:19-20):
// a FailedScheduling event and the PodScheduled=False condition from C++, then unschedulableQ
// (PARKED) or podBackoffQ (BACKOFF, initial × 2^(attempts−1) capped at max), moved back on
// cluster events — a lane release, any Python move request, and per-node Scv hints that re-run
// the pod's filters on that node only — with upstream's moveRequestCycle rule and the periodic
// leftover flush.
//
// The lane owns the pod store (key → latest projected event), so the Python informer keeps no
// per-pod state for lane pods; a relist is diffed here too. Scheduling semantics match the
// Python runner's all-native batch path (same engine call, same assume, same annotations);
// the queue is the profile's QueueSort (scv/priority label or spec.priority) with a FIFO
// tie-break. The Python queue and the lane queue are independent: a pod is in exactly one.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <queue>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "engine.hpp"
#include "lane_port.hpp"

namespace yoda {

struct LaneOptions {
  int batch = 256;                 // pods per engine batch
  double bind_timeout_s = 30.0;
  int sort_kind = 0;               // 0: scv/priority label (yoda QueueSort), 1: spec.priority (PrioritySort)
  // Scheduled events (upstream EventRecorder semantics, native)
  bool events = true;
  bool events_v1 = true;           // events.k8s.io/v1 shape (else core/v1)
  double event_qps = 50.0;
  int event_burst = 300;
  int event_buffer = 1000;         // pending events kept; a full buffer drops the incoming one
  std::string host = "localhost";
  std::string name_prefix = "00000000";
  size_t e2e_keep = 1 << 20;       // raw e2e samples kept until Python takes them
  // runs on an engine worker thread, the lane serving its inbox (answers, echoes, deletions)
  // meanwhile: 0 never, 1 when the engine has a device scorer (the GPU places the batch),
  // 2 always (tests of the in-flight paths)
  int async_mode = 1;
  int engine_delay_us = 0;         // tests: widen the in-flight window of every run
  // async runs: the lane thread (run out) and the engine worker (between runs) busy-wait this
  // long for their next item before sleeping on the condition variable (0: never spin)
  int spin_us = 0;
  // queue timing (podInitialBackoffSeconds, podMaxBackoffSeconds, unschedulableQ leftover flush)
  double initial_backoff_s = 1.0, max_backoff_s = 10.0, unsched_flush_s = 60.0;
};

// metav1.LabelSelector + the namespaces it applies in (a pod (anti-)affinity term, a topology
// spread selector): models/selectors.py::LabelSelector semantics (nil matches nothing, {} all).
struct MatchTerm {
  std::vector<std::string> namespaces;   // empty: every namespace
  bool nothing = false;                  // nil selector
  std::vector<std::pair<std::string, std::string>> labels;
  struct Expr {
    std::string key;
    int op = 0;                          // 0 In, 1 NotIn, 2 Exists, 3 DoesNotExist
    std::vector<std::string> values;
    bool operator==(const Expr& o) const { return op == o.op && key == o.key && values == o.values; }
  };
  std::vector<Expr> exprs;
  bool operator==(const MatchTerm& o) const {
    return nothing == o.nothing && namespaces == o.namespaces && labels == o.labels && exprs == o.exprs;
  }
  bool matches(const std::string& ns, const std::vector<std::pair<std::string, std::string>>& labels) const;
  bool matches(const yk::PodProj& p) const { return matches(p.ns, p.labels); }
};

struct LaneStats {
  uint64_t admitted = 0, scheduled = 0, unschedulable = 0, bind_errors = 0, stale_retries = 0;
  uint64_t forwarded = 0, released = 0, batches = 0, confirmed = 0, events_recorded = 0, events_dropped = 0;
  uint64_t events_written = 0, event_errors = 0, lost_answers_kept = 0;
  uint64_t queued = 0, inflight = 0, binding = 0, owned = 0;   // gauges
  uint64_t parked = 0, backoff = 0;                            // gauges: unschedulableQ, podBackoffQ
  uint64_t native_failed = 0;      // of `unschedulable`: kept in the lane (no PostFilter could help)
  uint64_t moved = 0, retried = 0; // pods moved by move requests; pods back from backoff to the queue
  uint64_t status_patches = 0, status_patch_errors = 0;
  uint64_t status_patches_skipped = 0;   // the pod's condition already said the same (upstream updatePod)
  uint64_t census_calls = 0, census_entries = 0;   // count_matching: calls, reserved pods walked
  double census_s = 0;
  uint64_t left_in_flight = 0;   // pods gone (deleted, bound elsewhere) while their run was on the engine
  double engine_s = 0;        // wall time inside Engine::schedule_batch (lane thread)
  double engine_cpu_s = 0;    // ... of which on the CPU (the rest: the engine lock, the device)
  double lock_wait_s = 0;     // waiting for the engine lock before a run
  uint64_t engine_pods = 0;   // pods those calls placed or rejected
  // async runs: picked → worker start, worker end → lane completes them, and the engine
  // worker's idle time between runs while pods that arrived before the last run ended waited
  double handoff_s = 0, return_s = 0, idle_queued_s = 0;
  uint64_t async_runs = 0;
  // per profile: (pods scheduled, unschedulable attempts kept native) — the attempts metric
  std::unordered_map<std::string, std::pair<uint64_t, uint64_t>> by_profile;
};

class Lane : public yk::PodSink {
 public:
  enum St : uint8_t { PY = 0, QUEUED, INFLIGHT, BINDING, BOUND, PARKED, BACKOFF };

  struct Profile {
    std::string name;
    bool enabled = false;
    int flag_mask = 0;       // a pod with any of these flags goes to Python
    bool annotate = true;    // yoda filter in the profile: the Binding carries the GPU assignment
    // an unschedulable pod whose spec.priority is above this goes to Python (its PostFilter —
    // DefaultPreemption — may act); at or below it the lane fails it natively. INT64_MIN: every
    // unschedulable pod goes to Python; INT64_MAX: none (no PostFilter that can act)
    int64_t preempt_above = INT64_MIN;
    // bound pods' required anti-affinity terms (InterPodAffinity's symmetric rule): a pod
    // matching any of them goes to Python, where that rule is checked; the others are unaffected
    std::vector<MatchTerm> gate_terms;
    // a pod whose only flag in flag_mask is PF_CLAIMS is admissible when every claim it mounts
    // is in the inert set (set_inert_claims): the profile's volume plugins are all no-ops for
    // it (plugins/volumes.py::inert_claims), so its cycle is the native one
    bool claims_ok = false;
    // VolumeBinding / VolumeZone are enabled: a bound claim's PV node affinity / zone labels
    // (the claim table's constraints) are engine filters of the pod's cycle
    bool vol_node = false, vol_zone = false;
    bool vol_limits = false;   // NodeVolumeLimits is enabled: the pods' PVC volumes count against CSI limits
    EngineConfig cfg;
  };
  // What VolumeBinding and VolumeZone check of one bound claim (plugins/volumes.py::claim_lane):
  // the PV's nodeAffinity terms and its zone / region labels as node-affinity terms, OR'ed
  struct ClaimCons {
    bool has_node = false, has_zone = false;
    std::vector<SelTerm> node, zone;
    bool operator==(const ClaimCons& o) const {
      return has_node == o.has_node && has_zone == o.has_zone && node == o.node && zone == o.zone;
    }
  };
  using ClaimConsP = std::shared_ptr<const ClaimCons>;

  // What the Python informer sees of a forwarded pod event: type 'A'/'M'/'D', the event,
  // and the previous event of the key (nullptr for a new one).
  struct Fwd {
    char type;
    std::shared_ptr<yk::PodEv> ev, old;
  };
  // A pod the lane gives up to the Python path.
  struct Handoff {
    // kRequeue: a waiting pod (unschedulableQ / podBackoffQ) the lane may no longer run (a gate or
    // profile change): Python requeues it into backoff with its attempts, no new FailedScheduling
    enum Kind : int { kUnschedulable = 0, kBindError = 1, kRequeue = 2 };
    int kind = 0;
    std::shared_ptr<yk::PodEv> ev;
    std::string profile;
    CycleResult res;         // kUnschedulable: the engine's cycle (reasons for FitError)
    int status = 0;          // kBindError: HTTP status / -1 / -2
    std::string msg;
    double t_enqueue = 0;    // monotonic seconds, when the pod entered the lane queue
    double t_cycle = 0;
    uint32_t attempts = 1;   // scheduling attempts so far (the Python queue's backoff continues)
  };

  Lane(Engine* e, std::recursive_mutex* engine_mu, LaneOptions o);
  ~Lane() override;
  Lane(const Lane&) = delete;
  Lane& operator=(const Lane&) = delete;

  // ---- configuration (Python thread)
  void set_port(yk::PodPort* p) { port_.store(p); }
  void set_profile(const Profile& p);          // replaces a profile of the same name
  // only the selector gates of a declared profile (no engine-config snapshot); false if the
  // lane has no profile of that name
  bool set_gates(const std::string& name, std::vector<MatchTerm> terms);
  // the PersistentVolumeClaims ("namespace/name") the volume plugins have nothing to check for;
  // waiting pods mounting a claim that left the set go to Python
  void set_inert_claims(std::vector<std::string> keys);
  // the same set changed by a few claims (a PVC / PV event): O(change), not O(claims)
  void update_inert_claims(std::vector<std::string> add, std::vector<std::string> remove);
  // the claim table: every claim the lane may admit, with the constraints its PV puts on nodes
  // (null: none). `reset`: `add` is the whole table. A claim that leaves it or whose
  // constraints change sends the waiting lane pods that mount it to Python
  void update_claims(bool reset, std::vector<std::pair<std::string, ClaimConsP>> add,
                     std::vector<std::string> remove);
  void set_active(bool on);                    // leader: schedule; otherwise only keep the store
  void set_node_cards(const std::string& node, std::vector<std::pair<std::string, std::string>> vis);
  void remove_node_cards(const std::string& node);
  void close();

  // ---- yk::PodSink (transport I/O thread)
  void on_pod_events(uint64_t watch_id, std::vector<yk::WatchEvent>& evs) override;
  void on_answers(std::vector<yk::PodSink::Answer>& answers) override;

  // ---- Python side
  int fileno() const { return efd_; }
  void drain(std::vector<Fwd>* fwd, std::vector<Handoff>* hand, uint64_t* moves);
  // A relist's items (full state of the pod collection): diffed against the store on the
  // lane thread; returns the events Python must see. Blocks until processed.
  std::vector<Fwd> relist(std::vector<std::shared_ptr<yk::PodEv>> items);
  std::shared_ptr<yk::PodEv> lookup(const std::string& key, bool* owned);
  // a lane-owned pod by its engine ledger id (the event and its node), or null
  std::shared_ptr<yk::PodEv> lookup_id(uint64_t id, std::string* node);
  std::vector<std::string> keys();
  size_t store_size();
  LaneStats stats();
  std::vector<float> take_e2e();
  std::vector<float> take_pod_latency();
  void wait_idle(double timeout_s);            // tests: inbox and queue drained
  // Hold the lane thread between steps (a Python what-if on the ledger — preemption —
  // must not interleave with lane releases); blocks until the thread is parked.
  void pause(bool on);
  // A move request (upstream MoveAllToActiveOrBackoffQueue): node < 0 moves every parked pod;
  // node >= 0 is a queueing hint for that node (its Scv grew): only parked pods that now pass
  // every filter there move. Applied on the lane thread in order with its other input.
  void move(int32_t node);

  // The lane pods holding a reservation, for the Python cache's view of the cluster (pod
  // affinity / spread / preemption plugins). The first call returns the full set and turns
  // on a change log; later calls return what changed since (add: id, event, node, cards;
  // remove: id). `full` is set when the log overflowed and the set is complete again.
  // The log is coalesced by ledger id (a release cancels an add Python has not taken yet),
  // so it never holds more than the live lane pods plus the releases of pods Python saw;
  // stop_log() turns it off again (Python dropped its mirror: nothing reads it any more).
  struct Change {
    uint64_t id;
    bool add;
    std::shared_ptr<yk::PodEv> ev;
    std::string node;
    std::vector<int32_t> cards;
  };
  std::vector<Change> changes(bool* full);
  // Lane pods holding a reservation (assumed or bound) that match every term of a query, counted
  // per node — what InterPodAffinity and PodTopologySpread read of them, without a Python mirror.
  // skip_deleting: leave out pods with a deletionTimestamp (spread's countPodsMatchSelector).
  std::vector<std::unordered_map<std::string, int32_t>> count_matching(
      const std::vector<std::vector<MatchTerm>>& queries, bool skip_deleting);
  // The census behind count_matching is kept only while queried: the first query builds it,
  // stop_census() (Python, after a settle window without queries) drops it.
  void stop_census();
  void stop_log();
  bool log_on();

 private:
  struct Entry {
    std::shared_ptr<yk::PodEv> ev;
    St st = PY;
    uint64_t id = 0;         // engine ledger id while lane-owned
    int prof = -1;
    int64_t prio = 0;
    uint64_t seq = 0;
    double t_enq = 0, t_cycle = 0;
    int32_t node = -1;
    std::string node_name;
    std::vector<int32_t> cards;
    bool confirmed = false;  // the watch echo showed the pod bound to node_name
    bool acked = false;      // the Binding POST was answered 2xx
    bool bind_out = false;   // a Binding POST is in flight (no answer yet)
    uint32_t attempts = 0;   // scheduling attempts (incremented when picked)
    uint64_t cycle = 0;      // the lane's scheduling cycle of the last pick
    double t_fail = 0;       // when the last attempt failed (backoff counts from here)
    double t_park = 0;       // when it entered unschedulableQ
    uint64_t bseq = 0;       // backoff heap item of this entry (stale items are skipped)
    std::shared_ptr<PodReq> req;   // the request of the failed attempt (move hints re-filter with it)
    // the PodScheduled=False condition this lane last wrote for the pod (message and
    // lastTransitionTime): what the pod says until the write's echo arrives
    std::string cond_msg, cond_ltt;
    // a reserved pod's event whose labels are current: later watch echoes keep it while their
    // labels hash says the labels did not change, so the selector census never projects them
    std::shared_ptr<yk::PodEv> lab_ev;
    int32_t crow = -1;       // row in census_ (reserved pods, while the census is on)
  };
  struct QItem {             // max-heap: higher priority first, then FIFO
    int64_t prio;
    uint64_t seq;
    uint64_t id;             // entry id; an item whose entry moved on is skipped when popped
    bool operator<(const QItem& o) const { return prio != o.prio ? prio < o.prio : seq > o.seq; }
  };
  // one engine batch of consecutive same-profile pods (engine_step fills the second half)
  struct Run {
    int prof = -1;
    Profile pr;                                      // a copy: profiles may change meanwhile
    EngineConfig cfg;
    double t0 = 0;
    double t_wstart = 0, t_wend = 0;                 // on the engine worker (async)
    std::vector<uint64_t> ids;                       // entry ids, run order
    std::vector<std::shared_ptr<yk::PodEv>> evs;
    std::vector<PodReq> reqs;
    std::vector<char> ok;                            // projection expressible natively
    std::vector<size_t> slot;                        // run index of each engine batch member
    std::vector<CycleResult> res;
    std::vector<std::string> names;
    std::vector<uint64_t> cycles;                    // each pod's scheduling cycle (pick order)
    std::vector<char> hinted;                        // per result: a node hint since its cycle fits it
    std::vector<std::vector<ClaimConsP>> vols;       // per pod: its claims' constraints (claim table)
    std::vector<char> vol_ok;                        // per pod: every claim was in the table
    bool failed = false;
  };
  struct Item {             // inbox: events, answers, commands — applied in order
    enum K : uint8_t { kEvent, kAnswer, kRelist, kProfiles, kRunDone, kMove, kGates, kClaims } k = kEvent;
    char type = 0;
    std::shared_ptr<yk::PodEv> ev;
    uint64_t tag = 0;
    int status = 0;
    std::string body;
    double t = 0;             // answers: when the I/O thread read it
    std::shared_ptr<std::vector<std::shared_ptr<yk::PodEv>>> items;
    uint64_t token = 0;
    std::shared_ptr<std::vector<std::shared_ptr<Run>>> runs;   // kRunDone
  };
  struct PendingEvent {
    std::string ns, name, uid, node, profile;
    double ts;
    std::string note;        // empty: Scheduled ("Successfully assigned ... to <node>")
  };

  void run();
  void handle_event(char type, const std::shared_ptr<yk::PodEv>& ev, std::vector<Fwd>* out);
  void handle_answer(uint64_t tag, int status, std::string& body, double t_ack);
  void handle_relist(const std::vector<std::shared_ptr<yk::PodEv>>& items, std::vector<Fwd>* out);
  void apply_gates(std::vector<Fwd>* out);
  void drop_owned(Entry* e, bool release);
  // a waiting (PARKED / BACKOFF) entry leaves for the Python queue keeping attempts and backoff
  void requeue_to_python(Entry* e);
  void apply_profiles(std::vector<Fwd>* out);
  void count(St s, int d);
  void set_state(Entry* e, St s);
  void bind_settled(Entry* e);
  void schedule_some();
  void engine_step(Run& r);
  void finish_run(Run& r, std::vector<yk::BindSpec>* binds, std::vector<uint64_t>* tags, std::vector<Fwd>* fwd);
  void complete_runs(std::vector<std::shared_ptr<Run>>& runs);
  void engine_worker();
  bool admissible(const yk::PodProj& p, int* prof) const;
  int64_t prio_of(const yk::PodProj& p) const;
  bool make_req(const yk::PodProj& p, PodReq* r);
  Labels intern_labels(const std::vector<std::pair<std::string, std::string>>& kv);   // engine lock held
  void annotations(const Profile& pr, const Entry& e, const PodReq& req, const CycleResult& r,
                   std::string* out);
  void record_scheduled(const Entry& e);
  // native unschedulable path
  void fail_native(Entry* e, const Profile& pr, const CycleResult& res, bool hinted);
  void to_backoff(Entry* e, double until);
  void activate(Entry* e);
  void route(Entry* e, double now);
  double backoff_of(const Entry& e) const;
  void move_parked(const std::vector<Entry*>& which);
  void process_moves();
  void flush_queues(double now);
  bool hinted_since(uint64_t cycle, const PodReq& req);
  double next_timer() const;
  std::string fit_error(const CycleResult& r, const yk::PodProj& p) const;
  void patch_condition(Entry& e, const std::string& msg);
  void flush_events();
  void forward(char type, std::shared_ptr<yk::PodEv> ev, std::shared_ptr<yk::PodEv> old, std::vector<Fwd>* out);
  void publish(std::vector<Fwd>&& fwd, std::vector<Handoff>&& hand);
  void signal_python();
  static double mono();
  static double thread_cpu();   // this thread's CPU seconds

  Engine* eng_;
  std::recursive_mutex* emu_;
  LaneOptions o_;
  std::atomic<yk::PodPort*> port_{nullptr};
  int efd_ = -1;
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> active_{false};

  std::mutex in_mu_;
  std::condition_variable in_cv_;
  std::deque<Item> inbox_;
  uint64_t relist_next_ = 0, relist_done_ = 0;
  std::condition_variable relist_cv_;
  std::unordered_map<uint64_t, std::vector<Fwd>> relist_out_;
  bool busy_ = false;                // lane thread is processing (wait_idle)
  bool paused_ = false;
  bool run_inflight_ = false;        // runs on the engine worker (in_mu_)
  // the last runs' timeline (diagnostics): pick, worker start, worker end, lane completion, pods
 public:
  struct RunRec {
    double t_pick, t_wstart, t_wend, t_done;
    uint32_t pods;
  };
  std::vector<RunRec> run_log();          // and clear it
 private:
  std::mutex rlog_mu_;
  std::vector<RunRec> rlog_;
  std::atomic<bool> inbox_flag_{false};   // inbox_ non-empty (set under in_mu_, read spinning)
  std::atomic<bool> wk_flag_{false};      // wk_jobs_ non-empty (set under wk_mu_)
  void push_locked(Item&& it);            // inbox_.push_back under in_mu_
  void spin_until(const std::atomic<bool>& flag) const;
  double last_wend_ = 0;             // when the engine worker finished the last async run (lane thread)

  // engine worker (async device runs)
  std::thread wk_th_;
  std::mutex wk_mu_;
  std::condition_variable wk_cv_;
  std::vector<std::shared_ptr<Run>> wk_jobs_;
  std::condition_variable idle_cv_;

  // selector census of reserved lane pods (count_matching): one contiguous row per pod with its
  // namespace and label (key, key=value) hashes, scanned per query without touching the
  // entries; rows whose labels changed are re-derived lazily at the next query (store_mu_)
  static constexpr int kCLab = 6;
  struct CRow {
    Entry* e = nullptr;
    uint64_t ns = 0;
    uint32_t node = 0;       // cnode_names_ index
    bool deleting = false, dirty = true, big = false;
    uint8_t n = 0;
    uint64_t k[kCLab], kv[kCLab];
  };
  bool census_on_ = false;
  std::vector<CRow> census_;
  std::vector<std::string> cnode_names_;
  std::unordered_map<std::string, uint32_t> cnode_ids_;
  void census_add(Entry* e);
  void census_remove(Entry* e);
  void census_fill(CRow& r);

  // change log of reserved lane pods (changes()); off until Python first asks
  std::mutex log_mu_;
  bool log_on_ = false, log_full_ = false;
  std::vector<Change> log_;
  std::unordered_map<uint64_t, size_t> log_adds_;   // id → index in log_ of an add Python has not taken
  size_t log_dead_ = 0;                             // cancelled adds (id 0) in log_
  void log_add(const Entry& e);
  void log_remove(uint64_t id);

  std::mutex prof_mu_;
  std::vector<Profile> profiles_;    // copied into lane-thread state on kProfiles
  // set_gates: per profile, the terms a gate update added (only those can make a waiting pod
  // inadmissible); taken by the lane thread on kGates (prof_mu_)
  std::vector<std::pair<std::string, std::vector<MatchTerm>>> gate_adds_;
  std::vector<Profile> lp_;          // lane thread's view
  // set_inert_claims / update_inert_claims, in call order; taken by the lane thread on kClaims
  // (prof_mu_)
  struct ClaimOp {
    bool reset = false;                     // `add` is the whole table
    std::vector<std::pair<std::string, ClaimConsP>> add;
    std::vector<std::string> remove;
  };
  std::vector<ClaimOp> claim_ops_;
  std::unordered_map<std::string, ClaimConsP> claim_table_;   // lane thread's view of the claim table
  bool claims_in_table(const yk::PodProj& p) const;
  // a picked pod's claims' constraints (run formation, lane thread); false if a claim is not in
  // the table (the pod goes to Python)
  bool claim_cons(const yk::PodProj& p, std::vector<ClaimConsP>* out) const;
  void apply_claims(std::vector<Fwd>* out);

  std::mutex vis_mu_;
  std::unordered_map<std::string, std::vector<std::pair<std::string, std::string>>> vis_;

  // store: written by the lane thread, read by Python (lookup / keys)
  std::mutex store_mu_;
  std::unordered_map<std::string, std::unique_ptr<Entry>> by_key_;
  std::unordered_map<uint64_t, Entry*> by_id_;       // lane-owned entries
  std::priority_queue<QItem> heap_;
  // ledger ids of lane pods: a range disjoint from the Python side's (models/pod.py::pod_num_id)
  uint64_t seq_ = 0, next_id_ = (1ull << 62);
  bool active_admission_ = false;                    // some profile hands pods to the lane

  // lane-thread scratch, flushed once per loop turn
  std::vector<std::shared_ptr<yk::PodEv>> grave_;   // lane thread: events to drop on the I/O thread
  std::vector<uint64_t> to_release_;                 // engine ledger releases (one lock per turn)
  // reserved pods whose labels / deletionTimestamp changed: the engine ledger's copy follows
  std::vector<std::pair<uint64_t, std::shared_ptr<yk::PodEv>>> meta_pending_;
  std::vector<Handoff> hand_pending_;
  uint64_t out_moves_pending_ = 0;
 public:
  std::atomic<uint64_t> scheduled_{0};               // Bindings acknowledged (incl. lost answers kept)
  // the lane signals its eventfd once scheduled_ reaches this (a waiter on the Python side)
  std::atomic<uint64_t> watermark_{UINT64_MAX};
  void set_watermark(uint64_t n);
 private:

  std::mutex out_mu_;
  std::vector<Fwd> out_fwd_;
  std::vector<Handoff> out_hand_;
  uint64_t out_moves_ = 0;
  bool signalled_ = false;

  std::mutex stat_mu_;
  LaneStats st_;
  std::vector<float> e2e_, pod_lat_;

  // native event recorder (lane thread)
  std::deque<PendingEvent> ev_q_;
  double ev_tokens_ = 0, ev_last_ = 0;
  uint64_t ev_seq_ = 0;
  // FailedScheduling de-duplication (framework/events.py): a repeat of an isomorphic event bumps
  // the series of the one written first. key → (event name, count)
  std::unordered_map<std::string, std::pair<std::string, int>> ev_dedup_;

  // native queues (lane thread): scheduling cycles, move requests, unschedulableQ, podBackoffQ
  uint64_t cycle_ = 0;
  int64_t move_cycle_ = -1;                          // upstream moveRequestCycle
  std::vector<int32_t> pending_moves_;               // this turn's move requests (-1: all)
  std::vector<std::pair<uint64_t, int32_t>> hints_;  // (cycle, node) of recent node hints
  uint64_t hint_dropped_cycle_ = 0;
  bool hint_dropped_ = false;
  std::unordered_map<uint64_t, Entry*> parked_;      // id → PARKED entry
  struct BItem {
    double until;
    uint64_t seq, id;
    bool operator<(const BItem& o) const { return until > o.until; }   // min-heap
  };
  std::priority_queue<BItem> bheap_;
  uint64_t bseq_ = 0;
  double next_leftover_ = 0;
};

}  // namespace yoda
