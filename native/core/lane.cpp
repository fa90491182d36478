// Native pod lane (see lane.hpp).
#include "lane.hpp"

#include <sys/eventfd.h>
#include <pthread.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <chrono>
#include <cmath>
#include <cstring>
#include <ctime>

namespace yoda {

namespace {

constexpr uint64_t kEventTag = 1ull << 63;
constexpr uint64_t kPatchBit = 1ull << 62;   // with kEventTag: a PodScheduled=False status patch

// engine Reason → FitError text (framework/scheduler.py::_fit_error)
const char* const kReasonName[] = {"OK", "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity",
                                         "NodeResourcesFit", "NoScv", "ScvStale", "GpuNumber", "GpuMemory",
                                         "GpuClock", "GpuFit", "NodeGone", "NodeResourcesFitExtended",
                                         "PodTopologySpread", "PodTopologySpreadLabel", "InterPodAffinityExisting",
                                         "InterPodAffinity", "InterPodAntiAffinity", "NodePorts", "VolumeBinding",
                                         "VolumeZone", "NodeVolumeLimits"};
static_assert(sizeof(kReasonName) / sizeof(kReasonName[0]) == RS_NUM, "kReasonName must name every engine Reason");
const char* reason_text(int i) {
  switch (i) {
    case RS_UNSCHEDULABLE: return "node(s) were unschedulable";
    case RS_NODE_NAME: return "node(s) didn't match the requested node name";
    case RS_TAINT: return "node(s) had taints that the pod didn't tolerate";
    case RS_AFFINITY: return "node(s) didn't match node selector";
    case RS_RESOURCES: return "Insufficient cpu/memory/pods";
    case RS_NO_SCV: return "node(s) have no Scv telemetry";
    case RS_STALE: return "node(s) have stale Scv telemetry";
    case RS_GPU_NUMBER: return "node(s) have too few GPUs";
    case RS_GPU_MEMORY: return "node(s) have too few GPUs with enough free HBM";
    case RS_GPU_CLOCK: return "node(s) have too few GPUs with the requested clock";
    case RS_GPU_FIT: return "node(s) have too few healthy GPUs matching scv/memory+scv/clock";
    case RS_EXT_RESOURCES: return "node(s) had insufficient extended resources";
    case RS_SPREAD: return "node(s) didn't match pod topology spread constraints";
    case RS_SPREAD_LABEL: return "node(s) didn't match pod topology spread constraints (missing required label)";
    case RS_EXISTING_ANTI: return "node(s) didn't satisfy existing pods anti-affinity rules";
    case RS_POD_AFFINITY: return "node(s) didn't match pod affinity rules";
    case RS_POD_ANTI: return "node(s) didn't match pod anti-affinity rules";
    case RS_NODE_PORTS: return "node(s) didn't have free ports for the requested pod ports";
    case RS_VOLUME_NODE: return "node(s) had volume node affinity conflict";
    case RS_VOLUME_ZONE: return "node(s) had no available volume zone";
    case RS_VOLUME_LIMITS: return "node(s) exceed max volume count";
    default: return i >= 0 && i < RS_NUM ? kReasonName[i] : "unknown";
  }
}

// Go strconv.Atoi: optional sign, decimal digits only, int64 range (utils/gonum.py::atoi).
bool go_atoi(const std::string& s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (!s.empty() && (s[0] == '+' || s[0] == '-')) {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  unsigned __int128 v = 0;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (c < '0' || c > '9') return false;
    v = v * 10 + (unsigned)(c - '0');
    if (v > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && v > (unsigned __int128)INT64_MAX) return false;
  *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
  return true;
}

int64_t atoi_or_zero(const std::string& s) {
  int64_t v;
  return go_atoi(s, &v) ? v : 0;
}

// filter.strToUint / StrToUint64 (filter.go:60-74): Atoi, error → 0, negative wraps
uint64_t str_to_uint(const std::string& s) { return (uint64_t)atoi_or_zero(s); }

int8_t effect_of(const std::string& e) {
  if (e == "NoSchedule") return kNoSchedule;
  if (e == "PreferNoSchedule") return kPreferNoSchedule;
  if (e == "NoExecute") return kNoExecute;
  return kEffectAny;
}

bool selop_of(const std::string& op, int8_t* out) {
  if (op == "In") *out = kIn;
  else if (op == "NotIn") *out = kNotIn;
  else if (op == "Exists") *out = kExists;
  else if (op == "DoesNotExist") *out = kDoesNotExist;
  else if (op == "Gt") *out = kGt;
  else if (op == "Lt") *out = kLt;
  else return false;
  return true;
}

void json_str(const std::string& s, std::string& o) {
  o.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o.push_back((char)c);
        }
    }
  }
  o.push_back('"');
}

// metav1.MicroTime (framework/events.py::micro_time)
std::string micro_time(double ts) {
  time_t sec = (time_t)ts;
  long us = std::lround((ts - (double)sec) * 1e6);
  if (us >= 1000000) {
    sec += 1;
    us -= 1000000;
  }
  struct tm tm;
  gmtime_r(&sec, &tm);
  char buf[48];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%S", &tm);
  char out[80];   // 47 + "." + up to 20 digits + "Z"
  snprintf(out, sizeof out, "%s.%06ldZ", buf, us);
  return out;
}

double wall() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

// metav1.Time: RFC 3339 in whole seconds, UTC
std::string rfc3339(double ts) {
  time_t sec = (time_t)ts;
  struct tm tm;
  gmtime_r(&sec, &tm);
  char buf[40];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tm);
  return buf;
}

std::string key_of(const yk::PodProj& p) {
  std::string k;                          // one allocation (ns + "/" + name builds a temporary)
  k.reserve(p.ns.size() + 1 + p.name.size());
  k.append(p.ns).push_back('/');
  k.append(p.name);
  return k;
}

bool terminal(const yk::PodProj& p) { return p.phase == "Succeeded" || p.phase == "Failed"; }

bool config_eq(const EngineConfig& a, const EngineConfig& b) {
  if (a.filters != b.filters || a.settle_s != b.settle_s) return false;
  for (int i = 0; i < S_NUM; ++i)
    if (a.score_w[i] != b.score_w[i]) return false;
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < 3; ++j)
      if (a.alloc_w[k][j] != b.alloc_w[k][j]) return false;
  const Weights &x = a.wt, &y = b.wt;
  return x.w_link == y.w_link && x.w_numa == y.w_numa && x.w_fit == y.w_fit && x.w_occ == y.w_occ &&
         x.gpu_binpack == y.gpu_binpack && x.w_gang_score == y.w_gang_score && x.enum_limit == y.enum_limit &&
         x.w_minlink == y.w_minlink;
}

}  // namespace

bool MatchTerm::matches(const std::string& ns, const std::vector<std::pair<std::string, std::string>>& lab) const {
  if (nothing) return false;
  if (!namespaces.empty() && std::find(namespaces.begin(), namespaces.end(), ns) == namespaces.end()) return false;
  auto get = [&](const std::string& k) -> const std::string* {
    for (const auto& kv : lab)
      if (kv.first == k) return &kv.second;
    return nullptr;
  };
  for (const auto& kv : labels) {
    const std::string* v = get(kv.first);
    if (!v || *v != kv.second) return false;
  }
  for (const auto& x : exprs) {
    const std::string* v = get(x.key);
    const bool in = v && std::find(x.values.begin(), x.values.end(), *v) != x.values.end();
    switch (x.op) {
      case 0: if (!in) return false; break;
      case 1: if (in) return false; break;
      case 2: if (!v) return false; break;
      case 3: if (v) return false; break;
      default: return false;
    }
  }
  return true;
}

double Lane::thread_cpu() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (double)ts.tv_sec + ts.tv_nsec * 1e-9;
}

double Lane::mono() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

Lane::Lane(Engine* e, std::recursive_mutex* engine_mu, LaneOptions o) : eng_(e), emu_(engine_mu), o_(std::move(o)) {
  if (o_.batch < 1) o_.batch = 1;
  efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (efd_ < 0) throw std::runtime_error("eventfd failed");
  ev_tokens_ = o_.event_burst > 0 ? o_.event_burst : 1;
  ev_last_ = mono();
  th_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "yoda-lane");   // per-thread CPU in bench / top -H
    run();
  });
  wk_th_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "yoda-lane-eng");
    engine_worker();
  });
}

Lane::~Lane() { close(); }

void Lane::close() {
  {
    std::lock_guard<std::mutex> g(in_mu_);
    if (stop_.exchange(true)) {
      if (!th_.joinable() && !wk_th_.joinable()) return;
    }
    in_cv_.notify_all();
  }
  if (th_.joinable()) th_.join();
  {
    std::lock_guard<std::mutex> g(wk_mu_);
    wk_cv_.notify_all();
  }
  if (wk_th_.joinable()) wk_th_.join();
  relist_cv_.notify_all();
  if (efd_ >= 0) {
    ::close(efd_);
    efd_ = -1;
  }
}

void Lane::push_locked(Item&& it) {
  inbox_.push_back(std::move(it));
  inbox_flag_.store(true, std::memory_order_relaxed);
}

// Busy-wait up to LaneOptions::spin_us for `flag` (or stop); the caller then takes the lock
// and re-checks its own predicate, so a missed flag only costs the futex wait it replaces.
void Lane::spin_until(const std::atomic<bool>& flag) const {
  if (o_.spin_us <= 0) return;
  const double end = mono() + o_.spin_us * 1e-6;
  for (int i = 0; !flag.load(std::memory_order_relaxed) && !stop_.load(std::memory_order_relaxed); ++i) {
    __builtin_ia32_pause();
    if ((i & 63) == 63 && mono() > end) return;
  }
}

// ------------------------------------------------------------------ configuration
void Lane::set_profile(const Profile& p) {
  {
    std::lock_guard<std::mutex> g(prof_mu_);
    auto it = std::find_if(profiles_.begin(), profiles_.end(), [&](const Profile& x) { return x.name == p.name; });
    if (it == profiles_.end()) profiles_.push_back(p);
    else *it = p;
  }
  std::lock_guard<std::mutex> g(in_mu_);
  Item it;
  it.k = Item::kProfiles;
  push_locked(std::move(it));
  in_cv_.notify_one();
}

bool Lane::set_gates(const std::string& name, std::vector<MatchTerm> terms) {
  {
    std::lock_guard<std::mutex> g(prof_mu_);
    auto it = std::find_if(profiles_.begin(), profiles_.end(), [&](const Profile& x) { return x.name == name; });
    if (it == profiles_.end()) return false;
    std::vector<MatchTerm> added;
    for (const MatchTerm& t : terms)
      if (std::find(it->gate_terms.begin(), it->gate_terms.end(), t) == it->gate_terms.end()) added.push_back(t);
    it->gate_terms = std::move(terms);
    if (!added.empty()) gate_adds_.emplace_back(name, std::move(added));
  }
  std::lock_guard<std::mutex> g(in_mu_);
  Item it;
  it.k = Item::kGates;
  push_locked(std::move(it));
  in_cv_.notify_one();
  return true;
}

void Lane::set_inert_claims(std::vector<std::string> keys) {
  std::vector<std::pair<std::string, ClaimConsP>> add;
  add.reserve(keys.size());
  for (auto& k : keys) add.emplace_back(std::move(k), nullptr);
  update_claims(true, std::move(add), {});
}

void Lane::update_inert_claims(std::vector<std::string> add, std::vector<std::string> remove) {
  std::vector<std::pair<std::string, ClaimConsP>> a;
  a.reserve(add.size());
  for (auto& k : add) a.emplace_back(std::move(k), nullptr);
  update_claims(false, std::move(a), std::move(remove));
}

void Lane::update_claims(bool reset, std::vector<std::pair<std::string, ClaimConsP>> add,
                         std::vector<std::string> remove) {
  ClaimOp op;
  op.reset = reset;
  op.add = std::move(add);
  op.remove = std::move(remove);
  {
    std::lock_guard<std::mutex> g(prof_mu_);
    claim_ops_.push_back(std::move(op));
  }
  std::lock_guard<std::mutex> g(in_mu_);
  Item it;
  it.k = Item::kClaims;
  push_locked(std::move(it));
  in_cv_.notify_one();
}

void Lane::set_active(bool on) {
  std::lock_guard<std::mutex> g(in_mu_);
  active_.store(on);
  in_cv_.notify_one();
}

void Lane::move(int32_t node) {
  std::lock_guard<std::mutex> g(in_mu_);
  Item it;
  it.k = Item::kMove;
  it.status = node;
  push_locked(std::move(it));
  in_cv_.notify_one();
}

void Lane::set_node_cards(const std::string& node, std::vector<std::pair<std::string, std::string>> vis) {
  std::lock_guard<std::mutex> g(vis_mu_);
  vis_[node] = std::move(vis);
}

void Lane::remove_node_cards(const std::string& node) {
  std::lock_guard<std::mutex> g(vis_mu_);
  vis_.erase(node);
}

// ------------------------------------------------------------------ transport callbacks
void Lane::on_pod_events(uint64_t, std::vector<yk::WatchEvent>& evs) {
  size_t kept = 0;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    for (auto& e : evs) {
      if (e.pod && (e.type == 'A' || e.type == 'M' || e.type == 'D')) {
        Item it;
        it.k = Item::kEvent;
        it.type = e.type;
        it.ev = std::move(e.pod);
        push_locked(std::move(it));
      } else {
        if (&evs[kept] != &e) evs[kept] = std::move(e);
        ++kept;
      }
    }
    in_cv_.notify_one();
  }
  evs.resize(kept);
}

void Lane::on_answers(std::vector<yk::PodSink::Answer>& answers) {
  std::lock_guard<std::mutex> g(in_mu_);
  for (auto& a : answers) {
    Item it;
    it.k = Item::kAnswer;
    it.tag = a.tag;
    it.status = a.status;
    it.body = std::move(a.body);
    it.t = a.t;
    push_locked(std::move(it));
  }
  in_cv_.notify_one();
}

// ------------------------------------------------------------------ Python side
void Lane::drain(std::vector<Fwd>* fwd, std::vector<Handoff>* hand, uint64_t* moves) {
  uint64_t v;
  while (::read(efd_, &v, sizeof v) > 0) {
  }
  std::lock_guard<std::mutex> g(out_mu_);
  fwd->swap(out_fwd_);
  hand->swap(out_hand_);
  *moves = out_moves_;
  out_moves_ = 0;
  signalled_ = false;
}

std::vector<Lane::Fwd> Lane::relist(std::vector<std::shared_ptr<yk::PodEv>> items) {
  uint64_t token;
  std::unique_lock<std::mutex> lk(in_mu_);
  token = ++relist_next_;
  Item it;
  it.k = Item::kRelist;
  it.items = std::make_shared<std::vector<std::shared_ptr<yk::PodEv>>>(std::move(items));
  it.token = token;
  push_locked(std::move(it));
  in_cv_.notify_one();
  relist_cv_.wait(lk, [&] { return relist_done_ >= token || stop_.load(); });
  std::vector<Fwd> out;
  auto f = relist_out_.find(token);
  if (f != relist_out_.end()) {
    out = std::move(f->second);
    relist_out_.erase(f);
  }
  return out;
}

std::shared_ptr<yk::PodEv> Lane::lookup(const std::string& key, bool* owned) {
  std::lock_guard<std::mutex> g(store_mu_);
  auto it = by_key_.find(key);
  if (it == by_key_.end()) return nullptr;
  if (owned) *owned = it->second->st != PY;
  return it->second->ev;
}

std::shared_ptr<yk::PodEv> Lane::lookup_id(uint64_t id, std::string* node) {
  std::lock_guard<std::mutex> g(store_mu_);
  auto it = by_id_.find(id);
  if (it == by_id_.end()) return nullptr;
  if (node) *node = it->second->node_name;
  return it->second->ev;
}

std::vector<std::string> Lane::keys() {
  std::lock_guard<std::mutex> g(store_mu_);
  std::vector<std::string> out;
  out.reserve(by_key_.size());
  for (auto& kv : by_key_) out.push_back(kv.first);
  return out;
}

size_t Lane::store_size() {
  std::lock_guard<std::mutex> g(store_mu_);
  return by_key_.size();
}

LaneStats Lane::stats() {
  LaneStats s;
  {
    std::lock_guard<std::mutex> g(stat_mu_);
    s = st_;
  }
  return s;
}

std::vector<float> Lane::take_e2e() {
  std::lock_guard<std::mutex> g(stat_mu_);
  std::vector<float> v;
  v.swap(e2e_);
  return v;
}

std::vector<float> Lane::take_pod_latency() {
  std::lock_guard<std::mutex> g(stat_mu_);
  std::vector<float> v;
  v.swap(pod_lat_);
  return v;
}

void Lane::wait_idle(double timeout_s) {
  const auto until = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  std::unique_lock<std::mutex> lk(in_mu_);
  while (std::chrono::steady_clock::now() < until) {
    bool queued;
    {
      std::lock_guard<std::mutex> g(stat_mu_);
      queued = st_.queued > 0 && active_.load();
    }
    if (inbox_.empty() && !busy_ && !run_inflight_ && !queued) return;
    lk.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    lk.lock();
  }
}

// ------------------------------------------------------------------ lane thread
void Lane::publish(std::vector<Fwd>&& fwd, std::vector<Handoff>&& hand) {
  if (fwd.empty() && hand.empty()) return;
  bool sig = false;
  {
    std::lock_guard<std::mutex> g(out_mu_);
    if (out_fwd_.empty()) out_fwd_.swap(fwd);
    else
      for (auto& f : fwd) out_fwd_.push_back(std::move(f));
    if (out_hand_.empty()) out_hand_.swap(hand);
    else
      for (auto& h : hand) out_hand_.push_back(std::move(h));
    if (!signalled_) signalled_ = sig = true;
  }
  if (sig) {
    const uint64_t one = 1;
    ssize_t w = ::write(efd_, &one, sizeof one);
    (void)w;
  }
}

void Lane::forward(char type, std::shared_ptr<yk::PodEv> ev, std::shared_ptr<yk::PodEv> old, std::vector<Fwd>* out) {
  ev->materialize();                      // Python may read it from another thread
  out->push_back(Fwd{type, std::move(ev), std::move(old)});
  std::lock_guard<std::mutex> g(stat_mu_);
  st_.forwarded++;
}

int64_t Lane::prio_of(const yk::PodProj& p) const {
  if (o_.sort_kind == 1) return p.priority;
  for (const auto& kv : p.labels)
    if (kv.first == "scv/priority") return atoi_or_zero(kv.second);
  return 0;
}

bool Lane::admissible(const yk::PodProj& p, int* prof) const {
  if (!p.ok || !p.node.empty() || p.deleting || terminal(p)) return false;
  for (size_t i = 0; i < lp_.size(); ++i) {
    if (lp_[i].name != p.sched) continue;
    const int f = p.flags & lp_[i].flag_mask;
    if (!lp_[i].enabled || (f && (f != yk::PF_CLAIMS || !lp_[i].claims_ok || !claims_in_table(p)))) return false;
    for (const MatchTerm& t : lp_[i].gate_terms)
      if (t.matches(p)) return false;     // an existing pod's required anti-affinity may reject it
    *prof = (int)i;
    return true;
  }
  return false;
}

namespace {
// a pod the Python side does not need to see: unassigned, of a scheduler no profile serves
bool uninteresting(const yk::PodProj& p, const std::vector<Lane::Profile>& lp) {
  if (!p.node.empty()) return false;
  for (const auto& x : lp)
    if (x.name == p.sched) return false;
  return true;
}
}  // namespace

// store mutations: lane thread, store_mu_ held by the caller
void Lane::handle_event(char type, const std::shared_ptr<yk::PodEv>& ev, std::vector<Fwd>* out) {
  const yk::PodProj& p = ev->p;
  std::string key = key_of(p);
  auto it = by_key_.find(key);
  if (it != by_key_.end() && it->second->ev->p.uid != p.uid && type != 'D') {
    // the key now names another pod (deleted + recreated while we were not watching)
    handle_event('D', it->second->ev, out);
    it = by_key_.end();
  }
  if (type == 'D') {
    if (it == by_key_.end()) return;
    Entry* e = it->second.get();
    if (e->st == PY) {
      if (!uninteresting(e->ev->p, lp_)) forward('D', ev, e->ev, out);
    } else {
      const bool held = e->st == BINDING || e->st == BOUND;
      drop_owned(e, held);
      if (held) {
        std::lock_guard<std::mutex> g(stat_mu_);
        st_.released++;
        out_moves_pending_++;
      }
    }
    grave_.push_back(std::move(it->second->ev));   // freed on the I/O thread (recycle)
    by_key_.erase(it);
    return;
  }
  if (it == by_key_.end()) {
    auto e = std::make_unique<Entry>();
    e->ev = ev;
    int prof = -1;
    if (active_admission_ && admissible(ev->full(), &prof)) {
      e->st = QUEUED;
      e->id = next_id_++;
      e->prof = prof;
      e->prio = prio_of(ev->full());
      e->seq = ++seq_;
      e->t_enq = mono();
      by_id_[e->id] = e.get();
      heap_.push(QItem{e->prio, e->seq, e->id});
      count(QUEUED, +1);
      std::lock_guard<std::mutex> g(stat_mu_);
      st_.admitted++;
    } else if (!uninteresting(p, lp_)) {
      forward('A', ev, nullptr, out);
    }
    by_key_.emplace(std::move(key), std::move(e));
    return;
  }
  Entry* e = it->second.get();
  std::shared_ptr<yk::PodEv> old = e->ev;
  if (e->st == PY) {
    e->ev = ev;
    if (!uninteresting(p, lp_)) forward(uninteresting(old->p, lp_) ? 'A' : 'M', ev, old, out);
    return;
  }
  // lane-owned
  if (p.node.empty()) {
    const bool waiting = e->st == PARKED || e->st == BACKOFF;
    if ((e->st == QUEUED || waiting) && ev->hash() != old->hash()) {
      int prof = -1;
      if (!admissible(ev->full(), &prof)) {
        // no longer for the lane (a feature a Python plugin handles, another scheduler, ...)
        drop_owned(e, false);
        e->ev = ev;
        if (!uninteresting(p, lp_)) forward('A', ev, nullptr, out);
        return;
      }
      e->prof = prof;
      const int64_t pr = prio_of(ev->full());
      if (waiting) {
        // an update may make an unschedulable pod schedulable: retry now (queue.update)
        e->prio = pr;
        e->req.reset();
        if (e->st == PARKED) parked_.erase(e->id);
        activate(e);
      } else if (pr != e->prio) {          // re-sorted, FIFO position kept (activeQ.Update)
        e->prio = pr;
        heap_.push(QItem{e->prio, e->seq, e->id});
      }
    }
    ev->full();                            // a queued / assumed pod's event must stay complete
    e->ev = ev;                            // assumed pods: status noise only (skipPodUpdate)
    return;
  }
  // the pod is bound
  if (terminal(p)) {
    const bool held = e->st == BINDING || e->st == BOUND;
    drop_owned(e, held);
    e->ev = ev;
    if (held) {
      std::lock_guard<std::mutex> g(stat_mu_);
      st_.released++;
      out_moves_pending_++;
    }
    return;                                // stays in the store as a Python-visible terminal pod
  }
  if ((e->st == BINDING || e->st == BOUND) && p.node == e->node_name) {
    const bool was_deleting = old->p.deleting;
    if (!e->lab_ev || !p.labels_hash || p.labels_hash != e->lab_ev->p.labels_hash) {
      // the engine ledger's copy of the labels (spread counts) follows a real change only:
      // the first echo carries the labels the pod was placed with
      if (e->lab_ev && (!p.labels_hash || p.labels_hash != e->lab_ev->p.labels_hash)) meta_pending_.push_back({e->id, ev});
      e->lab_ev = ev;
      if (e->crow >= 0) census_[e->crow].dirty = true;
    } else if (p.deleting != was_deleting) {
      meta_pending_.push_back({e->id, ev});
    }
    if (e->crow >= 0) census_[e->crow].deleting = p.deleting;
    if (e->ev != e->lab_ev) grave_.push_back(std::move(e->ev));
    e->ev = ev;
    if (!e->confirmed) {
      e->confirmed = true;
      set_state(e, BOUND);
      std::lock_guard<std::mutex> g(stat_mu_);
      st_.confirmed++;
      if (pod_lat_.size() < o_.e2e_keep) pod_lat_.push_back((float)(mono() - e->t_enq));
    }
    return;
  }
  // bound elsewhere (another scheduler, a user): our reservation (if any) goes, Python tracks it
  drop_owned(e, e->st == BINDING || e->st == BOUND);
  e->ev = ev;
  forward('M', ev, old, out);
}

void Lane::count(St s, int d) {
  std::lock_guard<std::mutex> g(stat_mu_);
  if (s == QUEUED) st_.queued += d;
  else if (s == INFLIGHT) st_.inflight += d;
  else if (s == PARKED) st_.parked += d;
  else if (s == BACKOFF) st_.backoff += d;
  if (s != PY) st_.owned += d;
}

void Lane::bind_settled(Entry* e) {
  if (!e->bind_out) return;
  e->bind_out = false;
  std::lock_guard<std::mutex> g(stat_mu_);
  st_.binding--;
}

void Lane::set_state(Entry* e, St s) {
  if (e->st == s) return;
  count(e->st, -1);
  e->st = s;
  count(s, +1);
}

// a lane-owned entry becomes a Python (store-only) entry; `release` drops its reservation
void Lane::drop_owned(Entry* e, bool release) {
  bind_settled(e);
  if (e->st == PARKED) parked_.erase(e->id);      // a BACKOFF heap item goes stale by itself
  e->req.reset();
  if (e->crow >= 0) census_remove(e);
  if (e->lab_ev) grave_.push_back(std::move(e->lab_ev));
  if (release && e->id) {
    to_release_.push_back(e->id);
    log_remove(e->id);
  }
  if (e->id) by_id_.erase(e->id);
  set_state(e, PY);
  e->id = 0;
  e->confirmed = e->acked = false;
  e->node = -1;
  e->node_name.clear();
}

void Lane::handle_answer(uint64_t tag, int status, std::string& body, double t_ack) {
  if (tag & kEventTag) {
    std::lock_guard<std::mutex> g(stat_mu_);
    const bool ok = status >= 200 && status < 300;
    if (tag & kPatchBit) {
      if (!ok) st_.status_patch_errors++;
    } else if (ok) {
      st_.events_written++;
    } else {
      st_.event_errors++;
    }
    return;
  }
  auto it = by_id_.find(tag);
  if (it == by_id_.end()) return;            // deleted meanwhile: its reservation is gone already
  Entry* e = it->second;
  if (e->st != BINDING && e->st != BOUND) return;
  // the bind is acknowledged when the I/O thread read the answer, not when this thread got to it
  const double now = t_ack > 0 ? t_ack : mono();
  bind_settled(e);
  if (status >= 200 && status < 300) {
    e->acked = true;
    set_state(e, BOUND);
    {
      std::lock_guard<std::mutex> g(stat_mu_);
      st_.scheduled++;
      if (e->prof >= 0 && e->prof < (int)lp_.size()) st_.by_profile[lp_[e->prof].name].first++;
      if (e2e_.size() < o_.e2e_keep) e2e_.push_back((float)(now - e->t_cycle));
    }
    if (scheduled_.fetch_add(1, std::memory_order_relaxed) + 1 == watermark_.load(std::memory_order_relaxed))
      signal_python();
    record_scheduled(*e);
    return;
  }
  {
    std::lock_guard<std::mutex> g(stat_mu_);
    st_.bind_errors++;
  }
  if (e->confirmed) {
    // the Binding was applied (its echo confirmed the pod), only the answer was lost: the
    // pod is bound — keep it (upstream ForgetPod refuses pods that are no longer assumed)
    {
      std::lock_guard<std::mutex> g(stat_mu_);
      st_.scheduled++;
      st_.lost_answers_kept++;
    }
    scheduled_.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  Handoff h;
  h.kind = Handoff::kBindError;
  h.ev = e->ev;
  h.profile = e->prof >= 0 && e->prof < (int)lp_.size() ? lp_[e->prof].name : std::string();
  h.status = status;
  h.msg = std::move(body);
  h.t_enqueue = e->t_enq;
  h.t_cycle = e->t_cycle;
  h.attempts = std::max<uint32_t>(1, e->attempts);
  drop_owned(e, true);
  hand_pending_.push_back(std::move(h));
}

void Lane::handle_relist(const std::vector<std::shared_ptr<yk::PodEv>>& items, std::vector<Fwd>* out) {
  std::unordered_map<std::string, const std::shared_ptr<yk::PodEv>*> fresh;
  fresh.reserve(items.size());
  for (const auto& ev : items) fresh[key_of(ev->p)] = &ev;
  std::vector<std::shared_ptr<yk::PodEv>> gone;
  for (auto& kv : by_key_)
    if (!fresh.count(kv.first)) gone.push_back(kv.second->ev);
  for (auto& ev : gone) handle_event('D', ev, out);
  for (const auto& ev : items) {
    auto it = by_key_.find(key_of(ev->p));
    if (it == by_key_.end()) handle_event('A', ev, out);
    else if (it->second->ev->p.rv != ev->p.rv) handle_event('M', ev, out);
  }
}

// A gates-only update (set_gates): the lane's profiles take the new terms; waiting pods are
// re-checked against the ADDED terms only — a removed term cannot make a pod inadmissible, and
// re-running every term for every waiting pod on each update cost O(waiting × terms) per
// Python cycle while anti-affinity holders accumulate.
void Lane::apply_gates(std::vector<Fwd>* out) {
  std::vector<std::pair<std::string, std::vector<MatchTerm>>> adds;
  {
    std::lock_guard<std::mutex> g(prof_mu_);
    adds.swap(gate_adds_);
    for (auto& lp : lp_)
      for (const auto& p : profiles_)
        if (p.name == lp.name) {
          lp.gate_terms = p.gate_terms;
          break;
        }
  }
  if (adds.empty()) return;
  std::vector<Entry*> evict;
  for (auto& kv : by_id_) {
    Entry* e = kv.second;
    if (e->st != QUEUED && e->st != PARKED && e->st != BACKOFF) continue;
    const yk::PodProj& p = e->ev->full();
    bool hit = false;
    for (const auto& a : adds) {
      if (a.first != p.sched) continue;
      for (const MatchTerm& t : a.second)
        if (t.matches(p)) {
          hit = true;
          break;
        }
      if (hit) break;
    }
    if (hit) evict.push_back(e);
  }
  for (Entry* e : evict) {
    if (e->st == PARKED || e->st == BACKOFF) {
      requeue_to_python(e);
      continue;
    }
    drop_owned(e, false);
    if (!uninteresting(e->ev->p, lp_)) forward('A', e->ev, nullptr, out);
  }
}

bool Lane::claims_in_table(const yk::PodProj& p) const {
  if (p.cold().claims.empty() || claim_table_.empty()) return false;
  std::string key;
  for (const std::string& c : p.cold().claims) {
    key.assign(p.ns).append("/").append(c);
    if (!claim_table_.count(key)) return false;
  }
  return true;
}

bool Lane::claim_cons(const yk::PodProj& p, std::vector<ClaimConsP>* out) const {
  std::string key;
  for (const std::string& c : p.cold().claims) {
    key.assign(p.ns).append("/").append(c);
    auto it = claim_table_.find(key);
    if (it == claim_table_.end()) return false;
    if (it->second) out->push_back(it->second);
  }
  return true;
}

// A claim-table change: waiting pods that mount a claim which left the table, or whose
// constraints changed (their cached request holds the old ones), go to Python. A claim that
// joined cannot make a pod inadmissible; pods Python holds stay there.
void Lane::apply_claims(std::vector<Fwd>* out) {
  std::vector<ClaimOp> ops;
  {
    std::lock_guard<std::mutex> g(prof_mu_);
    ops.swap(claim_ops_);                   // an earlier kClaims may have taken them already
  }
  if (ops.empty()) return;
  std::unordered_set<std::string> removed;  // left the table or changed at some op
  // a reset rebuilds every claim's record: compare the constraints, not the pointers
  auto changed = [](const ClaimConsP& a, const ClaimConsP& b) { return a != b && (!a || !b || !(*a == *b)); };
  for (auto& op : ops) {
    if (op.reset) {
      std::unordered_map<std::string, ClaimConsP> next;
      for (auto& kv : op.add) next.emplace(std::move(kv.first), std::move(kv.second));
      for (const auto& kv : claim_table_) {
        auto it = next.find(kv.first);
        if (it == next.end() || changed(it->second, kv.second)) removed.insert(kv.first);
      }
      claim_table_.swap(next);
      continue;
    }
    for (auto& k : op.remove)
      if (claim_table_.erase(k)) removed.insert(std::move(k));
    for (auto& kv : op.add) {
      auto it = claim_table_.find(kv.first);
      if (it != claim_table_.end()) {
        if (changed(it->second, kv.second)) removed.insert(kv.first);
        it->second = std::move(kv.second);
      } else {
        claim_table_.emplace(std::move(kv.first), std::move(kv.second));
      }
    }
  }
  if (removed.empty()) return;
  std::vector<Entry*> evict;
  std::string key;
  for (auto& kv : by_id_) {
    Entry* e = kv.second;
    if (e->st != QUEUED && e->st != PARKED && e->st != BACKOFF) continue;
    const yk::PodProj& p = e->ev->full();
    if (!(p.flags & yk::PF_CLAIMS)) continue;
    for (const std::string& c : p.cold().claims) {
      key.assign(p.ns).append("/").append(c);
      if (removed.count(key)) {
        evict.push_back(e);
        break;
      }
    }
  }
  for (Entry* e : evict) {
    if (e->st == PARKED || e->st == BACKOFF) {
      requeue_to_python(e);
      continue;
    }
    drop_owned(e, false);
    if (!uninteresting(e->ev->p, lp_)) forward('A', e->ev, nullptr, out);
  }
}

void Lane::requeue_to_python(Entry* e) {
  // the pod keeps its attempt count and goes to Python's podBackoffQ instead of
  // arriving as a fresh add (which retried at once and restarted backoff from the initial value)
  Handoff h;
  h.kind = Handoff::kRequeue;
  h.ev = e->ev;
  h.profile = e->prof >= 0 && e->prof < (int)lp_.size() ? lp_[e->prof].name : std::string();
  h.t_enqueue = e->t_enq;
  h.t_cycle = e->t_fail;
  h.attempts = std::max<uint32_t>(1, e->attempts);
  drop_owned(e, false);
  hand_pending_.push_back(std::move(h));
}

void Lane::apply_profiles(std::vector<Fwd>* out) {
  {
    std::lock_guard<std::mutex> g(prof_mu_);
    lp_ = profiles_;
  }
  active_admission_ = false;
  for (const auto& p : lp_) active_admission_ |= p.enabled;
  // queued pods a profile no longer hands to the lane go to the Python queue
  std::vector<Entry*> evict;
  for (auto& kv : by_id_) {
    Entry* e = kv.second;
    if (e->st != QUEUED && e->st != PARKED && e->st != BACKOFF) continue;
    int prof = -1;
    // a waiting pod whose profile now has a PostFilter that may help it goes to Python too
    if (!admissible(e->ev->full(), &prof) ||
        (e->st != QUEUED && e->ev->full().priority > lp_[prof].preempt_above))
      evict.push_back(e);
    else
      e->prof = prof;
  }
  for (Entry* e : evict) {
    // a waiting pod of a profile that is still served (now by Python) keeps its backoff state
    if ((e->st == PARKED || e->st == BACKOFF) && !uninteresting(e->ev->p, lp_) && e->ev->full().ok &&
        e->ev->full().node.empty()) {
      requeue_to_python(e);
      continue;
    }
    drop_owned(e, false);
    if (!uninteresting(e->ev->p, lp_)) forward('A', e->ev, nullptr, out);
  }
}

bool Lane::make_req(const yk::PodProj& p, PodReq* r) {
  const std::string *n = nullptr, *m = nullptr, *c = nullptr, *pr = nullptr, *cm = nullptr;
  for (const auto& kv : p.labels) {
    const std::string& k = kv.first;
    if (k.size() < 5 || k[0] != 's' || k[1] != 'c' || k[2] != 'v') continue;
    if (k == "scv/number") n = &kv.second;
    else if (k == "scv/memory") m = &kv.second;
    else if (k == "scv/clock") c = &kv.second;
    else if (k == "scv/priority") pr = &kv.second;
    else if (k == "scv.amd.com/clock-min") cm = &kv.second;
  }
  // models/labels.py::parse_gpu_request + ops/native.py::pod_req (Engine.make_req)
  r->has_number = n != nullptr;
  r->number = n ? str_to_uint(*n) : 1;
  r->has_memory = m != nullptr;
  r->memory = m ? str_to_uint(*m) : 0;
  r->has_clock = c != nullptr;
  r->clock = c ? str_to_uint(*c) : 0;
  r->clock_min = cm ? str_to_uint(*cm) : 0;
  r->priority = pr ? atoi_or_zero(*pr) : 0;
  r->pod_priority = p.priority;
  r->node_name = p.node.empty() ? -1 : eng_->intern(p.node);
  r->cpu_m = p.cpu;
  r->mem = p.mem;
  r->nz_cpu_m = p.nzc;
  r->nz_mem = p.nzm;
  for (const auto& kv : p.cold().node_selector) r->node_selector.emplace_back(eng_->intern(kv.first), eng_->intern(kv.second));
  auto term = [&](const yk::TermP& t, SelTerm* out) {
    for (const auto& q : t) {
      SelReq x;
      x.key = eng_->intern(q.key);
      if (!selop_of(q.op, &x.op)) return false;
      x.num = 0;
      for (const auto& v : q.values) {
        x.values.push_back(eng_->intern(v));
        if (x.op == kGt || x.op == kLt) {
          int64_t num;
          if (!go_atoi(v, &num)) return false;   // Python's stoll would raise: its path decides
          x.num = num;
        }
      }
      out->reqs.push_back(std::move(x));
    }
    return true;
  };
  for (const auto& t : p.cold().req_terms) {
    SelTerm st;
    if (!term(t, &st)) return false;
    r->required_terms.push_back(std::move(st));
  }
  for (const auto& wt : p.cold().pref_terms) {
    PrefTerm pt;
    pt.weight = (int32_t)wt.first;
    if (!term(wt.second, &pt.term)) return false;
    r->preferred_terms.push_back(std::move(pt));
  }
  for (const auto& t : p.cold().tolerations) {
    Toleration x;
    x.key = t.has_key ? eng_->intern(t.key) : -1;
    if (x.key == 0) x.key = -1;
    x.value = eng_->intern(t.value);
    x.op = t.op == "Exists" ? kTolExists : kTolEqual;
    x.effect = effect_of(t.effect);
    r->tolerations.push_back(x);
  }
  // default-plugin inputs (ops/native.py::pod_req → Engine.set_req_extras)
  r->ns = eng_->intern(p.ns);
  r->labels = intern_labels(p.labels);
  r->deleting = p.deleting;
  for (const auto& im : p.images) r->images.push_back(eng_->intern(im));
  r->containers = p.containers;
  for (const auto& x : p.cold().ext) r->ext.emplace_back(eng_->intern(x.first), x.second);
  std::sort(r->ext.begin(), r->ext.end());
  HostPort hp;
  for (const auto& x : p.cold().ports)
    if (eng_->host_port(x.host_port, x.protocol, x.host_ip, &hp)) r->host_ports.push_back(hp);
  for (size_t i = 0; i < p.cold().claims.size(); ++i)   // the ledger keeps every pod's PVC claims (NodeVolumeLimits)
    if (i < p.cold().claim_pvc.size() && p.cold().claim_pvc[i]) r->pvc_claims.push_back(eng_->intern(p.ns + "/" + p.cold().claims[i]));
  if (const yk::PodProj::Owners* o = p.owners.get()) {
    if (o->has_owner) {
      r->owner_kind = o->owner_api == "v1" && o->owner_kind == "ReplicationController" ? 1
                      : o->owner_api == "apps/v1" && o->owner_kind == "ReplicaSet"  ? 2
                      : o->owner_api == "apps/v1" && o->owner_kind == "StatefulSet" ? 3 : 0;
      if (r->owner_kind) r->owner_name = eng_->intern(o->owner_name);
    }
    if (o->has_avoid) {
      r->avoid_kind = o->avoid_kind == "ReplicationController" ? 1 : 2;
      r->avoid_uid = eng_->intern(o->avoid_uid);
    }
  }
  r->spread_explicit = !p.cold().spread.empty();
  for (const auto& c : p.cold().spread) {
    if (c.when == 2) continue;               // neither DoNotSchedule nor ScheduleAnyway: in no list
    SpreadC x;
    x.key = eng_->intern(c.key);
    x.max_skew = (int32_t)c.max_skew;
    x.hard = c.when == 0;
    x.sel.nothing = !c.has_sel;
    for (const auto& kv : c.labels) x.sel.reqs.push_back(LReq{eng_->intern(kv.first), kIn, {eng_->intern(kv.second)}});
    for (const auto& q : c.exprs) {
      LReq lr;
      lr.key = eng_->intern(q.key);
      if (!selop_of(q.op, &lr.op) || lr.op == kGt || lr.op == kLt) return false;
      for (const auto& v : q.values) lr.values.push_back(eng_->intern(v));
      x.sel.reqs.push_back(std::move(lr));
    }
    r->spread.push_back(std::move(x));
  }
  if (p.cold().has_pod_aff) {
    auto pa = std::make_shared<PodAffinity>();
    auto conv = [&](const std::vector<yk::PodProj::PodTermP>& src, std::vector<PodTerm>* dst) {
      for (const auto& t : src) {
        PodTerm x;
        x.key = eng_->intern(t.key);
        if (t.ns.empty()) x.ns.push_back(r->ns);
        for (const auto& n : t.ns) x.ns.push_back(eng_->intern(n));
        x.sel.nothing = !t.has_sel;
        for (const auto& kv : t.labels) x.sel.reqs.push_back(LReq{eng_->intern(kv.first), kIn, {eng_->intern(kv.second)}});
        for (const auto& q : t.exprs) {
          LReq lr;
          lr.key = eng_->intern(q.key);
          if (!selop_of(q.op, &lr.op) || lr.op == kGt || lr.op == kLt) return false;
          for (const auto& v : q.values) lr.values.push_back(eng_->intern(v));
          x.sel.reqs.push_back(std::move(lr));
        }
        x.weight = (int32_t)t.weight;
        dst->push_back(std::move(x));
      }
      return true;
    };
    if (!conv(p.cold().aff_req, &pa->req_aff) || !conv(p.cold().anti_req, &pa->req_anti) || !conv(p.cold().aff_pref, &pa->pref_aff) ||
        !conv(p.cold().anti_pref, &pa->pref_anti))
      return false;
    if (!pa->empty()) r->aff = std::move(pa);
  }
  return true;
}

Labels Lane::intern_labels(const std::vector<std::pair<std::string, std::string>>& kv) {
  Labels l;
  l.reserve(kv.size());
  for (const auto& x : kv) l.emplace_back(eng_->intern(x.first), eng_->intern(x.second));
  std::sort(l.begin(), l.end());
  return l;
}

namespace {
// a JSON string literal (the kube module's dump_string is not linked into this module)
void json_quoted(std::string_view v, std::string& o) {
  static const char hx[] = "0123456789abcdef";
  o.push_back('"');
  for (unsigned char c : v) {
    if (c == '"' || c == '\\') {
      o.push_back('\\');
      o.push_back(char(c));
    } else if (c < 0x20) {
      o.append("\\u00");
      o.push_back(hx[c >> 4]);
      o.push_back(hx[c & 15]);
    } else {
      o.push_back(char(c));
    }
  }
  o.push_back('"');
}
}  // namespace

void Lane::annotations(const Profile& pr, const Entry& e, const PodReq& req, const CycleResult& r,
                       std::string* out) {
  // plugins/defaults.py::bind_annotations, written as JSON object members
  if (!pr.annotate) return;
  thread_local std::string vis, uu;
  vis.clear();
  uu.clear();
  size_t nu = 0;
  char num[24];
  std::string& o = *out;
  o.append("\"scv.amd.com/gpus\":\"");
  {
    std::lock_guard<std::mutex> g(vis_mu_);
    auto it = vis_.find(e.node_name);
    const std::vector<std::pair<std::string, std::string>>* per = it == vis_.end() ? nullptr : &it->second;
    for (size_t i = 0; i < r.cards.size(); ++i) {
      const int32_t c = r.cards[i];
      const int nn = int(std::to_chars(num, num + sizeof num, c).ptr - num);   // snprintf: ~10x dearer
      if (i) {
        o.push_back(',');
        vis.push_back(',');
      }
      o.append(num, size_t(nn));
      if (per && c >= 0 && c < (int32_t)per->size()) {
        vis += (*per)[c].first;
        if (!(*per)[c].second.empty()) {
          if (nu) uu.push_back(',');
          uu += (*per)[c].second;
          ++nu;
        }
      } else {
        vis.append(num, size_t(nn));
      }
    }
  }
  o.append("\",\"scv.amd.com/visible-devices\":");
  json_quoted(vis, o);
  if (nu && nu == r.cards.size()) {
    o.append(",\"scv.amd.com/gpu-uuids\":");
    json_quoted(uu, o);
  }
  if (req.has_memory) {
    const int nn = int(std::to_chars(num, num + sizeof num, (long long)req.memory).ptr - num);
    o.append(",\"scv.amd.com/reserved-mb\":\"").append(num, size_t(nn)).push_back('"');
  }
}

// The engine's part of a run: requests from the pods' projections, the batch cycle under the
// engine lock (a device batch drops it while the GPU works), node names. Touches no lane
// store state, so it runs on the lane thread or on the engine worker alike.
void Lane::engine_step(Run& r) {
  const size_t n = r.evs.size();
  r.reqs.resize(n);
  r.ok.assign(n, 1);
  std::vector<uint64_t> eids;
  std::vector<const PodReq*> rp;
  const double tw = mono();
  std::unique_lock<std::recursive_mutex> lk(*emu_);
  {
    const double dw = mono() - tw;
    std::lock_guard<std::mutex> g(stat_mu_);
    st_.lock_wait_s += dw;
  }
  for (size_t k = 0; k < n; ++k) {
    try {
      r.ok[k] = make_req(r.evs[k]->full(), &r.reqs[k]);
    } catch (const std::exception&) {
      r.ok[k] = 0;
    }
    if (k < r.vol_ok.size() && !r.vol_ok[k]) r.ok[k] = 0;   // a claim left the table meanwhile
    if (r.ok[k] && r.pr.vol_limits && !r.reqs[k].pvc_claims.empty()) r.reqs[k].count_vols = true;
    if (r.ok[k] && k < r.vols.size()) {
      // VolumeBinding then VolumeZone (upstream's filter order, the hybrid runner's too), as
      // engine filters; the aliasing pointers keep each claim's constraints alive
      for (const ClaimConsP& c : r.vols[k])
        if (c->has_node && r.pr.vol_node)
          r.reqs[k].vol.push_back({std::shared_ptr<const std::vector<SelTerm>>(c, &c->node), RS_VOLUME_NODE});
      for (const ClaimConsP& c : r.vols[k])
        if (c->has_zone && r.pr.vol_zone)
          r.reqs[k].vol.push_back({std::shared_ptr<const std::vector<SelTerm>>(c, &c->zone), RS_VOLUME_ZONE});
    }
    if (!r.ok[k]) continue;
    eids.push_back(r.ids[k]);
    rp.push_back(&r.reqs[k]);
    r.slot.push_back(k);
  }
  const EngineConfig saved = eng_->config();
  eng_->set_config(r.cfg);
  const double te = mono(), tc = thread_cpu();
  try {
    r.res = eng_->schedule_batch(eids, rp);
  } catch (const std::exception&) {
    r.res.clear();
  }
  {
    const double dc = thread_cpu() - tc;
    std::lock_guard<std::mutex> g(stat_mu_);
    st_.engine_s += mono() - te;
    st_.engine_cpu_s += dc;
    st_.engine_pods += eids.size();
  }
  // restore the caller's configuration unless it re-configured the engine while a device
  // batch had the lock dropped (then its newer configuration stays)
  if (config_eq(eng_->config(), r.cfg)) eng_->set_config(saved);
  r.failed = r.res.size() != eids.size();
  if (o_.engine_delay_us > 0) {
    lk.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(o_.engine_delay_us));
    lk.lock();
  }
  r.names.resize(r.res.size());
  for (size_t k = 0; k < r.res.size(); ++k)
    if (r.res[k].node >= 0) r.names[k] = eng_->node(r.res[k].node).name;
}

// The lane's part after the engine: assumed pods go to BINDING and their Bindings out;
// unschedulable ones to Python; failures back to the queue. Entries are looked up by id: a
// pod deleted, bound elsewhere or taken by Python while its run was on the engine worker is
// gone from by_id_, and whatever the engine reserved for it is released.
void Lane::finish_run(Run& r, std::vector<yk::BindSpec>* binds, std::vector<uint64_t>* tags, std::vector<Fwd>* fwd) {
  const Profile& pr = r.pr;
  std::lock_guard<std::mutex> g(store_mu_);
  auto entry = [&](size_t k) -> Entry* {
    auto it = by_id_.find(r.ids[k]);
    return it != by_id_.end() && it->second->st == INFLIGHT ? it->second : nullptr;
  };
  for (size_t k = 0; k < r.ids.size(); ++k)
    if (!r.ok[k])
      if (Entry* e = entry(k)) {          // a pod the projection cannot express natively
        drop_owned(e, false);
        forward('A', e->ev, nullptr, fwd);
      }
  if (r.failed) {                         // engine failure: the pods retry from the lane queue
    for (size_t k : r.slot) {
      to_release_.push_back(r.ids[k]);
      if (Entry* e = entry(k)) {
        set_state(e, QUEUED);
        e->seq = ++seq_;
        heap_.push(QItem{e->prio, e->seq, e->id});
      }
    }
    return;
  }
  for (size_t q = 0; q < r.res.size(); ++q) {
    const size_t k = r.slot[q];
    const CycleResult& res = r.res[q];
    Entry* e = entry(k);
    if (!e) {
      if (res.node >= 0 && !res.stale) to_release_.push_back(r.ids[k]);
      std::lock_guard<std::mutex> g2(stat_mu_);
      st_.left_in_flight++;
      continue;
    }
    e->t_cycle = r.t0;
    if (res.stale) {
      {
        std::lock_guard<std::mutex> g2(stat_mu_);
        st_.stale_retries++;
      }
      set_state(e, QUEUED);
      e->seq = ++seq_;
      heap_.push(QItem{e->prio, e->seq, e->id});
      continue;
    }
    if (res.node < 0) {
      if (e->ev->full().priority <= pr.preempt_above) {
        // no PostFilter can help: FitError, event, condition and queueing stay native
        e->req = std::make_shared<PodReq>(r.reqs[k]);
        fail_native(e, pr, res, q < r.hinted.size() && r.hinted[q]);
        continue;
      }
      Handoff h;
      h.kind = Handoff::kUnschedulable;
      h.ev = e->ev;
      h.profile = pr.name;
      h.res = res;
      h.t_enqueue = e->t_enq;
      h.t_cycle = r.t0;
      h.attempts = std::max<uint32_t>(1, e->attempts);
      drop_owned(e, false);
      hand_pending_.push_back(std::move(h));
      std::lock_guard<std::mutex> g2(stat_mu_);
      st_.unschedulable++;
      continue;
    }
    e->node = res.node;
    e->node_name = r.names[q];
    e->cards = res.cards;
    e->lab_ev = e->ev;                    // complete (queued pods keep full projections)
    set_state(e, BINDING);
    if (census_on_) census_add(e);
    log_add(*e);
    yk::BindSpec b;
    b.ns = e->ev->p.ns;
    b.name = e->ev->p.name;
    b.uid = e->ev->p.uid;
    b.node = e->node_name;
    annotations(pr, *e, r.reqs[k], res, &b.ann_json);
    binds->push_back(std::move(b));
    tags->push_back(e->id);
    e->bind_out = true;
    std::lock_guard<std::mutex> g2(stat_mu_);
    st_.binding++;
  }
}

void Lane::schedule_some() {
  if (!active_.load() || heap_.empty()) return;
  {
    std::lock_guard<std::mutex> g(in_mu_);
    if (paused_ || run_inflight_) return;
  }
  yk::PodPort* port = port_.load();
  if (!port) return;
  std::vector<Entry*> picked;
  {
    std::lock_guard<std::mutex> g(store_mu_);
    while (!heap_.empty() && (int)picked.size() < o_.batch) {
      const QItem q = heap_.top();
      heap_.pop();
      auto it = by_id_.find(q.id);
      if (it == by_id_.end()) continue;
      Entry* e = it->second;
      if (e->st != QUEUED || e->seq != q.seq || e->prio != q.prio) continue;   // stale heap item
      set_state(e, INFLIGHT);
      e->attempts++;
      e->cycle = ++cycle_;
      picked.push_back(e);
    }
  }
  if (picked.empty()) return;
  const double t0 = mono();
  // consecutive pods of one profile share an engine batch (profiles differ in engine config)
  std::vector<std::shared_ptr<Run>> runs;
  for (size_t i = 0; i < picked.size();) {
    auto r = std::make_shared<Run>();
    r->prof = picked[i]->prof;
    r->pr = lp_[r->prof];
    r->cfg = r->pr.cfg;
    r->t0 = t0;
    for (; i < picked.size() && picked[i]->prof == r->prof; ++i) {
      r->ids.push_back(picked[i]->id);
      r->evs.push_back(picked[i]->ev);
      r->cycles.push_back(picked[i]->cycle);
      // the claim table is the lane thread's: its constraints are copied into the run here
      std::vector<ClaimConsP> cons;
      const yk::PodProj& pp = picked[i]->ev->full();
      r->vol_ok.push_back(!(pp.flags & yk::PF_CLAIMS) || claim_cons(pp, &cons));
      r->vols.push_back(std::move(cons));
    }
    runs.push_back(std::move(r));
  }
  bool async = false;
  {
    std::lock_guard<std::recursive_mutex> lk(*emu_);
    async = o_.async_mode == 2 || (o_.async_mode == 1 && eng_->device_enabled());
  }
  if (async) {
    // the GPU places the batch while this thread keeps serving answers, echoes and deletions;
    // the runs come back through the inbox (kRunDone) and the next batch starts after them
    double oldest = t0;
    for (const Entry* e : picked) oldest = std::min(oldest, e->t_enq);
    if (last_wend_ > 0 && oldest < last_wend_) {
      std::lock_guard<std::mutex> g(stat_mu_);
      st_.idle_queued_s += t0 - last_wend_;
    }
    {
      std::lock_guard<std::mutex> g(in_mu_);
      run_inflight_ = true;
    }
    {
      std::lock_guard<std::mutex> g(wk_mu_);
      wk_jobs_ = std::move(runs);
      wk_flag_.store(true, std::memory_order_relaxed);
    }
    wk_cv_.notify_one();
    return;
  }
  for (auto& r : runs) {
    r->t_wstart = mono();
    engine_step(*r);
    r->t_wend = mono();
  }
  complete_runs(runs);
}

std::vector<Lane::RunRec> Lane::run_log() {
  std::lock_guard<std::mutex> g(rlog_mu_);
  std::vector<RunRec> out;
  out.swap(rlog_);
  return out;
}

void Lane::complete_runs(std::vector<std::shared_ptr<Run>>& runs) {
  std::vector<yk::BindSpec> binds;
  std::vector<uint64_t> tags;
  std::vector<Fwd> fwd;
  {
    const double now = mono();
    std::lock_guard<std::mutex> g(rlog_mu_);
    for (auto& r : runs)
      if (rlog_.size() < 4096) rlog_.push_back(RunRec{r->t0, r->t_wstart, r->t_wend, now, (uint32_t)r->ids.size()});
  }
  {
    // a node removed (its slot maybe reused) between the engine's cycle and now: the pod's
    // reservation went with it, and binding there would skip every filter — retry instead
    std::lock_guard<std::recursive_mutex> lk(*emu_);
    for (auto& r : runs)
      for (auto& res : r->res)
        if (res.node >= 0 && !res.stale && eng_->node_gen(res.node) != res.node_gen) res.stale = true;
    // unschedulable pods: did a node hint since their cycle make them fit there? (upstream's
    // in-flight events + QueueingHint: such a pod retries from backoff instead of parking)
    if (!hints_.empty()) {
      const EngineConfig saved = eng_->config();
      for (auto& r : runs) {
        r->hinted.assign(r->res.size(), 0);
        bool set = false;
        for (size_t q = 0; q < r->res.size(); ++q) {
          if (r->res[q].node >= 0 || r->res[q].stale) continue;
          if (!set) {
            eng_->set_config(r->cfg);
            set = true;
          }
          const size_t k = r->slot[q];
          r->hinted[q] = hinted_since(r->cycles[k], r->reqs[k]);
        }
      }
      eng_->set_config(saved);
    }
  }
  for (auto& r : runs) finish_run(*r, &binds, &tags, &fwd);
  yk::PodPort* port = port_.load();
  if (!binds.empty() && port) port->bind_native(std::move(binds), tags, o_.bind_timeout_s, this);
  {
    std::lock_guard<std::mutex> g(stat_mu_);
    st_.batches++;
  }
  if (!fwd.empty()) publish(std::move(fwd), {});
}

// The engine worker (async device runs): one set of runs at a time, handed back in order.
void Lane::engine_worker() {
  for (;;) {
    std::vector<std::shared_ptr<Run>> jobs;
    spin_until(wk_flag_);
    {
      std::unique_lock<std::mutex> lk(wk_mu_);
      wk_cv_.wait(lk, [&] { return stop_.load() || !wk_jobs_.empty(); });
      if (wk_jobs_.empty()) return;   // stopping and nothing left
      jobs.swap(wk_jobs_);
      wk_flag_.store(false, std::memory_order_relaxed);
    }
    const double ts = mono();
    {
      std::lock_guard<std::mutex> g(stat_mu_);
      st_.handoff_s += ts - jobs.front()->t0;
      st_.async_runs++;
    }
    for (auto& r : jobs) {
      r->t_wstart = ts;
      engine_step(*r);
      r->t_wend = mono();
    }
    Item it;
    it.k = Item::kRunDone;
    it.runs = std::make_shared<std::vector<std::shared_ptr<Run>>>(std::move(jobs));
    {
      std::lock_guard<std::mutex> g(in_mu_);
      push_locked(std::move(it));
    }
    in_cv_.notify_one();
  }
}

namespace {
constexpr size_t kLogCap = 1u << 18;   // live entries; beyond it Python resyncs from a full snapshot
}

void Lane::log_add(const Entry& e) {
  std::lock_guard<std::mutex> g(log_mu_);
  if (!log_on_ || log_full_) return;
  log_adds_[e.id] = log_.size();
  log_.push_back(Change{e.id, true, e.ev, e.node_name, e.cards});
  if (log_.size() - log_dead_ > kLogCap) {     // Python stopped asking: resync from scratch
    log_.clear();
    log_adds_.clear();
    log_dead_ = 0;
    log_full_ = true;
  }
}

void Lane::log_remove(uint64_t id) {
  std::lock_guard<std::mutex> g(log_mu_);
  if (!log_on_ || log_full_) return;
  auto it = log_adds_.find(id);
  if (it != log_adds_.end()) {
    // Python never saw this pod: the add and the release cancel (the event goes with them)
    Change& c = log_[it->second];
    c.id = 0;
    c.ev.reset();
    c.cards.clear();
    c.node.clear();
    log_adds_.erase(it);
    ++log_dead_;
    if (log_dead_ > 4096 && log_dead_ * 2 > log_.size()) {   // compact
      size_t w = 0;
      for (size_t r = 0; r < log_.size(); ++r) {
        if (log_[r].id == 0) continue;
        if (w != r) log_[w] = std::move(log_[r]);
        if (log_[w].add) log_adds_[log_[w].id] = w;
        ++w;
      }
      log_.resize(w);
      log_dead_ = 0;
    }
    return;
  }
  log_.push_back(Change{id, false, nullptr, std::string(), {}});
  if (log_.size() - log_dead_ > kLogCap) {
    log_.clear();
    log_adds_.clear();
    log_dead_ = 0;
    log_full_ = true;
  }
}

void Lane::stop_log() {
  std::lock_guard<std::mutex> g(log_mu_);
  log_on_ = log_full_ = false;
  std::vector<Change>().swap(log_);
  log_adds_.clear();
  log_dead_ = 0;
}

bool Lane::log_on() {
  std::lock_guard<std::mutex> g(log_mu_);
  return log_on_;
}

std::vector<Lane::Change> Lane::changes(bool* full) {
  std::vector<Change> out;
  {
    std::lock_guard<std::mutex> g(log_mu_);
    if (log_on_ && !log_full_) {
      out.reserve(log_.size() - log_dead_);
      for (auto& c : log_)
        if (c.id) out.push_back(std::move(c));
      log_.clear();
      log_adds_.clear();
      log_dead_ = 0;
      *full = false;
      return out;
    }
    log_on_ = true;
    log_full_ = false;
    log_.clear();
    log_adds_.clear();
    log_dead_ = 0;
  }
  // full snapshot; the log (now on) records everything after it
  std::lock_guard<std::mutex> g(store_mu_);
  std::lock_guard<std::mutex> g2(log_mu_);
  log_.clear();
  log_adds_.clear();
  log_dead_ = 0;
  for (auto& kv : by_id_) {
    const Entry* e = kv.second;
    if (e->st == BINDING || e->st == BOUND) out.push_back(Change{e->id, true, e->ev, e->node_name, e->cards});
  }
  *full = true;
  return out;
}

namespace {
uint64_t chash(std::string_view a, std::string_view b = std::string_view(), bool pair = false) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : a) h = (h ^ c) * 1099511628211ull;
  if (pair) {
    h = (h ^ 0x1f) * 1099511628211ull;
    for (unsigned char c : b) h = (h ^ c) * 1099511628211ull;
  }
  return h;
}

// a MatchTerm over census hashes
struct CTerm {
  bool nothing = false;
  std::vector<uint64_t> ns, kv;                        // allowed namespaces, required key=value
  struct X {
    int op;
    uint64_t k;
    std::vector<uint64_t> kvs;
  };
  std::vector<X> x;
};

CTerm compile(const MatchTerm& t) {
  CTerm c;
  c.nothing = t.nothing;
  for (const auto& n : t.namespaces) c.ns.push_back(chash(n));
  for (const auto& kv : t.labels) c.kv.push_back(chash(kv.first, kv.second, true));
  for (const auto& e : t.exprs) {
    CTerm::X x{e.op, chash(e.key), {}};
    for (const auto& v : e.values) x.kvs.push_back(chash(e.key, v, true));
    c.x.push_back(std::move(x));
  }
  return c;
}
}  // namespace

// A census row keeps 64-bit FNV-1a hashes of a pod's first kCLab labels (key, key=value); a
// pod with more labels is `big` and matched exactly against its projection. The hash path is a
// deliberate trade: a false match needs two different label strings with equal 64-bit hashes
// (≈ n²/2^65 for n distinct labels in a cluster — astronomically small), in exchange for a
// census scan that never touches strings.
void Lane::census_fill(CRow& r) {
  const Entry* e = r.e;
  const yk::PodProj& lp = (e->lab_ev ? e->lab_ev : e->ev)->full();
  r.ns = chash(e->ev->p.ns);
  r.deleting = e->ev->p.deleting;
  r.big = lp.labels.size() > (size_t)kCLab;
  r.n = (uint8_t)std::min<size_t>(lp.labels.size(), kCLab);
  for (int i = 0; i < r.n; ++i) {
    r.k[i] = chash(lp.labels[i].first);
    r.kv[i] = chash(lp.labels[i].first, lp.labels[i].second, true);
  }
  r.dirty = false;
}

void Lane::census_add(Entry* e) {
  CRow r;
  r.e = e;
  auto it = cnode_ids_.find(e->node_name);
  if (it == cnode_ids_.end()) {
    it = cnode_ids_.emplace(e->node_name, (uint32_t)cnode_names_.size()).first;
    cnode_names_.push_back(e->node_name);
  }
  r.node = it->second;
  e->crow = (int32_t)census_.size();
  census_.push_back(r);                     // derived (dirty) at the next query
}

void Lane::census_remove(Entry* e) {
  const int32_t i = e->crow;
  e->crow = -1;
  if (i < 0 || i >= (int32_t)census_.size()) return;
  if (i != (int32_t)census_.size() - 1) {
    census_[i] = census_.back();
    census_[i].e->crow = i;
  }
  census_.pop_back();
}

void Lane::stop_census() {
  std::lock_guard<std::mutex> g(store_mu_);
  for (auto& r : census_) r.e->crow = -1;
  std::vector<CRow>().swap(census_);
  census_on_ = false;
}

std::vector<std::unordered_map<std::string, int32_t>> Lane::count_matching(
    const std::vector<std::vector<MatchTerm>>& queries, bool skip_deleting) {
  std::vector<std::unordered_map<std::string, int32_t>> out(queries.size());
  if (queries.empty()) return out;
  const double t0 = mono();
  std::vector<std::vector<CTerm>> cq(queries.size());
  for (size_t q = 0; q < queries.size(); ++q)
    for (const auto& t : queries[q]) cq[q].push_back(compile(t));
  std::unique_lock<std::mutex> g(store_mu_);
  if (!census_on_) {
    census_on_ = true;
    for (auto& kv : by_id_)
      if ((kv.second->st == BINDING || kv.second->st == BOUND) && kv.second->crow < 0) census_add(kv.second);
  }
  std::vector<std::vector<int32_t>> cnt(queries.size(), std::vector<int32_t>(cnode_names_.size(), 0));
  auto has = [](const uint64_t* a, int n, uint64_t v) {
    for (int i = 0; i < n; ++i)
      if (a[i] == v) return true;
    return false;
  };
  for (auto& r : census_) {
    if (r.dirty) census_fill(r);
    if (skip_deleting && r.deleting) continue;
    for (size_t q = 0; q < cq.size(); ++q) {
      bool all = true;
      if (r.big) {                              // more labels than a row holds: exact path
        const yk::PodProj& lp = (r.e->lab_ev ? r.e->lab_ev : r.e->ev)->full();
        for (const MatchTerm& t : queries[q])
          if (!t.matches(r.e->ev->p.ns, lp.labels)) {
            all = false;
            break;
          }
      } else {
        for (const CTerm& t : cq[q]) {
          if (t.nothing || (!t.ns.empty() && std::find(t.ns.begin(), t.ns.end(), r.ns) == t.ns.end())) {
            all = false;
            break;
          }
          for (uint64_t v : t.kv)
            if (!has(r.kv, r.n, v)) {
              all = false;
              break;
            }
          for (size_t j = 0; all && j < t.x.size(); ++j) {
            const CTerm::X& x = t.x[j];
            bool in = false;
            for (uint64_t v : x.kvs) in |= has(r.kv, r.n, v);
            switch (x.op) {
              case 0: all = in; break;
              case 1: all = !in; break;
              case 2: all = has(r.k, r.n, x.k); break;
              case 3: all = !has(r.k, r.n, x.k); break;
              default: all = false;
            }
          }
          if (!all) break;
        }
      }
      if (all) cnt[q][r.node]++;
    }
  }
  const uint64_t walked = census_.size();
  for (size_t q = 0; q < cq.size(); ++q)
    for (size_t n = 0; n < cnt[q].size(); ++n)
      if (cnt[q][n]) out[q][cnode_names_[n]] = cnt[q][n];
  g.unlock();
  std::lock_guard<std::mutex> g2(stat_mu_);
  st_.census_calls++;
  st_.census_entries += walked;
  st_.census_s += mono() - t0;
  return out;
}

void Lane::signal_python() {
  bool sig = false;
  {
    std::lock_guard<std::mutex> g(out_mu_);
    if (!signalled_) signalled_ = sig = true;
  }
  if (sig) {
    const uint64_t one = 1;
    ssize_t w = ::write(efd_, &one, sizeof one);
    (void)w;
  }
}

void Lane::set_watermark(uint64_t n) {
  watermark_.store(n, std::memory_order_relaxed);
  if (scheduled_.load(std::memory_order_relaxed) >= n) signal_python();
}

void Lane::pause(bool on) {
  std::unique_lock<std::mutex> lk(in_mu_);
  paused_ = on;
  in_cv_.notify_all();
  if (on) idle_cv_.wait(lk, [&] { return (!busy_ && !run_inflight_) || stop_.load(); });
}

// ------------------------------------------------------------------ native unschedulable path
// (lane thread). upstream's FitError → FailedScheduling event → PodScheduled=False condition →
// AddUnschedulableIfNotPresent: unschedulableQ, or podBackoffQ when a move request arrived since
// the pod's cycle began (moveRequestCycle) or a node hint since then makes it fit.

std::string Lane::fit_error(const CycleResult& r, const yk::PodProj& p) const {
  std::vector<std::string> parts;
  for (int i = 1; i < (int)r.reason_counts.size() && i < RS_NUM; ++i) {
    if (!r.reason_counts[i]) continue;
    if (i == RS_EXT_RESOURCES) {
      // framework/scheduler.py::ext_text: "Insufficient <the pod's resources beyond cpu/memory>"
      std::vector<std::string> names;
      for (const auto& x : p.cold().ext) names.push_back(x.first);
      std::sort(names.begin(), names.end());
      std::string t = "Insufficient ";
      for (size_t k = 0; k < names.size(); ++k) t += (k ? "/" : "") + names[k];
      if (names.empty()) t += "extended resources";
      parts.push_back(std::to_string(r.reason_counts[i]) + " " + t);
      continue;
    }
    parts.push_back(std::to_string(r.reason_counts[i]) + " " + reason_text(i));
  }
  std::sort(parts.begin(), parts.end());
  std::string m = "0/" + std::to_string(r.evaluated) + " nodes are available: ";
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i) m += ", ";
    m += parts[i];
  }
  m += ".";
  return m;
}

double Lane::backoff_of(const Entry& e) const {
  // podInitialBackoffSeconds × 2^(attempts−1), capped at podMaxBackoffSeconds (queue.py)
  double d = o_.initial_backoff_s;
  for (uint32_t a = 1; a < e.attempts && d < o_.max_backoff_s; ++a) d *= 2;
  return std::min(d, o_.max_backoff_s);
}

void Lane::activate(Entry* e) {
  set_state(e, QUEUED);
  e->seq = ++seq_;
  heap_.push(QItem{e->prio, e->seq, e->id});
}

void Lane::to_backoff(Entry* e, double until) {
  set_state(e, BACKOFF);
  e->bseq = ++bseq_;
  bheap_.push(BItem{until, e->bseq, e->id});
}

// a waiting pod moved by a cluster event: backoffQ while its backoff runs, else activeQ
void Lane::route(Entry* e, double now) {
  const double b = backoff_of(*e);
  if (now - e->t_fail < b) to_backoff(e, e->t_fail + b);
  else activate(e);
}

void Lane::patch_condition(Entry& e, const std::string& msg) {
  // upstream v1.20 updatePod: the condition goes out as a strategic merge patch of pods/status
  // (conditions merged by type, so other conditions on the pod stay), and not at all when the
  // pod already carries the same PodScheduled=False reason and message
  yk::PodPort* port = port_.load();
  if (!port) return;
  // upstream podutil.UpdatePodCondition against the pod's current condition (the latest event
  // of the entry); while none is visible yet, the condition this lane last wrote stands in for
  // it (its echo is on the way). A condition another writer changed is written again.
  const yk::PodProj& cur = e.ev->full();
  bool same;
  std::string ltt;
  if (const auto& c = cur.sched_cond) {
    same = c->status == "False" && c->reason == "Unschedulable" && c->msg == msg;
    if (c->status == "False" && !c->ltt.empty()) ltt = c->ltt;   // no transition
  } else {
    same = !e.cond_msg.empty() && e.cond_msg == msg;
    ltt = e.cond_ltt;
  }
  if (same) {
    std::lock_guard<std::mutex> g(stat_mu_);
    st_.status_patches_skipped++;
    return;
  }
  if (ltt.empty()) ltt = rfc3339(wall());
  e.cond_msg = msg;
  e.cond_ltt = ltt;
  std::string b;
  b.reserve(200 + msg.size());
  b += "{\"status\":{\"conditions\":[{\"type\":\"PodScheduled\",\"status\":\"False\",\"lastProbeTime\":null,"
       "\"lastTransitionTime\":";
  json_str(ltt, b);
  b += ",\"reason\":\"Unschedulable\",\"message\":";
  json_str(msg, b);
  b += "}]}}";
  const std::string path = "/api/v1/namespaces/" + e.ev->p.ns + "/pods/" + e.ev->p.name + "/status";
  static std::atomic<uint64_t> seq{0};
  port->request_native("PATCH", path, std::move(b), true, 30.0, kEventTag | kPatchBit | (++seq & 0xffffffffull), this,
                       "application/strategic-merge-patch+json");
  std::lock_guard<std::mutex> g(stat_mu_);
  st_.status_patches++;
}

void Lane::fail_native(Entry* e, const Profile& pr, const CycleResult& res, bool hinted) {
  const double now = mono();
  e->t_fail = now;
  const std::string msg = fit_error(res, e->ev->full());
  {
    std::lock_guard<std::mutex> g(stat_mu_);
    st_.unschedulable++;
    st_.native_failed++;
    st_.by_profile[pr.name].second++;
    if (o_.events) {
      st_.events_recorded++;
      if ((int)ev_q_.size() >= o_.event_buffer) st_.events_dropped++;
      else ev_q_.push_back(PendingEvent{e->ev->p.ns, e->ev->p.name, e->ev->p.uid, std::string(), pr.name, wall(),
                                        msg.substr(0, 1024)});
    }
  }
  patch_condition(*e, msg);
  if (move_cycle_ >= (int64_t)e->cycle || hinted) {
    to_backoff(e, now + backoff_of(*e));
  } else {
    set_state(e, PARKED);
    e->t_park = now;
    parked_[e->id] = e;
  }
}

// caller holds the engine lock with the pod's profile configuration applied
bool Lane::hinted_since(uint64_t cycle, const PodReq& req) {
  if (hint_dropped_ && hint_dropped_cycle_ >= cycle) return true;   // too old to tell: retry
  uint64_t n, m, c;
  for (auto it = hints_.rbegin(); it != hints_.rend(); ++it) {
    if (it->first < cycle) break;
    if (it->second >= 0 && it->second < eng_->num_nodes() && eng_->node(it->second).alive &&
        eng_->filter_node(req, it->second, &n, &m, &c) == RS_OK)
      return true;
  }
  return false;
}

void Lane::move_parked(const std::vector<Entry*>& which) {
  if (which.empty()) return;
  const double now = mono();
  std::lock_guard<std::mutex> g(store_mu_);
  uint64_t moved = 0;
  for (Entry* e : which) {
    if (e->st != PARKED) continue;
    parked_.erase(e->id);
    route(e, now);
    ++moved;
  }
  std::lock_guard<std::mutex> g2(stat_mu_);
  st_.moved += moved;
}

void Lane::process_moves() {
  if (pending_moves_.empty()) return;
  bool all = false;
  for (int32_t n : pending_moves_) all |= n < 0;
  std::vector<Entry*> mv;
  if (all) {
    move_cycle_ = (int64_t)cycle_;
    for (auto& kv : parked_) mv.push_back(kv.second);
  } else {
    // queueing hints: a node's filter-visible capacity grew; a parked pod moves only if it now
    // passes every filter of its profile on that node (upstream QueueingHint, exact here)
    std::lock_guard<std::recursive_mutex> lk(*emu_);
    const EngineConfig saved = eng_->config();
    int cur = -2;
    uint64_t n, m, c;
    for (int32_t node : pending_moves_) {
      hints_.emplace_back(cycle_, node);
      if (hints_.size() > 256) {
        hint_dropped_cycle_ = hints_.front().first;
        hint_dropped_ = true;
        hints_.erase(hints_.begin());
      }
    }
    const int nn = eng_->num_nodes();
    for (auto& kv : parked_) {
      Entry* e = kv.second;
      bool go = !e->req || e->prof < 0 || e->prof >= (int)lp_.size();
      for (size_t k = 0; !go && k < pending_moves_.size(); ++k) {
        const int32_t node = pending_moves_[k];
        if (node < 0 || node >= nn || !eng_->node(node).alive) continue;
        if (e->prof != cur) {
          eng_->set_config(lp_[e->prof].cfg);
          cur = e->prof;
        }
        go = eng_->filter_node(*e->req, node, &n, &m, &c) == RS_OK;
      }
      if (go) mv.push_back(e);
    }
    eng_->set_config(saved);
  }
  pending_moves_.clear();
  move_parked(mv);
}

// backoffQ pods whose backoff ended → activeQ; unschedulableQ pods parked longer than the
// flush interval → activeQ / backoffQ (flushBackoffQCompleted, flushUnschedulableQLeftover)
void Lane::flush_queues(double now) {
  if (bheap_.empty() && parked_.empty()) return;
  std::vector<Entry*> left;
  if (!parked_.empty() && now >= next_leftover_) {
    for (auto& kv : parked_)
      if (now - kv.second->t_park > o_.unsched_flush_s) left.push_back(kv.second);
    next_leftover_ = now + std::max(0.05, std::min(1.0, o_.unsched_flush_s / 4));
  }
  if (!left.empty()) move_parked(left);
  if (bheap_.empty() || bheap_.top().until > now) return;
  std::lock_guard<std::mutex> g(store_mu_);
  uint64_t n = 0;
  while (!bheap_.empty() && bheap_.top().until <= now) {
    const BItem b = bheap_.top();
    bheap_.pop();
    auto it = by_id_.find(b.id);
    if (it == by_id_.end() || it->second->st != BACKOFF || it->second->bseq != b.seq) continue;   // stale
    activate(it->second);
    ++n;
  }
  std::lock_guard<std::mutex> g2(stat_mu_);
  st_.retried += n;
}

double Lane::next_timer() const {
  double t = 1e300;
  if (!bheap_.empty()) t = bheap_.top().until;
  if (!parked_.empty()) t = std::min(t, std::max(next_leftover_, mono() + 0.05));
  return t;
}

void Lane::record_scheduled(const Entry& e) {
  if (!o_.events) return;
  std::lock_guard<std::mutex> g(stat_mu_);
  st_.events_recorded++;
  if ((int)ev_q_.size() >= o_.event_buffer) {     // client-go DropIfChannelFull
    st_.events_dropped++;
    return;
  }
  const std::string& prof = e.prof >= 0 && e.prof < (int)lp_.size() ? lp_[e.prof].name : std::string();
  ev_q_.push_back(PendingEvent{e.ev->p.ns, e.ev->p.name, e.ev->p.uid, e.node_name, prof, wall(), std::string()});
}

void Lane::flush_events() {
  if (ev_q_.empty()) return;
  yk::PodPort* port = port_.load();
  if (!port) return;
  const double now = mono();
  const double cap = o_.event_burst > 0 ? o_.event_burst : 1;
  if (o_.event_qps > 0) ev_tokens_ = std::min(cap, ev_tokens_ + (now - ev_last_) * o_.event_qps);
  else ev_tokens_ = cap;
  ev_last_ = now;
  while (!ev_q_.empty() && ev_tokens_ >= 1.0) {
    ev_tokens_ -= 1.0;
    PendingEvent pe = std::move(ev_q_.front());
    ev_q_.pop_front();
    const std::string ctl = pe.profile.empty() ? std::string("yoda-scheduler") : pe.profile;
    const bool failed = !pe.note.empty();
    const char* reason = failed ? "FailedScheduling" : "Scheduled";
    const char* typ = failed ? "Warning" : "Normal";
    const std::string note = failed ? pe.note : "Successfully assigned " + pe.ns + "/" + pe.name + " to " + pe.node;
    const std::string t = micro_time(pe.ts);
    std::string b;
    b.reserve(512);
    std::string path;
    if (failed) {
      // an isomorphic repeat (same pod, reason, message, controller) bumps the first event's
      // series instead of creating another (framework/events.py::_write_v1)
      std::string key = pe.ns + "/" + pe.name + "\x1f" + ctl + "\x1f" + pe.note;
      auto it = ev_dedup_.find(key);
      if (it != ev_dedup_.end()) {
        const int count = ++it->second.second;
        if (o_.events_v1) {
          b += "{\"series\":{\"count\":" + std::to_string(count) + ",\"lastObservedTime\":";
          json_str(t, b);
          b += "}}";
          path = "/apis/events.k8s.io/v1/namespaces/" + pe.ns + "/events/" + it->second.first;
        } else {
          b += "{\"count\":" + std::to_string(count) + ",\"lastTimestamp\":";
          json_str(t, b);
          b += "}";
          path = "/api/v1/namespaces/" + pe.ns + "/events/" + it->second.first;
        }
        port->request_native("PATCH", path, std::move(b), false, 30.0, kEventTag | ++ev_seq_, this);
        continue;
      }
      if (ev_dedup_.size() > 10000) ev_dedup_.clear();
    }
    char seq[24];
    snprintf(seq, sizeof seq, "%08llx", (unsigned long long)++ev_seq_);
    const std::string name = pe.name + "." + o_.name_prefix + seq;
    if (failed) ev_dedup_.emplace(pe.ns + "/" + pe.name + "\x1f" + ctl + "\x1f" + pe.note, std::make_pair(name, 1));
    if (o_.events_v1) {
      // framework/events.py::EventRecorder._new_v1
      b += "{\"apiVersion\":\"events.k8s.io/v1\",\"kind\":\"Event\",\"metadata\":{\"name\":";
      json_str(name, b);
      b += ",\"namespace\":";
      json_str(pe.ns, b);
      b += "},\"eventTime\":";
      json_str(t, b);
      b += ",\"reportingController\":";
      json_str(ctl, b);
      b += ",\"reportingInstance\":";
      json_str(ctl + "-" + o_.host, b);
      b += failed ? ",\"action\":\"Scheduling\",\"reason\":" : ",\"action\":\"Binding\",\"reason\":";
      json_str(reason, b);
      b += ",\"regarding\":{\"apiVersion\":\"v1\",\"kind\":\"Pod\",\"name\":";
      json_str(pe.name, b);
      b += ",\"namespace\":";
      json_str(pe.ns, b);
      b += ",\"uid\":";
      json_str(pe.uid, b);
      b += "},\"note\":";
      json_str(note, b);
      b += ",\"type\":";
      json_str(typ, b);
      b += "}";
      path = "/apis/events.k8s.io/v1/namespaces/" + pe.ns + "/events";
    } else {
      b += "{\"apiVersion\":\"v1\",\"kind\":\"Event\",\"metadata\":{\"name\":";
      json_str(name, b);
      b += ",\"namespace\":";
      json_str(pe.ns, b);
      b += "},\"involvedObject\":{\"kind\":\"Pod\",\"name\":";
      json_str(pe.name, b);
      b += ",\"namespace\":";
      json_str(pe.ns, b);
      b += ",\"uid\":";
      json_str(pe.uid, b);
      b += "},\"reason\":";
      json_str(reason, b);
      b += ",\"message\":";
      json_str(note, b);
      b += ",\"type\":";
      json_str(typ, b);
      b += ",\"source\":{\"component\":";
      json_str(ctl, b);
      b += "},\"firstTimestamp\":";
      json_str(t, b);
      b += ",\"lastTimestamp\":";
      json_str(t, b);
      b += ",\"count\":1}";
      path = "/api/v1/namespaces/" + pe.ns + "/events";
    }
    port->request_native("POST", path, std::move(b), false, 30.0, kEventTag | ev_seq_, this);
  }
}

void Lane::run() {
  std::deque<Item> work;
  for (;;) {
    {
      std::unique_lock<std::mutex> lk(in_mu_);
      // paused: only a run already on the engine worker comes back (pause() waits for it)
      auto ready = [&] {
        return stop_.load() || (!inbox_.empty() && (!paused_ || run_inflight_)) ||
               (!paused_ && !run_inflight_ && active_.load() && !heap_.empty());
      };
      if (!ready() && run_inflight_ && o_.spin_us > 0) {
        // a device run is out: its return (or an answer, an echo) is likely within the spin,
        // and a futex wake-up would add tens of µs to the engine worker's idle gap
        lk.unlock();
        spin_until(inbox_flag_);
        lk.lock();
      }
      if (!ready()) {
        double wait = next_timer() - mono();             // backoff expiry, unschedulableQ flush
        if (!ev_q_.empty() && o_.event_qps > 0) wait = std::min(wait, (1.0 - ev_tokens_) / o_.event_qps);
        if (wait < 1e9) {
          wait = std::max(0.0005, wait);
          // system_clock deadline: pthread_cond_timedwait (steady-clock waits use
          // pthread_cond_clockwait, which ThreadSanitizer does not model)
          in_cv_.wait_until(lk, std::chrono::system_clock::now() +
                                    std::chrono::duration_cast<std::chrono::system_clock::duration>(
                                        std::chrono::duration<double>(wait)), ready);
        } else {
          in_cv_.wait(lk, ready);
        }
      }
      if (stop_.load()) break;
      work.swap(inbox_);
      inbox_flag_.store(false, std::memory_order_relaxed);
      busy_ = true;
    }
    std::vector<Fwd> fwd;
    std::vector<std::pair<uint64_t, std::vector<Fwd>>> relists;
    std::vector<std::shared_ptr<Run>> done;
    {
      std::lock_guard<std::mutex> g(store_mu_);
      for (auto& it : work) {
        switch (it.k) {
          case Item::kRunDone:
            for (auto& r : *it.runs) done.push_back(r);
            break;
          case Item::kEvent:
            handle_event(it.type, it.ev, &fwd);
            grave_.push_back(std::move(it.ev));
            break;
          case Item::kAnswer: handle_answer(it.tag, it.status, it.body, it.t); break;
          case Item::kProfiles: apply_profiles(&fwd); break;
          case Item::kGates: apply_gates(&fwd); break;
          case Item::kClaims: apply_claims(&fwd); break;
          case Item::kMove: pending_moves_.push_back(it.status); break;
          case Item::kRelist: {
            std::vector<Fwd> out;
            handle_relist(*it.items, &out);
            relists.emplace_back(it.token, std::move(out));
            break;
          }
        }
      }
    }
    work.clear();
    if (!grave_.empty()) {
      // the I/O thread allocated these events: freed there, their memory goes back to its
      // malloc cache instead of both threads contending for its arena (native profile of the
      // reset: a third of the lane's time in those frees, profiles/bench/r6/natprof/)
      if (yk::PodPort* port = port_.load()) port->recycle(std::move(grave_));
      grave_.clear();
    }
    // a lane release is a move request for the lane's own waiting pods too (AssignedPodDelete);
    // moves apply before this turn's runs complete (upstream's moveRequestCycle rule)
    if (out_moves_pending_ && !parked_.empty()) pending_moves_.push_back(-1);
    else if (out_moves_pending_) move_cycle_ = (int64_t)cycle_;
    process_moves();
    flush_queues(mono());
    auto release_pending = [&] {
      if (to_release_.empty() && meta_pending_.empty()) return;
      std::lock_guard<std::recursive_mutex> lk(*emu_);
      for (uint64_t id : to_release_) eng_->release(id);
      to_release_.clear();
      for (auto& m : meta_pending_) {
        const yk::PodProj& q = m.second->full();
        eng_->set_pod_meta(m.first, intern_labels(q.labels), q.deleting);
      }
      meta_pending_.clear();
    };
    if (!done.empty()) {
      release_pending();                  // deletions of this turn free capacity for the next run
      // after this turn's events: a pod deleted meanwhile is already out of by_id_
      last_wend_ = done.back()->t_wend;
      {
        std::lock_guard<std::mutex> g(stat_mu_);
        st_.return_s += mono() - last_wend_;
      }
      {
        std::lock_guard<std::mutex> g(in_mu_);
        run_inflight_ = false;
      }
      // the next batch goes to the engine worker first: its reservations already hold in the
      // engine, so building and posting this batch's Bindings overlaps the next device run
      schedule_some();
      complete_runs(done);
    }
    release_pending();
    if (!fwd.empty() || !hand_pending_.empty()) publish(std::move(fwd), std::move(hand_pending_));
    hand_pending_.clear();
    if (out_moves_pending_) {
      bool sig = false;
      {
        std::lock_guard<std::mutex> g(out_mu_);
        out_moves_ += out_moves_pending_;
        if (!signalled_) signalled_ = sig = true;
      }
      out_moves_pending_ = 0;
      if (sig) {
        const uint64_t one = 1;
        ssize_t w = ::write(efd_, &one, sizeof one);
        (void)w;
      }
    }
    if (!relists.empty()) {
      std::lock_guard<std::mutex> g(in_mu_);
      for (auto& r : relists) {
        relist_out_[r.first] = std::move(r.second);
        relist_done_ = std::max(relist_done_, r.first);
      }
      relist_cv_.notify_all();
    }
    schedule_some();
    if (!hand_pending_.empty()) {
      publish({}, std::move(hand_pending_));
      hand_pending_.clear();
    }
    release_pending();
    flush_events();
    {
      std::lock_guard<std::mutex> g(in_mu_);
      busy_ = false;
    }
    idle_cv_.notify_all();
  }
  std::lock_guard<std::mutex> g(in_mu_);
  busy_ = false;
  idle_cv_.notify_all();
}

}  // namespace yoda
