// Native scheduling engine: see engine.hpp for the design notes.
#include "engine.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cctype>
#include <cstring>

#include "yoda_dev_abi.h"
#include <cstdlib>
#include <stdexcept>

namespace yoda {

// (key, value) pair of interned strings as one map key
static inline uint64_t pair_key(int32_t k, int32_t v) { return ((uint64_t)(uint32_t)k << 32) | (uint32_t)v; }

// Python's // on int64
static inline int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}

// ============================================================== ThreadPool
ThreadPool::ThreadPool(int n) {
  for (int i = 0; i < n - 1; ++i) workers_.emplace_back([this] { worker(); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::worker() {
  uint64_t seen = 0;
  for (;;) {
    const std::function<void(int, int)>* job;
    int n, grain;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      // A worker that wakes after the caller already drained and retired the job must not
      // join it: the caller may reset next_ for the following job while this worker would
      // still be looping on the retired (dangling) one.
      if (job_ == nullptr) continue;
      job = job_;
      n = job_n_;
      grain = job_grain_;
      ++active_;
    }
    for (;;) {
      int b = next_.fetch_add(grain);
      if (b >= n) break;
      (*job)(b, std::min(n, b + grain));
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      if (--active_ == 0) done_cv_.notify_all();
    }
  }
}

void ThreadPool::parallel_for(int n, int grain, const std::function<void(int, int)>& fn) {
  if (workers_.empty() || n <= grain) {
    fn(0, n);
    return;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = &fn;
    job_n_ = n;
    job_grain_ = grain;
    next_.store(0);
    ++gen_;
  }
  cv_.notify_all();
  for (;;) {
    int b = next_.fetch_add(grain);
    if (b >= n) break;
    fn(b, std::min(n, b + grain));
  }
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return active_ == 0 && next_.load() >= n; });
  job_ = nullptr;
}

// ============================================================== Engine basics
Engine::Engine(bool compat, int threads) : compat_(compat) {
  if (threads > 1) pool_ = new ThreadPool(threads);
  intern("");
  unsched_key_ = intern("node.kubernetes.io/unschedulable");
  any_ip_ = intern("0.0.0.0");
  tcp_ = intern("TCP");
  dev_ext_res_ = intern("ephemeral-storage");
  field_name_key_ = intern("@metadata.name");   // '@' is not valid in a label key
}

Engine::~Engine() {
  disable_device();
  delete pool_;
}

EngineConfig Engine::config() const {
  EngineConfig c;
  c.filters = filters_;
  std::copy(score_w_, score_w_ + S_NUM, c.score_w);
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < 3; ++j) c.alloc_w[k][j] = alloc_w_[k][j];
  c.wt = wt_;
  c.settle_s = settle_s_;
  c.spread_defaults = spread_defaults_;
  c.ext_ignored = ext_ignored_;
  c.ext_ignored_groups = ext_ignored_groups_;
  c.hard_pod_affinity_weight = hard_aff_w_;
  return c;
}

void Engine::set_config(const EngineConfig& c) {
  filters_ = c.filters;
  std::copy(c.score_w, c.score_w + S_NUM, score_w_);
  for (int k = 0; k < 2; ++k)
    for (int j = 0; j < 3; ++j) alloc_w_[k][j] = c.alloc_w[k][j];
  wt_ = c.wt;
  settle_s_ = c.settle_s;
  spread_defaults_ = c.spread_defaults;
  ext_ignored_ = c.ext_ignored;
  ext_ignored_groups_ = c.ext_ignored_groups;
  hard_aff_w_ = c.hard_pod_affinity_weight;
}

int32_t Engine::intern(const std::string& s) {
  auto it = string_idx_.find(s);
  if (it != string_idx_.end()) return it->second;
  int32_t id = (int32_t)strings_.size();
  strings_.push_back(s);
  string_idx_.emplace(s, id);
  return id;
}

int32_t Engine::upsert_node(const std::string& name) {
  auto it = node_idx_.find(name);
  if (it != node_idx_.end()) return it->second;
  int32_t idx;
  if (!free_slots_.empty()) {
    idx = free_slots_.back();
    free_slots_.pop_back();
    nodes_[idx] = Node();
  } else {
    idx = (int32_t)nodes_.size();
    nodes_.emplace_back();
  }
  nodes_[idx].name = name;
  nodes_[idx].alive = true;
  nodes_[idx].gen = ++gen_counter_;
  node_idx_[name] = idx;
  ++live_;
  mark_dirty(idx);
  return idx;
}

int32_t Engine::node_index(const std::string& name) const {
  auto it = node_idx_.find(name);
  return it == node_idx_.end() ? -1 : it->second;
}

void Engine::remove_node(int32_t idx) {
  if (idx < 0 || idx >= (int32_t)nodes_.size() || !nodes_[idx].alive) return;
  // drop reservations that point at this node
  for (int32_t si : nodes_[idx].pods) {
    Assignment& a = slab_[si];
    if (!a.live || a.node != idx) continue;
    if (a.aff) {
      aff_holders_.erase(a.pod);
      anti_holders_.erase(a.pod);
      aff_set_remove(a);
    }
    free_entry(si);
  }
  node_idx_.erase(nodes_[idx].name);
  hard_taint_nodes_ -= nodes_[idx].hard_taint;
  prefer_taint_nodes_ -= nodes_[idx].prefer_taint;
  index_node_extras(nodes_[idx], -1);
  for (auto& kv : nodes_[idx].labels)
    if (--label_key_nodes_[kv.first] <= 0) label_key_nodes_.erase(kv.first);
  nodes_[idx] = Node();
  nodes_[idx].alive = false;
  nodes_[idx].gen = ++gen_counter_;
  if (batch_in_flight_.load(std::memory_order_acquire)) removed_in_flight_.push_back(idx);
  free_slots_.push_back(idx);
  --live_;
  mark_dirty(idx);
}

void Engine::set_node_meta(int32_t idx, bool unschedulable, const std::vector<std::pair<int32_t, int32_t>>& labels,
                           const std::vector<Taint>& taints, int64_t cpu_m, int64_t mem, int64_t pods) {
  Node& n = nodes_.at(idx);
  n.unschedulable = unschedulable;
  for (auto& kv : n.labels)
    if (--label_key_nodes_[kv.first] <= 0) label_key_nodes_.erase(kv.first);
  n.labels.clear();
  for (auto& kv : labels) n.labels[kv.first] = kv.second;
  for (auto& kv : n.labels) ++label_key_nodes_[kv.first];
  n.taints = taints;
  hard_taint_nodes_ -= n.hard_taint;
  prefer_taint_nodes_ -= n.prefer_taint;
  n.hard_taint = n.prefer_taint = false;
  for (const Taint& t : taints) {
    if (t.effect == kPreferNoSchedule) n.prefer_taint = true;
    else n.hard_taint = true;
  }
  hard_taint_nodes_ += n.hard_taint;
  prefer_taint_nodes_ += n.prefer_taint;
  n.alloc_cpu_m = cpu_m;
  n.alloc_mem = mem;
  n.alloc_pods = pods;
  mark_dirty(idx);
}

double Engine::now() const {
  if (fixed_now_ >= 0) return fixed_now_;
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}

void Engine::set_cards(int32_t idx, std::vector<Card> cards, uint64_t card_number, uint64_t free_sum,
                       uint64_t total_sum, bool stale, double sample_ts) {
  Node& n = nodes_.at(idx);
  // keep the ledger: reservations are per card index
  std::vector<uint64_t> res(cards.size(), 0);
  std::vector<int32_t> pods(cards.size(), 0);
  for (size_t i = 0; i < cards.size() && i < n.cards.size(); ++i) {
    res[i] = n.cards[i].reserved_mb;
    pods[i] = n.cards[i].pods;
  }
  n.cards = std::move(cards);
  for (size_t i = 0; i < n.cards.size(); ++i) {
    n.cards[i].reserved_mb = res[i];
    n.cards[i].pending_mb = 0;
    n.cards[i].pods = pods[i];
  }
  // recompute which reservations the new sample cannot reflect yet
  n.sample_ts = sample_ts;
  for (int32_t si : n.pods) {
    const Assignment& a = slab_[si];
    if (!is_pending(n, a)) continue;
    for (int32_t c : a.cards)
      if (c < (int32_t)n.cards.size()) n.cards[c].pending_mb += a.mb;
  }
  n.card_number = card_number;
  n.free_sum = free_sum;
  n.total_sum = total_sum;
  n.has_scv = true;
  n.stale = stale;
  int32_t np = 0;
  for (auto& c : n.cards) np = std::max(np, c.phys + 1);
  if (np != n.nphys) {
    n.nphys = np;
    n.link_q.assign((size_t)np * np, 10000);
  }
  mark_dirty(idx);
}

void Engine::clear_scv(int32_t idx) {
  Node& n = nodes_.at(idx);
  n.has_scv = false;
  n.cards.clear();
  n.card_number = n.free_sum = n.total_sum = 0;
  n.nphys = 0;
  n.link_q.clear();
  mark_dirty(idx);
}

void Engine::set_links(int32_t idx, int32_t nphys, std::vector<int32_t> q) {
  Node& n = nodes_.at(idx);
  if ((int64_t)q.size() != (int64_t)nphys * nphys) throw std::invalid_argument("link matrix size");
  n.nphys = nphys;
  n.link_q = std::move(q);
  mark_dirty(idx);
}

bool Engine::host_port(int64_t port, const std::string& protocol, const std::string& ip, HostPort* out) {
  // upstream v1.20 framework.HostPortInfo: sanitize (ip "" → 0.0.0.0, protocol "" → TCP); a port
  // <= 0 is no host port (Add / CheckConflict ignore it)
  if (port <= 0 || port > INT32_MAX) return false;
  out->port = (int32_t)port;
  out->proto = protocol.empty() ? tcp_ : intern(protocol);
  out->ip = ip.empty() ? any_ip_ : intern(ip);
  return true;
}

void Engine::set_node_vol_limits(int32_t idx, std::vector<std::pair<int32_t, int64_t>> limits) {
  std::sort(limits.begin(), limits.end());
  nodes_.at(idx).vol_limits = std::move(limits);
}

bool Engine::vols_fit(const PodReq& req, const Node& n) const {
  // plugins/volumes.py NodeVolumeLimits.filter: per CSI driver the node limits, the unique
  // volumes of the node's pods plus the pod's own must not exceed the limit
  std::vector<std::pair<int32_t, int32_t>> mine;   // (driver, volume id) of the pod's claims
  for (int32_t c : req.pvc_claims) {
    auto it = claim_vol_.find(c);
    if (it != claim_vol_.end()) mine.push_back(it->second);
  }
  if (mine.empty()) return true;
  std::sort(mine.begin(), mine.end());
  mine.erase(std::unique(mine.begin(), mine.end()), mine.end());
  for (size_t i = 0; i < mine.size();) {
    const int32_t d = mine[i].first;
    size_t j = i;
    while (j < mine.size() && mine[j].first == d) ++j;
    auto lim = std::lower_bound(n.vol_limits.begin(), n.vol_limits.end(), std::make_pair(d, INT64_MIN));
    if (lim != n.vol_limits.end() && lim->first == d) {
      std::unordered_set<int32_t> ids;
      for (const auto& kv : n.claims) {
        auto it = claim_vol_.find(kv.first);
        if (it != claim_vol_.end() && it->second.first == d) ids.insert(it->second.second);
      }
      // upstream CSILimits: only a driver the pod adds a new volume to is compared
      bool adds = false;
      for (size_t k = i; k < j; ++k) adds = ids.insert(mine[k].second).second || adds;
      if (adds && (int64_t)ids.size() > lim->second) return false;
    }
    i = j;
  }
  return true;
}

bool Engine::ports_free(const PodReq& req, const Node& n) const {
  // HostPortInfo.CheckConflict: a 0.0.0.0 request conflicts with the (protocol, port) on any ip;
  // a specific ip only with the same ip or 0.0.0.0
  for (const HostPort& h : req.host_ports) {
    if (h.ip == any_ip_) {
      if (n.ports_any.count({h.proto, h.port})) return false;
    } else if (n.ports.count(HostPort{any_ip_, h.proto, h.port}) || n.ports.count(h)) {
      return false;
    }
  }
  return true;
}

const Assignment* Engine::assignment(uint64_t pod) const {
  const int32_t si = ledger_.find(pod);
  return si < 0 ? nullptr : &slab_[si];
}

// ============================================================== ledger
bool U64Map::insert(uint64_t k, int32_t v) {
  if ((size_ + 1) * 10 > cap_ * 7) grow();
  for (size_t i = slot(k);; i = (i + 1) & (cap_ - 1)) {
    if (!used_[i]) {
      used_[i] = 1;
      keys_[i] = k;
      vals_[i] = v;
      ++size_;
      return true;
    }
    if (keys_[i] == k) return false;
  }
}

bool U64Map::erase(uint64_t k) {
  if (cap_ == 0) return false;
  size_t i = slot(k);
  for (;; i = (i + 1) & (cap_ - 1)) {
    if (!used_[i]) return false;
    if (keys_[i] == k) break;
  }
  // backward-shift deletion: move later members of the probe run into the hole when their home
  // slot does not lie (cyclically) after it, so lookups never need tombstones
  for (size_t j = (i + 1) & (cap_ - 1);; j = (j + 1) & (cap_ - 1)) {
    if (!used_[j]) break;
    const size_t h = slot(keys_[j]);
    const bool between = i <= j ? (i < h && h <= j) : (i < h || h <= j);
    if (between) continue;
    keys_[i] = keys_[j];
    vals_[i] = vals_[j];
    i = j;
  }
  used_[i] = 0;
  --size_;
  return true;
}

void U64Map::grow() {
  std::vector<uint64_t> k;
  std::vector<int32_t> v;
  std::vector<uint8_t> u;
  k.swap(keys_);
  v.swap(vals_);
  u.swap(used_);
  const size_t old = cap_;
  cap_ = cap_ ? cap_ * 2 : 64;
  keys_.assign(cap_, 0);
  vals_.assign(cap_, 0);
  used_.assign(cap_, 0);
  size_ = 0;
  for (size_t i = 0; i < old; ++i)
    if (u[i]) insert(k[i], v[i]);
}

uint64_t labset_hash(int32_t ns, const Labels& l) {
  uint64_t h = (uint64_t)(uint32_t)ns * 0x9E3779B97F4A7C15ull;
  for (const auto& kv : l) {
    h ^= ((uint64_t)(uint32_t)kv.first << 32 | (uint32_t)kv.second) + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdull;
  }
  return h ^ (h >> 33);
}

int32_t Engine::labset_acquire(int32_t ns, const Labels& labels) {
  const uint64_t h = labset_hash(ns, labels);
  auto it = labset_by_hash_.find(h);
  if (it != labset_by_hash_.end())
    for (int32_t id = it->second; id >= 0; id = labsets_[id].next) {
      LabSetRec& r = labsets_[id];
      if (r.ns == ns && r.labels == labels) {
        if (r.refs++ == 0) --labset_idle_;
        return id;
      }
    }
  int32_t id;
  if (!labset_free_.empty()) {
    id = labset_free_.back();
    labset_free_.pop_back();
  } else {
    id = (int32_t)labsets_.size();
    labsets_.emplace_back();
  }
  LabSetRec& r = labsets_[id];
  r.ns = ns;
  r.labels = labels;
  r.hash = h;
  r.refs = 1;
  r.used = true;
  if (it != labset_by_hash_.end()) {
    r.next = it->second;
    it->second = id;
  } else {
    r.next = -1;
    labset_by_hash_.emplace(h, id);
  }
  return id;
}

void Engine::labset_release(int32_t id) {
  if (id < 0 || id >= (int32_t)labsets_.size()) return;
  LabSetRec& r = labsets_[id];
  if (r.refs <= 0 || --r.refs > 0) return;
  // idle: kept (the next pod of the template finds it without allocating) until idle sets
  // outnumber held ones
  if (++labset_idle_ > 1024 && labset_idle_ * 2 > (int64_t)labsets_used()) labset_sweep();
}

void Engine::labset_sweep() {
  // node groups of an idle set hold count 0 (a set's refs are its ledger entries), so recycling
  // its id leaves them correct: a zero-count group matches nothing, and a later set with the id
  // counts from 0
  for (int32_t id = 0; id < (int32_t)labsets_.size(); ++id) {
    LabSetRec& r = labsets_[id];
    if (!r.used || r.refs > 0) continue;
    auto it = labset_by_hash_.find(r.hash);
    if (it != labset_by_hash_.end()) {
      if (it->second == id) {
        if (r.next >= 0) it->second = r.next;
        else labset_by_hash_.erase(it);
      } else {
        for (int32_t p = it->second; p >= 0; p = labsets_[p].next)
          if (labsets_[p].next == id) {
            labsets_[p].next = r.next;
            break;
          }
      }
    }
    r.used = false;
    r.next = -1;
    Labels().swap(r.labels);
    labset_free_.push_back(id);
  }
  labset_idle_ = 0;
}

bool Engine::reserve(uint64_t pod, const PodReq& req, int32_t idx, const std::vector<int32_t>& cards) {
  if (ledger_.find(pod) >= 0) return false;
  if (idx < 0 || idx >= (int32_t)nodes_.size() || !nodes_[idx].alive) return false;
  Node& n = nodes_[idx];
  for (int32_t c : cards) {
    if (c < 0 || c >= (int32_t)n.cards.size()) return false;
  }
  // a free slab entry keeps its vectors' capacity: a pod like one released before allocates nothing
  int32_t si;
  if (!slab_free_.empty()) {
    si = slab_free_.back();
    slab_free_.pop_back();
  } else {
    si = (int32_t)slab_.size();
    slab_.emplace_back();
  }
  Assignment& a = slab_[si];
  a.pod = pod;
  a.live = true;
  a.node = idx;
  a.mb = req.has_memory ? req.memory : 0;
  a.cards.assign(cards.begin(), cards.end());
  a.t_res = now();
  a.cpu_m = req.cpu_m;
  a.mem = req.mem;
  a.nz_cpu_m = req.nz_cpu_m;
  a.nz_mem = req.nz_mem;
  a.has_label_mem = req.has_memory;
  a.label_mem = req.memory;
  a.prio = req.pod_priority;
  a.ns = req.ns;
  a.labset = labset_acquire(req.ns, req.labels);
  a.deleting = req.deleting;
  a.aff.reset();
  a.aff_hash = 0;
  if (req.aff && !req.aff->empty()) a.aff = req.aff;
  a.pvc_claims.assign(req.pvc_claims.begin(), req.pvc_claims.end());
  a.host_ports.assign(req.host_ports.begin(), req.host_ports.end());
  a.ext.assign(req.ext.begin(), req.ext.end());
  attach(si);
  ledger_.insert(pod, si);
  return true;
}

// A ledger entry's effect on its node (card reservations, requests, label index and groups,
// ports, claims, extended resources) and on the cluster-wide affinity sets. reserve / release
// attach / detach once; a preemption what-if detaches a node's victims and re-attaches them.
void Engine::attach(int32_t si) {
  Assignment& a = slab_[si];
  Node& n = nodes_[a.node];
  if (!compat_) {
    const bool pend = is_pending(n, a);
    for (int32_t c : a.cards) {
      n.cards[c].reserved_mb += a.mb;
      if (pend) n.cards[c].pending_mb += a.mb;
      n.cards[c].pods += 1;
    }
  }
  a.slot = (int32_t)n.pods.size();
  n.pods.push_back(si);
  n.req_cpu_m += a.cpu_m;
  n.req_mem += a.mem;
  n.nz_cpu_m += a.nz_cpu_m;
  n.nz_mem += a.nz_mem;
  n.pod_count += 1;
  if (a.has_label_mem) n.label_mem_sum += a.label_mem;
  if (a.aff) {
    aff_holders_.insert(a.pod);
    if (!a.aff->req_anti.empty()) anti_holders_.insert(a.pod);
    aff_set_add(a);
  }
  index_pod(n, a, +1);
  for (int32_t c : a.pvc_claims) ++n.claims[c];
  for (const HostPort& h : a.host_ports) {
    ++n.ports[h];
    ++n.ports_any[{h.proto, h.port}];
  }
  for (const auto& r : a.ext) {
    auto it = std::lower_bound(n.ext_used.begin(), n.ext_used.end(), std::make_pair(r.first, INT64_MIN));
    if (it != n.ext_used.end() && it->first == r.first) it->second += r.second;
    else n.ext_used.insert(it, r);
  }
  mark_dirty(a.node);
}

void Engine::detach(int32_t si) {
  Assignment& a = slab_[si];
  if (a.node >= 0 && a.node < (int32_t)nodes_.size() && nodes_[a.node].alive) {
    Node& n = nodes_[a.node];
    if (!compat_) {
      const bool pend = is_pending(n, a);
      for (int32_t c : a.cards) {
        if (c < (int32_t)n.cards.size()) {
          n.cards[c].reserved_mb -= std::min(n.cards[c].reserved_mb, a.mb);
          if (pend) n.cards[c].pending_mb -= std::min(n.cards[c].pending_mb, a.mb);
          n.cards[c].pods = std::max(0, n.cards[c].pods - 1);
        }
      }
    }
    if (a.slot >= 0 && a.slot < (int32_t)n.pods.size()) {
      const int32_t last = n.pods.back();
      n.pods[a.slot] = last;
      n.pods.pop_back();
      if (last != si) slab_[last].slot = a.slot;
    }
    a.slot = -1;
    n.req_cpu_m -= a.cpu_m;
    n.req_mem -= a.mem;
    n.nz_cpu_m -= a.nz_cpu_m;
    n.nz_mem -= a.nz_mem;
    n.pod_count -= 1;
    if (a.has_label_mem) n.label_mem_sum -= a.label_mem;
    for (const auto& r : a.ext) {
      auto it = std::lower_bound(n.ext_used.begin(), n.ext_used.end(), std::make_pair(r.first, INT64_MIN));
      if (it != n.ext_used.end() && it->first == r.first && (it->second -= r.second) == 0) n.ext_used.erase(it);
    }
    index_pod(n, a, -1);
    for (int32_t c : a.pvc_claims) {
      auto q = n.claims.find(c);
      if (q != n.claims.end() && --q->second <= 0) n.claims.erase(q);
    }
    for (const HostPort& h : a.host_ports) {
      auto p = n.ports.find(h);
      if (p != n.ports.end() && --p->second <= 0) n.ports.erase(p);
      auto q = n.ports_any.find({h.proto, h.port});
      if (q != n.ports_any.end() && --q->second <= 0) n.ports_any.erase(q);
    }
    mark_dirty(a.node);
  }
  if (a.aff) {
    aff_holders_.erase(a.pod);
    anti_holders_.erase(a.pod);
    aff_set_remove(a);
  }
}

void Engine::free_entry(int32_t si) {
  Assignment& a = slab_[si];
  ledger_.erase(a.pod);
  labset_release(a.labset);
  a.labset = -1;
  a.live = false;
  a.detached = false;
  a.node = -1;
  a.slot = -1;
  a.aff.reset();
  a.cards.clear();
  a.ext.clear();
  a.host_ports.clear();
  a.pvc_claims.clear();
  slab_free_.push_back(si);
}

bool Engine::release(uint64_t pod) {
  const int32_t si = ledger_.find(pod);
  if (si < 0) return false;
  if (!slab_[si].detached) detach(si);
  free_entry(si);
  return true;
}

// ============================================================== DefaultPreemption
static bool tolerates(const Toleration& t, const Taint& x);

bool Engine::preemption_might_help(const PodReq& req, int32_t idx) const {
  // upstream v1.20 default filter order with each plugin's failure code: Unschedulable and
  // Unresolvable for NodeUnschedulable, NodeName, NodeAffinity, TaintToleration, VolumeBinding,
  // VolumeZone, a missing spread topology key and unmet required pod affinity; Unschedulable
  // (preemption may help) for the rest. yoda (out-of-tree, after the defaults) says Unschedulable
  // — except for a node without a fresh Scv sample, which no eviction can fix (skipped here).
  const Node& n = nodes_[idx];
  if (!n.alive) return false;
  if ((filters_ & F_NODE_UNSCHEDULABLE) && n.unschedulable) {
    bool tol = false;
    Taint t{unsched_key_, 0, kNoSchedule};
    for (const Toleration& x : req.tolerations)
      if (tolerates(x, t)) { tol = true; break; }
    if (!tol) return false;
  }
  if (filters_ & F_NODE_RESOURCES_FIT) {
    if (n.pod_count + 1 > n.alloc_pods) return true;
    if (req.cpu_m > 0 && n.alloc_cpu_m < req.cpu_m + n.req_cpu_m) return true;
    if (req.mem > 0 && n.alloc_mem < req.mem + n.req_mem) return true;
    for (const auto& r : req.ext)
      if (ext_checked(r.first) && ext_amount(n.ext_used, r.first) + r.second > ext_amount(n.ext_alloc, r.first))
        return true;
  }
  if ((filters_ & F_NODE_NAME) && req.node_name > 0 && strings_[req.node_name] != n.name) return false;
  if ((filters_ & F_NODE_PORTS) && !req.host_ports.empty() && !ports_free(req, n)) return true;
  if ((filters_ & F_NODE_AFFINITY) && !affinity_ok(req, n)) return false;
  if ((filters_ & F_TAINT_TOLERATION) && !taints_ok(req, n)) return false;
  if (req.count_vols && !req.pvc_claims.empty() && !n.vol_limits.empty() && !vols_fit(req, n)) return true;
  for (const PodReq::VolTerms& v : req.vol) {
    bool ok = false;
    for (const SelTerm& t : *v.terms)
      if (term_matches(t, n)) { ok = true; break; }
    if (!ok) return false;
  }
  return true;   // PodTopologySpread, InterPodAffinity and yoda: preempt_status goes on
}

bool Engine::detach_pod(uint64_t pod) {
  const int32_t si = ledger_.find(pod);
  if (si < 0 || slab_[si].detached) return false;
  detach(si);
  slab_[si].detached = true;
  return true;
}

bool Engine::attach_pod(uint64_t pod) {
  const int32_t si = ledger_.find(pod);
  if (si < 0 || !slab_[si].detached) return false;
  const Assignment& a = slab_[si];
  if (a.node < 0 || a.node >= (int32_t)nodes_.size() || !nodes_[a.node].alive) return false;
  slab_[si].detached = false;
  attach(si);
  return true;
}

int Engine::preempt_status(const PodReq& req, int32_t idx, const SpreadPF* spf, const InterPodPF* ipf) const {
  // -1: the first failing filter (upstream order) is Unschedulable and Unresolvable; +1: it is
  // not (or every filter passes)
  if (!preemption_might_help(req, idx)) return -1;
  const Node& n = nodes_[idx];
  // the early-decided resolvable failures (NodeResourcesFit, NodePorts, NodeVolumeLimits) come
  // before the checks below in upstream order: preemption_might_help returned true for them
  // too, so the checks below apply only when those pass
  const bool early = ((filters_ & F_NODE_RESOURCES_FIT) && [&] {
                       if (n.pod_count + 1 > n.alloc_pods) return true;
                       if (req.cpu_m > 0 && n.alloc_cpu_m < req.cpu_m + n.req_cpu_m) return true;
                       if (req.mem > 0 && n.alloc_mem < req.mem + n.req_mem) return true;
                       for (const auto& r : req.ext)
                         if (ext_checked(r.first) &&
                             ext_amount(n.ext_used, r.first) + r.second > ext_amount(n.ext_alloc, r.first))
                           return true;
                       return false;
                     }()) ||
                     ((filters_ & F_NODE_PORTS) && !req.host_ports.empty() && !ports_free(req, n)) ||
                     (req.count_vols && !req.pvc_claims.empty() && !n.vol_limits.empty() && !vols_fit(req, n));
  if (early) return 1;
  if (spf && !spf->cons.empty()) {
    const Reason r = spread_filter(req, n, *spf);
    if (r == RS_SPREAD_LABEL) return -1;
    if (r != RS_OK) return 1;
  }
  if (ipf && ipf->active) {
    const Reason r = interpod_filter(req, n, *ipf);
    if (r == RS_POD_AFFINITY) return -1;
    if (r != RS_OK) return 1;
  }
  // yoda: Unschedulable in the reference, but no eviction gives a node a fresh Scv sample
  if ((filters_ & F_YODA) && (!n.has_scv || (!compat_ && n.stale))) return -1;
  return 1;
}

bool Engine::preempt(const PodReq& req, const PreemptArgs& args, PreemptResult* out) {
  *out = PreemptResult();
  const std::vector<int32_t> potential = preempt_potential(req);   // nodesWherePreemptionMightHelp
  out->potential = (int32_t)potential.size();
  if (potential.empty()) return false;
  return preempt_over(req, args, potential, out);
}

std::vector<int32_t> Engine::preempt_potential(const PodReq& req) const {
  SpreadPF spf;
  InterPodPF ipf;
  const bool sp = wants_spread_filter(req), ia = wants_interpod_filter(req);
  if (sp) spread_prefilter(req, &spf);
  if (ia) interpod_prefilter(req, &ipf);
  std::vector<int32_t> potential;
  for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i)
    if (preempt_status(req, i, sp ? &spf : nullptr, ia ? &ipf : nullptr) > 0) potential.push_back(i);
  return potential;
}

bool Engine::preempt_over(const PodReq& req, const PreemptArgs& args, const std::vector<int32_t>& potential,
                          PreemptResult* out) {
  const bool sp = wants_spread_filter(req), ia = wants_interpod_filter(req);
  if (potential.empty()) return false;
  // calculateNumCandidates and a random offset (dryRunPreemption walks from it, wrapping)
  const int32_t np = (int32_t)potential.size();
  int32_t want = (int32_t)((int64_t)np * args.min_pct / 100);
  want = std::min(std::max(want, args.min_abs), np);
  const int32_t offset = args.offset >= 0 ? (int32_t)(args.offset % np) : (int32_t)(rng_() % (uint64_t)np);
  // a what-if filter: the pre-filter states follow the detached / re-attached pods as upstream's
  // RunPreFilterExtensionRemovePod / AddPod do (recomputed: only for spread / affinity pods)
  auto fits = [&](int32_t idx) {
    if (sp || ia) return filter_node(req, idx, nullptr, nullptr, nullptr) == RS_OK;
    return filter_node_pf(req, idx, nullptr, nullptr, nullptr, nullptr, nullptr) == RS_OK;
  };
  struct Cand {
    int32_t node;
    std::vector<int32_t> victims;   // slab indices, in eviction-decision order
    int32_t violations;
  };
  std::vector<Cand> nonviol, viol;
  std::vector<int32_t> lower;
  std::vector<std::pair<int32_t, bool>> order;
  std::vector<int64_t> budget;
  for (int32_t k = 0; k < np; ++k) {
    const int32_t idx = potential[(offset + k) % np];
    ++out->evaluated;
    Node& n = nodes_[idx];
    lower.clear();
    for (int32_t si : n.pods)
      if (slab_[si].prio < args.priority) lower.push_back(si);
    if (!lower.empty()) {
      for (int32_t si : lower) detach(si);
      if (!fits(idx)) {
        for (auto it = lower.rbegin(); it != lower.rend(); ++it) attach(*it);
      } else {
        // MoreImportantPod: higher priority first, then the earlier start (reservation)
        std::sort(lower.begin(), lower.end(), [&](int32_t x, int32_t y) {
          const Assignment &a = slab_[x], &b = slab_[y];
          return a.prio != b.prio ? a.prio > b.prio : a.t_res != b.t_res ? a.t_res < b.t_res : a.pod < b.pod;
        });
        // filterPodsWithPDBViolation: budgets consumed in that order
        budget.assign(args.pdbs.size(), 0);
        for (size_t q = 0; q < args.pdbs.size(); ++q) budget[q] = args.pdbs[q].allowed;
        order.clear();
        for (int32_t si : lower) {
          const Assignment& a = slab_[si];
          bool bad = false;
          for (size_t q = 0; q < args.pdbs.size(); ++q) {
            const Pdb& d = args.pdbs[q];
            if (d.ns != a.ns || d.sel.nothing || d.sel.reqs.empty() || !d.sel.matches(labsets_[a.labset].labels))
              continue;
            if (--budget[q] < 0) bad = true;
          }
          order.emplace_back(si, bad);
        }
        std::stable_partition(order.begin(), order.end(), [](const std::pair<int32_t, bool>& x) { return x.second; });
        Cand c{idx, {}, 0};
        for (const auto& o : order) {   // reprieve: PDB-violating victims first, then the others
          attach(o.first);
          if (!fits(idx)) {
            detach(o.first);
            c.victims.push_back(o.first);
            c.violations += o.second;
          }
        }
        for (int32_t si : c.victims) attach(si);   // restore the node
        if (!c.victims.empty()) (c.violations ? viol : nonviol).push_back(std::move(c));
      }
    }
    if (!nonviol.empty() && (int32_t)(nonviol.size() + viol.size()) >= want) break;
  }
  out->candidates = (int32_t)(nonviol.size() + viol.size());
  if (!out->candidates) return false;
  // pickOneNodeForPreemption over non-violating then violating candidates
  std::vector<Cand*> all;
  for (auto& c : nonviol) all.push_back(&c);
  for (auto& c : viol) all.push_back(&c);
  struct Key {
    int32_t violations;
    int64_t top;          // highest victim priority
    __int128 sum;         // Σ (priority + MaxInt32 + 1)
    size_t count;
    double earliest;      // earliest start among the highest-priority victims (later wins)
  };
  auto key_of = [&](const Cand& c) {
    Key k{c.violations, INT64_MIN, 0, c.victims.size(), 0};
    for (int32_t si : c.victims) {
      k.top = std::max(k.top, slab_[si].prio);
      k.sum += (__int128)slab_[si].prio + ((__int128)1 << 31);
    }
    k.earliest = 1e300;
    for (int32_t si : c.victims)
      if (slab_[si].prio == k.top) k.earliest = std::min(k.earliest, slab_[si].t_res);
    return k;
  };
  Cand* best = all[0];
  Key bk = key_of(*best);
  for (size_t i = 1; i < all.size(); ++i) {
    const Key k = key_of(*all[i]);
    bool better;
    if (k.violations != bk.violations) better = k.violations < bk.violations;
    else if (k.top != bk.top) better = k.top < bk.top;
    else if (k.sum != bk.sum) better = k.sum < bk.sum;
    else if (k.count != bk.count) better = k.count < bk.count;
    else better = k.earliest > bk.earliest;
    if (better) {
      best = all[i];
      bk = k;
    }
  }
  out->node = best->node;
  out->violations = best->violations;
  for (int32_t si : best->victims) out->victims.push_back(slab_[si].pod);
  // the GPUs the preemptor would take on the nominated node once the victims are gone
  for (int32_t si : best->victims) detach(si);
  int32_t q = 10000;
  if (filters_ & F_YODA) select_gpus(req, best->node, &out->cards, &q);
  for (auto it = best->victims.rbegin(); it != best->victims.rend(); ++it) attach(*it);
  return true;
}

// ============================================================== default filters
static bool tolerates(const Toleration& t, const Taint& x) {
  if (t.effect != kEffectAny && t.effect != x.effect) return false;
  if (t.key >= 0 && t.key != x.key) return false;
  if (t.key < 0 && t.op != kTolExists) return false;   // empty key requires Exists
  if (t.op == kTolExists) return true;
  return t.value == x.value;
}

bool Engine::taints_ok(const PodReq& req, const Node& n) const {
  for (const Taint& x : n.taints) {
    if (x.effect == kPreferNoSchedule) continue;
    bool ok = false;
    for (const Toleration& t : req.tolerations)
      if (tolerates(t, x)) { ok = true; break; }
    if (!ok) return false;
  }
  return true;
}

bool Engine::term_matches(const SelTerm& t, const Node& n) const {
  if (t.reqs.empty()) return false;   // empty term matches no objects (upstream)
  for (const SelReq& r : t.reqs) {
    const std::string& key = strings_[r.key];
    if (!key.empty() && key[0] == '@') {
      // matchFields (upstream v1.20 NodeSelectorRequirementsAsFieldSelector): In / NotIn with
      // exactly one value, anything else is an error that fails the term; the node's fields
      // are {metadata.name}, so any other field reads as ""
      if ((r.op != kIn && r.op != kNotIn) || r.values.size() != 1) return false;
      const bool eq = strings_[r.values[0]] == (r.key == field_name_key_ ? n.name : std::string());
      if (r.op == kIn ? !eq : eq) return false;
      continue;
    }
    auto it = n.labels.find(r.key);
    bool has = it != n.labels.end();
    switch (r.op) {
      case kIn:
        if (!has || std::find(r.values.begin(), r.values.end(), it->second) == r.values.end()) return false;
        break;
      case kNotIn:
        if (has && std::find(r.values.begin(), r.values.end(), it->second) != r.values.end()) return false;
        break;
      case kExists:
        if (!has) return false;
        break;
      case kDoesNotExist:
        if (has) return false;
        break;
      case kGt:
      case kLt: {
        if (!has) return false;
        const std::string& s = strings_[it->second];
        char* end = nullptr;
        long long v = std::strtoll(s.c_str(), &end, 10);
        if (s.empty() || std::isspace((unsigned char)s[0]) || *end != '\0') return false;   // ParseInt syntax
        if (r.op == kGt ? !(v > r.num) : !(v < r.num)) return false;
        break;
      }
    }
  }
  return true;
}

bool Engine::affinity_ok(const PodReq& req, const Node& n) const {
  for (auto& kv : req.node_selector) {
    auto it = n.labels.find(kv.first);
    if (it == n.labels.end() || it->second != kv.second) return false;
  }
  if (req.required_terms.empty()) return true;
  for (const SelTerm& t : req.required_terms)
    if (term_matches(t, n)) return true;
  return false;
}

// ============================================================== yoda policy
uint64_t Engine::eff_free(const Card& c) const {
  // Sampled free HBM minus reservations the sample cannot contain yet, capped by the
  // ledger view (total − all reservations, for pods that have not allocated yet).
  if (compat_) return c.free_mb;
  uint64_t cap = c.total_mb > c.reserved_mb ? c.total_mb - c.reserved_mb : 0;
  uint64_t sampled = c.free_mb > c.pending_mb ? c.free_mb - c.pending_mb : 0;
  return std::min(sampled, cap);
}

bool Engine::yoda_card_eligible(const PodReq& req, const Card& c, uint64_t m, uint64_t cl) const {
  if (!c.healthy) return false;
  if (eff_free(c) < m) return false;
  if (req.has_clock && c.clock != cl) return false;
  if (req.clock_min && c.clock < req.clock_min) return false;
  return true;
}

Reason Engine::filter_node(const PodReq& req, int32_t idx, uint64_t* pn, uint64_t* pm, uint64_t* pc) const {
  SpreadPF pf;
  InterPodPF ip;
  const bool sp = wants_spread_filter(req), ia = wants_interpod_filter(req);
  if (sp) spread_prefilter(req, &pf);
  if (ia) interpod_prefilter(req, &ip);
  return filter_node_pf(req, idx, pn, pm, pc, sp ? &pf : nullptr, ia ? &ip : nullptr);
}

Reason Engine::filter_node_pf(const PodReq& req, int32_t idx, uint64_t* pn, uint64_t* pm, uint64_t* pc,
                              const SpreadPF* pf, const InterPodPF* ip) const {
  const Node& n = nodes_[idx];
  if (!n.alive) return RS_DEAD;
  if (filters_ & F_NODE_UNSCHEDULABLE) {
    if (n.unschedulable) {
      // tolerated only by node.kubernetes.io/unschedulable:NoSchedule
      bool tol = false;
      Taint t{unsched_key_, 0, kNoSchedule};
      for (const Toleration& x : req.tolerations)
        if (tolerates(x, t)) { tol = true; break; }
      if (!tol) return RS_UNSCHEDULABLE;
    }
  }
  if (filters_ & F_NODE_RESOURCES_FIT) {
    if (n.pod_count + 1 > n.alloc_pods) return RS_RESOURCES;
    if (req.cpu_m > 0 && n.alloc_cpu_m < req.cpu_m + n.req_cpu_m) return RS_RESOURCES;
    if (req.mem > 0 && n.alloc_mem < req.mem + n.req_mem) return RS_RESOURCES;
    // resources beyond cpu/memory/pods (plugins/defaults.py NodeResourcesFit): requested +
    // already used must fit the node's allocatable (absent = 0)
    for (const auto& r : req.ext) {
      if (!ext_checked(r.first)) continue;
      int64_t alloc = 0, used = 0;
      auto a = std::lower_bound(n.ext_alloc.begin(), n.ext_alloc.end(), std::make_pair(r.first, INT64_MIN));
      if (a != n.ext_alloc.end() && a->first == r.first) alloc = a->second;
      auto u = std::lower_bound(n.ext_used.begin(), n.ext_used.end(), std::make_pair(r.first, INT64_MIN));
      if (u != n.ext_used.end() && u->first == r.first) used = u->second;
      if (used + r.second > alloc) return RS_EXT_RESOURCES;
    }
  }
  if ((filters_ & F_NODE_NAME) && req.node_name > 0 && strings_[req.node_name] != n.name) return RS_NODE_NAME;
  // upstream v1.20 default filter order: NodeName, NodePorts, NodeAffinity, ..., TaintToleration
  if ((filters_ & F_NODE_PORTS) && !req.host_ports.empty() && !ports_free(req, n)) return RS_NODE_PORTS;
  if ((filters_ & F_NODE_AFFINITY) && !affinity_ok(req, n)) return RS_AFFINITY;
  if ((filters_ & F_TAINT_TOLERATION) && !taints_ok(req, n)) return RS_TAINT;
  if (filters_ & F_YODA) {
    const Reason r = yoda_filter(req, idx, pn, pm, pc);
    if (r != RS_OK) return r;
  }
  // PodTopologySpread runs after the built-in filters (a Python filter in the hybrid runner,
  // where every native filter comes first): same first-failing reason on both paths
  if (pf && !pf->cons.empty()) {
    const Reason r = spread_filter(req, n, *pf);
    if (r != RS_OK) return r;
  }
  if (ip && ip->active) {
    const Reason r = interpod_filter(req, n, *ip);
    if (r != RS_OK) return r;
  }
  // the volume plugins run after every other filter (where the hybrid runner's Python filters
  // run: same first-failing reason on both paths): NodeVolumeLimits, then VolumeBinding and
  // VolumeZone — a PV's NodeSelector: any term matches; a term with no requirement matches nothing
  if (req.count_vols && !req.pvc_claims.empty() && !n.vol_limits.empty() && !vols_fit(req, n)) return RS_VOLUME_LIMITS;
  for (const PodReq::VolTerms& v : req.vol) {
    bool ok = false;
    for (const SelTerm& t : *v.terms)
      if (term_matches(t, n)) {
        ok = true;
        break;
      }
    if (!ok) return (Reason)v.reason;
  }
  return RS_OK;
}

bool Engine::ext_checked(int32_t res) const {
  if (ext_ignored_.empty() && ext_ignored_groups_.empty()) return true;
  if (std::find(ext_ignored_.begin(), ext_ignored_.end(), res) != ext_ignored_.end()) return false;
  if (ext_ignored_groups_.empty()) return true;
  const std::string& name = strings_[res];
  const std::string group = name.substr(0, name.find('/'));
  return std::find(ext_ignored_groups_.begin(), ext_ignored_groups_.end(), group) == ext_ignored_groups_.end();
}

Reason Engine::yoda_filter(const PodReq& req, int32_t idx, uint64_t* pn, uint64_t* pm, uint64_t* pc) const {
  // (*Yoda).Filter: scheduler.go:76-93
  const Node& n = nodes_[idx];
  if (!n.has_scv) return RS_NO_SCV;
  uint64_t num = req.has_number ? req.number : 1;
  uint64_t m = req.has_memory ? req.memory : 0;
  uint64_t cl = req.has_clock ? req.clock : 0;
  if (pn) *pn = num;
  if (pm) *pm = m;
  if (pc) *pc = cl;
  // PodFitsNumber (filter.go:11-16)
  if (req.has_number ? !(req.number <= n.card_number) : !(n.card_number > 0)) return RS_GPU_NUMBER;
  if (compat_) {
    if (req.has_memory) {
      uint64_t cnt = 0;
      for (const Card& c : n.cards)
        if (c.healthy && c.free_mb >= m) ++cnt;
      if (cnt < num) return RS_GPU_MEMORY;
    }
    if (req.has_clock) {
      uint64_t cnt = 0;
      for (const Card& c : n.cards)
        if (c.healthy && c.clock == cl) ++cnt;
      if (cnt < num) return RS_GPU_CLOCK;
    }
    return RS_OK;
  }
  if (n.stale) return RS_STALE;
  uint64_t cnt = 0;
  for (const Card& c : n.cards)
    if (yoda_card_eligible(req, c, m, cl)) ++cnt;
  return cnt >= num ? RS_OK : RS_GPU_FIT;
}

FilterView Engine::filter_view(int32_t idx) const {
  // exactly what yoda_filter / yoda_card_eligible read of a node, so the Scv queueing hint
  // (framework/scheduler.py::_capacity) cannot drift from the filter: keep the two together
  FilterView v;
  if (idx < 0 || idx >= (int32_t)nodes_.size() || !nodes_[idx].alive) return v;
  const Node& n = nodes_[idx];
  v.known = true;
  v.has_scv = n.has_scv;
  v.stale = n.stale;
  v.card_number = n.card_number;
  for (const Card& c : n.cards) v.cards.push_back({c.healthy, c.free_mb, eff_free(c), c.clock});
  return v;
}

void Engine::collect_max(const PodReq& req, const std::vector<int32_t>& idxs, uint64_t mx[6]) const {
  // order: bandwidth, clock, core, free, power, total; all seeded 1 (collection.go:31-38)
  for (int i = 0; i < 6; ++i) mx[i] = 1;
  for (int32_t idx : idxs) {
    uint64_t num, m, cl;
    if (!nodes_[idx].alive || !nodes_[idx].has_scv) continue;
    if (yoda_filter(req, idx, &num, &m, &cl) != RS_OK) continue;
    for (const Card& c : nodes_[idx].cards) {
      bool take = compat_ ? (c.free_mb >= m && c.clock >= cl) : yoda_card_eligible(req, c, m, cl);
      if (!take) continue;
      uint64_t f = eff_free(c);
      mx[0] = std::max(mx[0], c.bandwidth);
      mx[1] = std::max(mx[1], c.clock);
      mx[2] = std::max(mx[2], c.core);
      mx[3] = std::max(mx[3], f);
      mx[4] = std::max(mx[4], c.power);
      mx[5] = std::max(mx[5], c.total_mb);
    }
  }
}

uint64_t Engine::yoda_raw_score(const PodReq& req, int32_t idx, const uint64_t mx[6]) const {
  const Node& n = nodes_[idx];
  uint64_t num, m, cl;
  uint64_t basic = 0;
  if (yoda_filter(req, idx, &num, &m, &cl) == RS_OK) {
    for (const Card& c : n.cards) {
      bool take = compat_ ? (c.free_mb >= m && c.clock >= cl) : yoda_card_eligible(req, c, m, cl);
      if (!take) continue;
      uint64_t f = eff_free(c);
      uint64_t bw = c.bandwidth * 100 / mx[0];
      uint64_t clk = c.clock * 100 / (compat_ ? mx[0] : mx[1]);   // Q2: algorithm.go:60
      uint64_t core = c.core * 100 / mx[2];
      uint64_t pw = c.power * 100 / mx[4];
      uint64_t fm = f * 100 / mx[3];
      uint64_t tm = c.total_mb * 100 / mx[5];
      basic += (bw + clk + core + pw) + fm * 2 + tm * 1;
    }
  }
  uint64_t total, free, alloc;
  if (compat_) {
    total = n.total_sum;
    free = n.free_sum;
    alloc = n.label_mem_sum;
  } else {
    total = free = alloc = 0;
    for (const Card& c : n.cards) {
      total += c.total_mb;
      free += eff_free(c);
      alloc += c.reserved_mb;
    }
  }
  uint64_t actual = total ? (free * 100 / total) * 2 : 0;                        // Q4 guard
  uint64_t allocate = (total == 0 || total < alloc) ? 0 : (total - alloc) * 100 / total * 3;
  uint64_t s = basic + allocate + actual;
  if (!compat_ && req.has_number && req.number > 1 && req.number <= n.cards.size()) {
    std::vector<int32_t> sel;
    int32_t q = 0;
    if (select_gpus(req, idx, &sel, &q)) s += (uint64_t)(q / 100) * (uint64_t)wt_.w_gang_score;
  }
  return s > (uint64_t)INT64_MAX ? 0 : s;   // filter.Uint64ToInt64 (filter.go:84)
}

void Engine::normalize_yoda(std::vector<int64_t>& s) {
  if (s.empty()) return;
  int64_t highest = 0, lowest = s[0];
  for (int64_t v : s) {
    lowest = std::min(lowest, v);
    highest = std::max(highest, v);
  }
  if (highest == lowest) --lowest;
  int64_t den = (int64_t)((uint64_t)highest - (uint64_t)lowest);
  for (auto& v : s) {
    int64_t num = (int64_t)(((uint64_t)v - (uint64_t)lowest) * (uint64_t)kMaxNodeScore);
    v = num / den;
  }
}

// ============================================================== gang selection
int64_t Engine::gang_objective(const Node& n, const std::vector<int32_t>& set, uint64_t m,
                               int64_t* link_bad_out) const {
  const int64_t k = (int64_t)set.size();
  int64_t P = k * (k - 1) / 2;
  int64_t qsum = 0, qmin = 10000;
  uint64_t numa_mask = 0;
  int64_t free_after = 0, total = 0, occ = 0;
  for (int64_t a = 0; a < k; ++a) {
    const Card& ca = n.cards[set[a]];
    numa_mask |= 1ull << (ca.numa & 63);
    free_after += (int64_t)(eff_free(ca) - m);
    total += (int64_t)ca.total_mb;
    occ += ca.occ_q;
    for (int64_t b = a + 1; b < k; ++b) {
      const Card& cb = n.cards[set[b]];
      int32_t q = 10000;
      if (ca.phys != cb.phys && ca.phys < n.nphys && cb.phys < n.nphys)
        q = n.link_q[(size_t)ca.phys * n.nphys + cb.phys];
      qsum += q;
      qmin = q < qmin ? q : qmin;
    }
  }
  int64_t link_bad = P ? (P * 10000 - qsum) * 100 / P : 0;
  int64_t minlink_bad = P ? (10000 - qmin) * 100 : 0;
  int64_t d = __builtin_popcountll(numa_mask);
  int64_t numa_bad = k > 1 ? (d - 1) * 1000000 / (k - 1) : 0;
  int64_t leftover = total ? free_after * 1000000 / total : 0;
  int64_t fit = wt_.gpu_binpack ? leftover : 1000000 - leftover;
  int64_t occ_bad = k ? occ * 100 / k : 0;
  if (link_bad_out) *link_bad_out = link_bad;
  return wt_.w_link * link_bad + wt_.w_minlink * minlink_bad + wt_.w_numa * numa_bad + wt_.w_fit * fit +
         wt_.w_occ * occ_bad;
}

static uint64_t n_choose_k(uint64_t n, uint64_t k, uint64_t cap) {
  if (k > n) return 0;
  k = std::min(k, n - k);
  uint64_t r = 1;
  for (uint64_t i = 1; i <= k; ++i) {
    r = r * (n - k + i) / i;
    if (r > cap) return cap + 1;
  }
  return r;
}

bool Engine::select_gpus(const PodReq& req, int32_t idx, std::vector<int32_t>* out, int32_t* quality) const {
  const Node& n = nodes_[idx];
  out->clear();
  if (quality) *quality = 10000;
  uint64_t k = req.has_number ? req.number : 1;
  uint64_t m = req.has_memory ? req.memory : 0;
  uint64_t cl = req.has_clock ? req.clock : 0;
  if (k == 0) return true;
  thread_local std::vector<int32_t> E;   // reused: no allocation per node per pod
  E.clear();
  out->reserve(k);
  for (int32_t i = 0; i < (int32_t)n.cards.size(); ++i) {
    const Card& c = n.cards[i];
    bool ok = compat_ ? (c.healthy && c.free_mb >= m && (!req.has_clock || c.clock == cl))
                      : yoda_card_eligible(req, c, m, cl);
    if (ok) E.push_back(i);
  }
  if (compat_) {
    // the reference never assigns GPUs; report the first k candidates (informational)
    for (uint64_t i = 0; i < k && i < E.size(); ++i) out->push_back(E[i]);
    return out->size() == k;
  }
  if (E.size() < k) return false;
  if (n.cards.size() <= 16 && n_choose_k(E.size(), k, (uint64_t)wt_.enum_limit) <= (uint64_t)wt_.enum_limit)
    return select_gpus_small(n, E, k, m, out, quality);
  int64_t best = INT64_MAX, best_link = 0, lb = 0;
  std::vector<int32_t> cur;
  uint64_t total = n_choose_k(E.size(), k, (uint64_t)wt_.enum_limit);
  if (total <= (uint64_t)wt_.enum_limit) {
    // exhaustive lexicographic k-subset enumeration
    std::vector<int32_t> pos(k);
    for (uint64_t i = 0; i < k; ++i) pos[i] = (int32_t)i;
    cur.resize(k);
    for (;;) {
      for (uint64_t i = 0; i < k; ++i) cur[i] = E[pos[i]];
      int64_t obj = gang_objective(n, cur, m, &lb);
      if (obj < best) {
        best = obj;
        best_link = lb;
        *out = cur;
      }
      int64_t i = (int64_t)k - 1;
      while (i >= 0 && pos[i] == (int32_t)(E.size() - k + i)) --i;
      if (i < 0) break;
      ++pos[i];
      for (uint64_t j = i + 1; j < k; ++j) pos[j] = pos[j - 1] + 1;
    }
  } else {
    // greedy growth: add the card that minimises the objective of the partial set
    std::vector<char> used(n.cards.size(), 0);
    for (uint64_t step = 0; step < k; ++step) {
      int64_t bo = INT64_MAX;
      int32_t bi = -1;
      for (int32_t e : E) {
        if (used[e]) continue;
        cur.push_back(e);
        int64_t obj = gang_objective(n, cur, m, &lb);
        cur.pop_back();
        if (obj < bo) {
          bo = obj;
          bi = e;
        }
      }
      used[bi] = 1;
      cur.push_back(bi);
    }
    std::sort(cur.begin(), cur.end());
    best = gang_objective(n, cur, m, &best_link);
    *out = cur;
  }
  if (quality) *quality = (int32_t)(10000 - best_link / 100);
  return true;
}

// Exhaustive search for nodes of ≤ 16 cards (every MI355X/MI350X node, partitioned ones up to
// DPX): per-card terms and pair qualities are read once, subsets are bitmasks enumerated in
// Gosper order, and gang_objective's integer arithmetic is applied to them. Ties go to the
// lexicographically smallest set — the one holding the lowest card of the symmetric
// difference — which is the set the lexicographic enumeration above keeps first.
bool Engine::select_gpus_small(const Node& n, const std::vector<int32_t>& E, uint64_t k, uint64_t m,
                               std::vector<int32_t>* out, int32_t* quality) const {
  const int ne = (int)E.size();
  int64_t fa[16], tt[16], oc[16];
  uint64_t nb[16];
  for (int j = 0; j < ne; ++j) {
    const Card& c = n.cards[E[j]];
    fa[j] = (int64_t)(eff_free(c) - m);
    tt[j] = (int64_t)c.total_mb;
    oc[j] = c.occ_q;
    nb[j] = 1ull << (c.numa & 63);
  }
  const int64_t K = (int64_t)k, P = K * (K - 1) / 2;
  int32_t q[16][16];
  bool uniform = true;
  int32_t q0 = -1;
  for (int a = 0; a < ne; ++a)
    for (int b = a + 1; b < ne; ++b) {
      const Card& ca = n.cards[E[a]];
      const Card& cb = n.cards[E[b]];
      int32_t v = 10000;
      if (ca.phys != cb.phys && ca.phys < n.nphys && cb.phys < n.nphys) v = n.link_q[(size_t)ca.phys * n.nphys + cb.phys];
      q[a][b] = v;
      if (q0 < 0) q0 = v;
      uniform = uniform && v == q0;
    }
  int64_t best = INT64_MAX, best_link = 0;
  uint32_t best_set = 0;
  // x: a k-bit subset of the ne eligible positions (Gosper's hack walks them all)
  const uint32_t last = ne >= 32 ? 0u : (1u << ne);
  for (uint32_t x = (1u << K) - 1u; x < last;) {
    int64_t qsum = 0, qmin = 10000, free_after = 0, total = 0, occ = 0;
    uint64_t numa_mask = 0;
    for (uint32_t r = x; r; r &= r - 1) {
      const int a = __builtin_ctz(r);
      numa_mask |= nb[a];
      free_after += fa[a];
      total += tt[a];
      occ += oc[a];
      if (!uniform)
        for (uint32_t r2 = r & (r - 1); r2; r2 &= r2 - 1) {
          const int32_t v = q[a][__builtin_ctz(r2)];
          qsum += v;
          qmin = v < qmin ? v : qmin;
        }
    }
    if (uniform && P) {
      qsum = P * q0;
      qmin = q0 < qmin ? q0 : qmin;
    }
    const int64_t link_bad = P ? (P * 10000 - qsum) * 100 / P : 0;
    const int64_t minlink_bad = P ? (10000 - qmin) * 100 : 0;
    const int64_t d = __builtin_popcountll(numa_mask);
    const int64_t numa_bad = K > 1 ? (d - 1) * 1000000 / (K - 1) : 0;
    const int64_t leftover = total ? free_after * 1000000 / total : 0;
    const int64_t fit = wt_.gpu_binpack ? leftover : 1000000 - leftover;
    const int64_t occ_bad = K ? occ * 100 / K : 0;
    const int64_t obj = wt_.w_link * link_bad + wt_.w_minlink * minlink_bad + wt_.w_numa * numa_bad +
                        wt_.w_fit * fit + wt_.w_occ * occ_bad;
    // positions are in card order, so the lowest differing position is the lowest differing card
    if (obj < best || (obj == best && ((x ^ best_set) & (0u - (x ^ best_set)) & x))) {
      best = obj;
      best_link = link_bad;
      best_set = x;
    }
    const uint32_t lo = x & (0u - x), up = x + lo;   // next subset with the same popcount
    x = lo ? (((x ^ up) >> 2) / lo) | up : last;
  }
  out->clear();
  for (uint32_t r = best_set; r; r &= r - 1) out->push_back(E[__builtin_ctz(r)]);
  if (quality) *quality = (int32_t)(10000 - best_link / 100);
  return true;
}

// ============================================================== cycle
int32_t Engine::num_feasible_to_find(int32_t all) const {
  const int32_t kMin = 100;
  if (all < kMin || pct_nodes_ >= 100) return all;
  int32_t pct = pct_nodes_;
  if (pct <= 0) {
    pct = 50 - all / 125;
    if (pct < 5) pct = 5;
  }
  int32_t num = (int32_t)((int64_t)all * pct / 100);
  return num < kMin ? kMin : num;
}

std::vector<int32_t> Engine::feasible_nodes(const PodReq& req, const std::vector<int32_t>& candidates,
                                            std::vector<int32_t>* reasons, bool exhaustive) {
  std::vector<int32_t> all;
  if (candidates.empty()) {
    all.reserve(live_);
    for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i)
      if (nodes_[i].alive) all.push_back(i);
  } else {
    all = candidates;
  }
  const int32_t N = (int32_t)all.size();
  std::vector<int32_t> feasible;
  if (reasons) reasons->assign(RS_NUM, 0);
  if (N == 0) return feasible;
  const int32_t want = exhaustive ? N : num_feasible_to_find(N);
  feasible.reserve(std::min(want, N));
  const int32_t start = next_start_ % N;
  SpreadPF pf_store;
  const SpreadPF* pf = nullptr;
  if (wants_spread_filter(req)) {
    spread_prefilter(req, &pf_store);
    pf = &pf_store;
  }
  InterPodPF ip_store;
  const InterPodPF* ip = nullptr;
  if (wants_interpod_filter(req)) {
    interpod_prefilter(req, &ip_store);
    ip = &ip_store;
  }
  std::vector<int8_t> res;
  int32_t processed = 0;
  // chunks big enough to amortise a parallel_for (>= 512 nodes) yet small enough that the
  // adaptive percentageOfNodesToScore early exit still saves work on huge clusters
  const int32_t chunk = pool_ ? std::max(1024, pool_->size() * 256) : N;
  for (int32_t base = 0; base < N && (int32_t)feasible.size() < want; base += chunk) {
    int32_t len = std::min(chunk, N - base);
    res.assign(len, 0);
    auto body = [&](int b, int e) {
      for (int j = b; j < e; ++j) {
        int32_t idx = all[(start + base + j) % N];
        res[j] = (int8_t)filter_node_pf(req, idx, nullptr, nullptr, nullptr, pf, ip);
      }
    };
    if (pool_ && len >= 512) pool_->parallel_for(len, 64, body);
    else body(0, len);
    for (int32_t j = 0; j < len; ++j) {
      ++processed;
      if (res[j] == RS_OK) {
        feasible.push_back(all[(start + base + j) % N]);
        if ((int32_t)feasible.size() >= want) break;
      } else if (reasons) {
        (*reasons)[res[j]]++;
      }
    }
  }
  next_start_ = (start + processed) % N;
  return feasible;
}

static void default_normalize(std::vector<int64_t>& s, bool reverse) {
  int64_t mx = 0;
  for (int64_t v : s) mx = std::max(mx, v);
  if (mx == 0) {
    if (reverse)
      for (auto& v : s) v = kMaxNodeScore;
    return;
  }
  for (auto& v : s) {
    v = kMaxNodeScore * v / mx;
    if (reverse) v = kMaxNodeScore - v;
  }
}

std::vector<int64_t> Engine::score_nodes(const PodReq& req, const std::vector<int32_t>& feas) {
  const size_t F = feas.size();
  std::vector<int64_t> total(F, 0);
  std::vector<int64_t> s(F);
  if (score_w_[S_YODA] && (filters_ & F_YODA)) {
    uint64_t mx[6];
    if (compat_) {
      // reference: maxima over every Scv in the cluster (collection.go:39)
      std::vector<int32_t> all;
      for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i)
        if (nodes_[i].alive && nodes_[i].has_scv) all.push_back(i);
      collect_max(req, all, mx);
    } else {
      collect_max(req, feas, mx);
    }
    auto body = [&](int b, int e) {
      for (int i = b; i < e; ++i) s[i] = (int64_t)yoda_raw_score(req, feas[i], mx);
    };
    if (pool_ && F >= 512) pool_->parallel_for((int)F, 64, body);
    else body(0, (int)F);
    normalize_yoda(s);
    for (size_t i = 0; i < F; ++i) total[i] += s[i] * score_w_[S_YODA];
  }
  // upstream resourceAllocationScorer: node NonZeroRequested + the pod's non-zero request
  const int64_t nz_cpu = req.nz_cpu_m, nz_mem = req.nz_mem;
  if (score_w_[S_LEAST_ALLOCATED] || score_w_[S_MOST_ALLOCATED] || score_w_[S_BALANCED_ALLOCATION]) {
    for (size_t i = 0; i < F; ++i) {
      const Node& n = nodes_[feas[i]];
      int64_t rc = n.nz_cpu_m + nz_cpu, rm = n.nz_mem + nz_mem;
      int64_t lc = 0, lm = 0, mc = 0, mm = 0;
      if (n.alloc_cpu_m > 0 && rc <= n.alloc_cpu_m) lc = (n.alloc_cpu_m - rc) * 100 / n.alloc_cpu_m;
      if (n.alloc_mem > 0 && rm <= n.alloc_mem) lm = (int64_t)((__int128)(n.alloc_mem - rm) * 100 / n.alloc_mem);
      if (n.alloc_cpu_m > 0) mc = std::min<int64_t>(rc, n.alloc_cpu_m) * 100 / n.alloc_cpu_m;
      if (n.alloc_mem > 0) mm = (int64_t)((__int128)std::min<int64_t>(rm, n.alloc_mem) * 100 / n.alloc_mem);
      // upstream resourceAllocationScorer: Σ score_r·w_r / Σ w_r (default cpu=memory=1 → (c+m)/2)
      const int64_t* wl = alloc_w_[0];
      const int64_t* wm = alloc_w_[1];
      const int64_t dl = wl[0] + wl[1] + wl[2], dm = wm[0] + wm[1] + wm[2];
      const int64_t least = dl > 0 ? (lc * wl[0] + lm * wl[1]) / dl : 0;
      const int64_t most = dm > 0 ? (mc * wm[0] + mm * wm[1]) / dm : 0;
      total[i] += score_w_[S_LEAST_ALLOCATED] * least + score_w_[S_MOST_ALLOCATED] * most;
      if (score_w_[S_BALANCED_ALLOCATION]) {
        double cf = n.alloc_cpu_m > 0 ? (double)rc / (double)n.alloc_cpu_m : 1.0;
        double mf = n.alloc_mem > 0 ? (double)rm / (double)n.alloc_mem : 1.0;
        int64_t b = (cf >= 1 || mf >= 1) ? 0 : (int64_t)((1.0 - std::abs(cf - mf)) * 100);
        total[i] += score_w_[S_BALANCED_ALLOCATION] * b;
      }
    }
  }
  if (score_w_[S_TAINT_TOLERATION]) {
    for (size_t i = 0; i < F; ++i) {
      int64_t cnt = 0;
      for (const Taint& x : nodes_[feas[i]].taints) {
        if (x.effect != kPreferNoSchedule) continue;
        bool ok = false;
        for (const Toleration& t : req.tolerations)
          if ((t.effect == kEffectAny || t.effect == kPreferNoSchedule) && tolerates(t, x)) { ok = true; break; }
        if (!ok) ++cnt;
      }
      s[i] = cnt;
    }
    default_normalize(s, true);
    for (size_t i = 0; i < F; ++i) total[i] += s[i] * score_w_[S_TAINT_TOLERATION];
  }
  if (score_w_[S_NODE_AFFINITY] && !req.preferred_terms.empty()) {
    for (size_t i = 0; i < F; ++i) {
      int64_t w = 0;
      for (const PrefTerm& p : req.preferred_terms)
        if (term_matches(p.term, nodes_[feas[i]])) w += p.weight;
      s[i] = w;
    }
    default_normalize(s, false);
    for (size_t i = 0; i < F; ++i) total[i] += s[i] * score_w_[S_NODE_AFFINITY];
  }
  if (score_w_[S_IMAGE_LOCALITY] && images_matter(req)) {
    // plugins/node_extras.py ImageLocality (upstream v1.20 imagelocality): Σ size × spread,
    // spread = nodes holding the image / all nodes, clamped to [23 MB, 1000 MB × containers]
    for (size_t i = 0; i < F; ++i) total[i] += score_w_[S_IMAGE_LOCALITY] * image_score(req, nodes_[feas[i]]);
  }
  if (score_w_[S_PREFER_AVOID]) {
    // plugins/node_extras.py NodePreferAvoidPods: 0 where the node's preferAvoidPods
    // annotation names the pod's RC / RS controller, 100 elsewhere
    for (size_t i = 0; i < F; ++i) {
      int64_t v = kMaxNodeScore;
      if (req.avoid_kind)
        for (const auto& a : nodes_[feas[i]].avoid)
          if (a.first == req.avoid_kind && a.second == req.avoid_uid) {
            v = 0;
            break;
          }
      total[i] += score_w_[S_PREFER_AVOID] * v;
    }
  }
  if (score_w_[S_SPREAD]) {
    spread_scores(req, feas, s);
    for (size_t i = 0; i < F; ++i) total[i] += s[i] * score_w_[S_SPREAD];
  }
  if (score_w_[S_INTERPOD]) {
    interpod_scores(req, feas, s);
    for (size_t i = 0; i < F; ++i) total[i] += s[i] * score_w_[S_INTERPOD];
  }
  return total;
}

// ============================================================== default plugins: inter-pod affinity
bool Engine::wants_interpod_filter(const PodReq& req) const {
  if (!(filters_ & F_INTERPOD)) return false;
  if (req.aff && (!req.aff->req_aff.empty() || !req.aff->req_anti.empty())) return true;
  return !anti_holders_.empty();
}

void Engine::interpod_prefilter(const PodReq& req, InterPodPF* pf) const {
  // InterPodAffinity.pre_filter (plugins/spread_affinity.py): the (key, value) domains where an
  // existing pod's required anti-affinity matches this pod; per required term of this pod the
  // domains holding pods that match it (affinity: pods matching every term)
  pf->active = true;
  pf->existing_anti.clear();
  pf->affinity.clear();
  pf->anti.clear();
  pf->any_aff_match = false;
  if (!anti_holders_.empty())
    for (const auto& bucket : aff_sets_)
      for (const AffSet& set : bucket.second)
        for (const PodTerm& t : set.aff->req_anti) {
          if (!t.matches(req.ns, req.labels)) continue;
          for (const auto& nc : set.nodes) {
            if (nc.first < 0 || nc.first >= (int32_t)nodes_.size() || !nodes_[nc.first].alive) continue;
            const Node& n = nodes_[nc.first];
            auto lab = n.labels.find(t.key);
            if (lab != n.labels.end()) pf->existing_anti[t.key].insert(lab->second);
          }
        }
  if (!req.aff) return;
  const auto& aff = req.aff->req_aff;
  const auto& anti = req.aff->req_anti;
  if (aff.empty() && anti.empty()) return;
  bool self = true;
  for (const PodTerm& t : aff) self = self && t.matches(req.ns, req.labels);
  pf->self_match = self;
  for (const Node& n : nodes_) {
    if (!n.alive || n.pods.empty()) continue;
    if (!aff.empty()) {
      int64_t all = 0;
      if (aff.size() == 1) {
        all = term_count(n, aff[0]);
      } else {                                  // a pod must match every term: per label-set group
        for (const auto& g : n.lab_groups) {
          if (g.second.all <= 0) continue;
          const LabSetRec& ls = labsets_[g.first];
          bool m = true;
          for (const PodTerm& t : aff)
            if (!t.matches(ls.ns, ls.labels)) {
              m = false;
              break;
            }
          if (m) all += g.second.all;
        }
      }
      if (all > 0) {
        // upstream topologyToMatchedAffinityTerms only gains pairs of nodes carrying the key
        for (const PodTerm& t : aff) {
          auto lab = n.labels.find(t.key);
          if (lab == n.labels.end()) continue;
          pf->affinity[pair_key(t.key, lab->second)] += all;
          pf->any_aff_match = true;
        }
      }
    }
    for (const PodTerm& t : anti) {
      auto lab = n.labels.find(t.key);
      if (lab == n.labels.end()) continue;
      const int64_t c = term_count(n, t);
      if (c) pf->anti[pair_key(t.key, lab->second)] += c;
    }
  }
}

Reason Engine::interpod_filter(const PodReq& req, const Node& n, const InterPodPF& pf) const {
  for (const auto& kv : pf.existing_anti) {
    auto lab = n.labels.find(kv.first);
    if (lab != n.labels.end() && kv.second.count(lab->second)) return RS_EXISTING_ANTI;
  }
  if (!req.aff) return RS_OK;
  const auto& aff = req.aff->req_aff;
  if (!aff.empty()) {
    bool ok = true, keys = true;
    for (const PodTerm& t : aff) {
      auto lab = n.labels.find(t.key);
      if (lab == n.labels.end()) {
        ok = keys = false;
        continue;
      }
      auto c = pf.affinity.find(pair_key(t.key, lab->second));
      if (c == pf.affinity.end() || c->second <= 0) ok = false;
    }
    // the first pod of a self-affine group may go to any node carrying the keys
    if (!ok && !(!pf.any_aff_match && pf.self_match && keys)) return RS_POD_AFFINITY;
  }
  for (const PodTerm& t : req.aff->req_anti) {
    auto lab = n.labels.find(t.key);
    if (lab == n.labels.end()) continue;
    auto c = pf.anti.find(pair_key(t.key, lab->second));
    if (c != pf.anti.end() && c->second > 0) return RS_POD_ANTI;
  }
  return RS_OK;
}

void Engine::interpod_scores(const PodReq& req, const std::vector<int32_t>& feas, std::vector<int64_t>& s) const {
  // InterPodAffinity.pre_score / score / normalize_score: per (key, value) domain, Σ ± weight of
  // this pod's preferred terms over the pods there, plus existing pods' required affinity
  // (hardPodAffinityWeight) and preferred terms that match this pod
  const size_t F = feas.size();
  s.assign(F, 0);
  std::unordered_map<uint64_t, int64_t> dom;   // (key, value) → score
  std::unordered_set<int32_t> keys;
  const bool pref = req.aff && (!req.aff->pref_aff.empty() || !req.aff->pref_anti.empty());
  if (pref) {
    // Σ over the pods a term matches of ± its weight = ± weight × the node's matching count
    for (const Node& n : nodes_) {
      if (!n.alive || n.pods.empty()) continue;
      for (int sign = 1; sign >= -1; sign -= 2)
        for (const PodTerm& t : sign > 0 ? req.aff->pref_aff : req.aff->pref_anti) {
          auto lab = n.labels.find(t.key);
          if (lab == n.labels.end()) continue;
          const int64_t c = term_count(n, t);
          if (!c) continue;
          dom[pair_key(t.key, lab->second)] += sign * (int64_t)t.weight * c;
          keys.insert(t.key);
        }
    }
  }
  // existing pods' terms, once per term set: a matching term adds its weight per holder pod
  for (const auto& bucket : aff_sets_)
    for (const AffSet& set : bucket.second) {
      auto add = [&](const PodTerm& t, int64_t w) {
        if (!t.matches(req.ns, req.labels)) return;
        for (const auto& nc : set.nodes) {
          if (nc.first < 0 || nc.first >= (int32_t)nodes_.size() || !nodes_[nc.first].alive) continue;
          const Node& n = nodes_[nc.first];
          auto lab = n.labels.find(t.key);
          if (lab == n.labels.end()) continue;
          dom[pair_key(t.key, lab->second)] += w * nc.second;
          keys.insert(t.key);
        }
      };
      if (hard_aff_w_)
        for (const PodTerm& t : set.aff->req_aff) add(t, hard_aff_w_);
      for (const PodTerm& t : set.aff->pref_aff) add(t, t.weight);
      for (const PodTerm& t : set.aff->pref_anti) add(t, -(int64_t)t.weight);
    }
  if (keys.empty() || F == 0) return;
  // upstream v1.20 InterPodAffinity.NormalizeScore: maxCount and minCount start at 0 (so the
  // range always spans 0) and the scale is float64, truncated
  int64_t hi = 0, lo = 0;
  for (size_t i = 0; i < F; ++i) {
    const Node& n = nodes_[feas[i]];
    int64_t v = 0;
    for (int32_t k : keys) {
      auto lab = n.labels.find(k);
      if (lab == n.labels.end()) continue;
      auto d = dom.find(pair_key(k, lab->second));
      if (d != dom.end()) v += d->second;
    }
    s[i] = v;
    hi = std::max(hi, v);
    lo = std::min(lo, v);
  }
  for (size_t i = 0; i < F; ++i)
    s[i] = hi - lo > 0 ? (int64_t)((double)kMaxNodeScore * ((double)(s[i] - lo) / (double)(hi - lo))) : 0;
}

bool Engine::interpod_inert(const PodReq& req) const {
  const bool filt = (filters_ & F_INTERPOD) != 0, score = score_w_[S_INTERPOD] != 0;
  if (filt && req.aff && (!req.aff->req_aff.empty() || !req.aff->req_anti.empty())) return false;
  if (score && req.aff && (!req.aff->pref_aff.empty() || !req.aff->pref_anti.empty())) return false;
  if (!filt && !score) return true;
  // existing pods' terms that would match this pod, once per term set
  for (const auto& bucket : aff_sets_)
    for (const AffSet& set : bucket.second) {
      const PodAffinity& x = *set.aff;
      if (filt)
        for (const PodTerm& t : x.req_anti)
          if (t.matches(req.ns, req.labels)) return false;
      if (score) {
        if (hard_aff_w_)
          for (const PodTerm& t : x.req_aff)
            if (t.matches(req.ns, req.labels)) return false;
        for (const PodTerm& t : x.pref_aff)
          if (t.matches(req.ns, req.labels)) return false;
        for (const PodTerm& t : x.pref_anti)
          if (t.matches(req.ns, req.labels)) return false;
      }
    }
  return true;
}

uint64_t PodAffinity::hash() const {
  uint64_t h = 0x5bd1e9955bd1e995ull;
  auto mix = [&](uint64_t x) {
    h ^= x + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
  };
  const std::vector<PodTerm>* lists[4] = {&req_aff, &req_anti, &pref_aff, &pref_anti};
  for (int l = 0; l < 4; ++l) {
    mix(0x100 + l);
    for (const PodTerm& t : *lists[l]) {
      mix((uint64_t)(uint32_t)t.key << 32 | (uint32_t)t.weight);
      for (int32_t n : t.ns) mix((uint32_t)n);
      mix(t.sel.nothing ? 1 : 2);
      for (const LReq& r : t.sel.reqs) {
        mix((uint64_t)(uint32_t)r.key << 8 | (uint8_t)r.op);
        for (int32_t v : r.values) mix((uint32_t)v);
      }
    }
  }
  return h;
}

void Engine::aff_set_add(Assignment& a) {
  const uint64_t h = a.aff->hash();
  a.aff_hash = h;
  auto& bucket = aff_sets_[h];
  for (AffSet& set : bucket)
    if (set.aff == a.aff || *set.aff == *a.aff) {
      set.nodes[a.node] += 1;
      set.pods += 1;
      return;
    }
  AffSet set;
  set.aff = a.aff;
  set.nodes[a.node] = 1;
  set.pods = 1;
  bucket.push_back(std::move(set));
}

void Engine::aff_set_remove(const Assignment& a, bool) {
  auto b = aff_sets_.find(a.aff_hash);
  if (b == aff_sets_.end()) return;
  auto& bucket = b->second;
  for (size_t i = 0; i < bucket.size(); ++i) {
    AffSet& set = bucket[i];
    if (set.aff != a.aff && !(*set.aff == *a.aff)) continue;
    auto nit = set.nodes.find(a.node);
    if (nit != set.nodes.end() && --nit->second <= 0) set.nodes.erase(nit);
    if (--set.pods <= 0) {
      bucket.erase(bucket.begin() + (long)i);
      if (bucket.empty()) aff_sets_.erase(b);
    }
    return;
  }
}

// ============================================================== default plugins: node extras
bool LSel::matches(const Labels& l) const {
  if (nothing) return false;
  for (const LReq& r : reqs) {
    auto it = std::lower_bound(l.begin(), l.end(), std::make_pair(r.key, INT32_MIN));
    const bool has = it != l.end() && it->first == r.key;
    switch (r.op) {
      case kIn:
        if (!has || std::find(r.values.begin(), r.values.end(), it->second) == r.values.end()) return false;
        break;
      case kNotIn:
        if (has && std::find(r.values.begin(), r.values.end(), it->second) != r.values.end()) return false;
        break;
      case kExists:
        if (!has) return false;
        break;
      case kDoesNotExist:
        if (has) return false;
        break;
      default:
        return false;
    }
  }
  return true;
}

void Engine::index_node_extras(const Node& n, int sign) {
  for (const auto& im : n.images) {
    int32_t& c = image_nodes_[im.first];
    c += sign;
    if (c <= 0) image_nodes_.erase(im.first);
    auto& sz = image_sizes_[im.first];
    int32_t& k = sz[im.second];
    k += sign;
    if (k <= 0) sz.erase(im.second);
    if (sz.empty()) image_sizes_.erase(im.first);
  }
  if (!n.avoid.empty()) avoid_nodes_ += sign;
}

void Engine::set_node_extras(int32_t idx, std::vector<std::pair<int32_t, int64_t>> images,
                             std::vector<std::pair<int32_t, int64_t>> ext_alloc,
                             std::vector<std::pair<int8_t, int32_t>> avoid) {
  Node& n = nodes_.at(idx);
  if (!n.alive) return;
  index_node_extras(n, -1);
  std::sort(images.begin(), images.end());
  images.erase(std::unique(images.begin(), images.end(),
                           [](const auto& a, const auto& b) { return a.first == b.first; }),
               images.end());
  std::sort(ext_alloc.begin(), ext_alloc.end());
  n.images = std::move(images);
  n.ext_alloc = std::move(ext_alloc);
  n.avoid = std::move(avoid);
  index_node_extras(n, +1);
  mark_dirty(idx);
}

int32_t Engine::image_nodes(int32_t image) const {
  auto it = image_nodes_.find(image);
  return it == image_nodes_.end() ? 0 : it->second;
}

int64_t Engine::image_score(const PodReq& req, const Node& n) const {
  const double all = (double)std::max<int32_t>(1, live_);
  const int64_t lo = 23LL << 20, hi = (1000LL << 20) * std::max<int32_t>(1, req.containers);
  int64_t sum = 0;
  for (int32_t im : req.images) {
    auto it = std::lower_bound(n.images.begin(), n.images.end(), std::make_pair(im, INT64_MIN));
    if (it != n.images.end() && it->first == im && it->second)
      sum += (int64_t)((double)it->second * ((double)image_nodes(im) / all));
  }
  sum = std::min(std::max(sum, lo), hi);
  return kMaxNodeScore * (sum - lo) / (hi - lo);
}

bool Engine::image_score_const(const PodReq& req, int64_t* v) const {
  *v = 0;
  if (!score_w_[S_IMAGE_LOCALITY] || !images_matter(req)) return true;
  for (int32_t im : req.images) {
    auto c = image_nodes_.find(im);
    if (c == image_nodes_.end()) continue;
    if (c->second != live_) return false;
    auto sz = image_sizes_.find(im);
    if (sz == image_sizes_.end() || sz->second.size() != 1) return false;
  }
  for (const Node& n : nodes_)
    if (n.alive) {
      *v = score_w_[S_IMAGE_LOCALITY] * image_score(req, n);
      return true;
    }
  return true;
}

int64_t Engine::ext_amount(const std::vector<std::pair<int32_t, int64_t>>& v, int32_t res) const {
  auto it = std::lower_bound(v.begin(), v.end(), std::make_pair(res, INT64_MIN));
  return it != v.end() && it->first == res ? it->second : 0;
}

bool Engine::images_matter(const PodReq& req) const {
  // no node reports any of the pod's images: every node scores 0
  for (int32_t im : req.images)
    if (image_nodes_.count(im)) return true;
  return false;
}

bool Engine::set_pod_meta(uint64_t pod, Labels labels, bool deleting) {
  const int32_t si = ledger_.find(pod);
  if (si < 0) return false;
  std::sort(labels.begin(), labels.end());
  Assignment& a = slab_[si];
  const bool live = a.node >= 0 && a.node < (int32_t)nodes_.size() && nodes_[a.node].alive;
  if (live) index_pod(nodes_[a.node], a, -1);
  const int32_t old = a.labset;
  a.labset = labset_acquire(a.ns, labels);
  labset_release(old);
  a.deleting = deleting;
  if (live) index_pod(nodes_[a.node], a, +1);
  return true;
}

void Engine::index_pod(Node& n, const Assignment& a, int sign) {
  // counts that reach 0 keep their entry (the next pod of the template bumps it without
  // allocating); a node sweeps them once they outnumber the live entries. A pod's label-index
  // entries are found once per (node, label set) — one hash lookup per reserve / release, not
  // one per label
  const int live = a.deleting ? 0 : sign;
  auto gr = n.lab_groups.try_emplace(a.labset);
  Node::LabGroup& g = gr.first->second;
  if (gr.second) ++n.lab_groups_zero;   // a fresh group counts as a zero one until bumped
  if (g.all <= 0) {
    g.idx.clear();
    auto bind = [&](LKey k) {
      auto r = n.lab_idx.try_emplace(k, 0, 0);
      if (r.second) ++n.lab_idx_zero;
      g.idx.push_back(&r.first->second);
    };
    bind(LKey{a.ns, -1, -1});
    for (const auto& kv : labsets_[a.labset].labels) bind(LKey{a.ns, kv.first, kv.second});
  }
  for (std::pair<int32_t, int32_t>* c : g.idx) {
    if (c->first <= 0) --n.lab_idx_zero;
    c->first += sign;
    c->second += live;
    if (c->first <= 0) ++n.lab_idx_zero;
  }
  if (g.all <= 0) --n.lab_groups_zero;
  g.all += sign;
  g.live += live;
  if (g.all <= 0) ++n.lab_groups_zero;
  if (sign < 0 && (n.lab_idx_zero > 64 || n.lab_groups_zero > 64)) sweep_lab_index(n);
}

void Engine::sweep_lab_index(Node& n) {
  if (n.lab_idx_zero * 2 > (int32_t)n.lab_idx.size()) {
    for (auto it = n.lab_idx.begin(); it != n.lab_idx.end();)
      it = it->second.first <= 0 ? n.lab_idx.erase(it) : std::next(it);
    n.lab_idx_zero = 0;
  }
  if (n.lab_groups_zero * 2 > (int32_t)n.lab_groups.size()) {
    for (auto it = n.lab_groups.begin(); it != n.lab_groups.end();)
      it = it->second.all <= 0 ? n.lab_groups.erase(it) : std::next(it);
    n.lab_groups_zero = 0;
  }
}

int64_t Engine::group_count(const Node& n, int32_t ns, const LSel& sel, bool skip_deleting) const {
  if (sel.nothing) return 0;
  int64_t c = 0;
  for (const auto& g : n.lab_groups) {
    if (g.second.all <= 0) continue;
    const LabSetRec& ls = labsets_[g.first];
    if (ls.ns == ns && sel.matches(ls.labels)) c += skip_deleting ? g.second.live : g.second.all;
  }
  return c;
}

int64_t Engine::term_count(const Node& n, const PodTerm& t) const {
  int64_t sum = 0, c = 0;
  bool ok = true;
  for (int32_t ns : t.ns) {
    if (!indexed_count(n, ns, t.sel, false, &c)) {
      ok = false;
      break;
    }
    sum += c;
  }
  if (ok) return sum;
  sum = 0;
  for (int32_t ns : t.ns) sum += group_count(n, ns, t.sel, false);
  return sum;
}

bool Engine::indexed_count(const Node& n, int32_t ns, const LSel& sel, bool skip_deleting, int64_t* out) const {
  if (sel.nothing) {
    *out = 0;
    return true;
  }
  LKey k{ns, -1, -1};
  if (sel.reqs.size() == 1 && sel.reqs[0].op == kIn && sel.reqs[0].values.size() == 1) {
    k.k = sel.reqs[0].key;
    k.v = sel.reqs[0].values[0];
  } else if (!sel.reqs.empty()) {
    return false;
  }
  auto it = n.lab_idx.find(k);
  *out = it == n.lab_idx.end() ? 0 : (skip_deleting ? it->second.second : it->second.first);
  return true;
}

// ============================================================== default plugins: topology spread
void Engine::set_service(int32_t ns, int32_t name, bool nil_selector, Labels selector) {
  std::sort(selector.begin(), selector.end());
  auto& v = svcs_[ns];
  for (auto& x : v)
    if (x.name == name) {
      x.nil = nil_selector;
      x.sel = std::move(selector);
      return;
    }
  v.push_back(Svc{name, nil_selector, std::move(selector)});
  // upstream GetPodServices lists them in name order (the merge below is order-independent for
  // services, which must all agree with the pod's labels, but keep the order anyway)
  std::sort(v.begin(), v.end(), [&](const Svc& a, const Svc& b) { return strings_[a.name] < strings_[b.name]; });
}

void Engine::remove_service(int32_t ns, int32_t name) {
  auto it = svcs_.find(ns);
  if (it == svcs_.end()) return;
  auto& v = it->second;
  v.erase(std::remove_if(v.begin(), v.end(), [&](const Svc& x) { return x.name == name; }), v.end());
  if (v.empty()) svcs_.erase(it);
}

void Engine::set_controller(int8_t kind, int32_t ns, int32_t name, LSel sel) {
  ctrls_[ctrl_key(kind, ns, name)] = std::move(sel);
}

void Engine::remove_controller(int8_t kind, int32_t ns, int32_t name) { ctrls_.erase(ctrl_key(kind, ns, name)); }

bool Engine::default_selector(const PodReq& req, LSel* out) const {
  // plugins/optional.py::default_selector (upstream helper.DefaultSelector): the matching
  // Services' selectors and an RC's map merged as equalities (later keys overwrite), an
  // RS's / StatefulSet's LabelSelector added as requirements
  out->nothing = false;
  out->reqs.clear();
  Labels eq;
  auto put = [&](int32_t k, int32_t v) {
    for (auto& kv : eq)
      if (kv.first == k) {
        kv.second = v;
        return;
      }
    eq.emplace_back(k, v);
  };
  auto sv = svcs_.find(req.ns);
  if (sv != svcs_.end())
    for (const Svc& x : sv->second) {
      if (x.nil) continue;                      // a nil selector matches nothing
      bool all = true;
      for (const auto& kv : x.sel) {
        auto it = std::lower_bound(req.labels.begin(), req.labels.end(), std::make_pair(kv.first, INT32_MIN));
        if (it == req.labels.end() || it->first != kv.first || it->second != kv.second) {
          all = false;
          break;
        }
      }
      if (all)
        for (const auto& kv : x.sel) put(kv.first, kv.second);
    }
  std::vector<LReq> extra;
  if (req.owner_kind) {
    auto c = ctrls_.find(ctrl_key(req.owner_kind, req.ns, req.owner_name));
    if (c != ctrls_.end()) {
      if (req.owner_kind == 1) {
        for (const LReq& r : c->second.reqs)
          if (r.op == kIn && r.values.size() == 1) put(r.key, r.values[0]);
      } else if (!c->second.nothing) {
        extra = c->second.reqs;
      }
    }
  }
  for (const auto& kv : eq) out->reqs.push_back(LReq{kv.first, kIn, {kv.second}});
  for (auto& r : extra) out->reqs.push_back(std::move(r));
  return !out->reqs.empty();
}

void Engine::spread_constraints(const PodReq& req, bool hard, std::vector<SpreadC>* out) const {
  out->clear();
  if (req.spread_explicit) {
    for (const SpreadC& c : req.spread)
      if (c.hard == hard) out->push_back(c);
    return;
  }
  bool any = false;
  for (const DefaultSpread& d : spread_defaults_) any |= d.hard == hard;
  if (!any) return;
  LSel sel;
  if (!default_selector(req, &sel)) return;
  for (const DefaultSpread& d : spread_defaults_)
    if (d.hard == hard) out->push_back(SpreadC{d.key, d.max_skew, d.hard, sel});
}

int64_t Engine::count_matching(int32_t idx, int32_t ns, const LSel& sel) const {
  // upstream countPodsMatchSelector: same namespace, not terminating, selector match
  if (idx < 0 || idx >= (int32_t)nodes_.size() || sel.nothing) return 0;
  int64_t c = 0;
  if (indexed_count(nodes_[idx], ns, sel, true, &c)) return c;
  return group_count(nodes_[idx], ns, sel, true);
}

bool Engine::wants_spread_filter(const PodReq& req) const {
  if (!(filters_ & F_SPREAD)) return false;
  if (req.spread_explicit) {
    for (const SpreadC& c : req.spread)
      if (c.hard) return true;
    return false;
  }
  for (const DefaultSpread& d : spread_defaults_)
    if (d.hard) return true;
  return false;
}


void Engine::spread_prefilter(const PodReq& req, SpreadPF* pf) const {
  // PodTopologySpread.pre_filter (plugins/spread_affinity.py): counts per (key, value) pair —
  // shared by constraints of the same key, as upstream v1.20 — over the nodes that pass the
  // pod's nodeSelector / required node affinity and carry every key
  spread_constraints(req, true, &pf->cons);
  pf->pair_counts.clear();
  pf->min_count.clear();
  if (pf->cons.empty()) return;
  for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i) {
    const Node& n = nodes_[i];
    if (!n.alive) continue;
    bool keys = true;
    for (const SpreadC& c : pf->cons)
      if (!n.labels.count(c.key)) {
        keys = false;
        break;
      }
    if (!keys || !affinity_ok(req, n)) continue;
    for (const SpreadC& c : pf->cons)
      pf->pair_counts[pair_key(c.key, n.labels.at(c.key))] += n.pods.empty() ? 0 : count_matching(i, req.ns, c.sel);
  }
  for (const auto& kv : pf->pair_counts) {
    const int32_t k = (int32_t)(kv.first >> 32);
    auto it = pf->min_count.find(k);
    if (it == pf->min_count.end() || kv.second < it->second) pf->min_count[k] = kv.second;
  }
}

Reason Engine::spread_filter(const PodReq& req, const Node& n, const SpreadPF& pf) const {
  for (const SpreadC& c : pf.cons) {
    auto lab = n.labels.find(c.key);
    if (lab == n.labels.end()) return RS_SPREAD_LABEL;
    const int64_t self = c.sel.matches(req.labels) ? 1 : 0;
    auto pc = pf.pair_counts.find(pair_key(c.key, lab->second));
    auto mc = pf.min_count.find(c.key);
    const int64_t skew = (pc == pf.pair_counts.end() ? 0 : pc->second) + self - (mc == pf.min_count.end() ? 0 : mc->second);
    if (skew > c.max_skew) return RS_SPREAD;
  }
  return RS_OK;
}

bool Engine::spread_soft_constant(const std::vector<SpreadC>& soft) const {
  for (const SpreadC& c : soft)
    if (!label_key_nodes_.count(c.key)) return true;   // every node is "ignored": all score 0
  return false;
}


void Engine::spread_scores(const PodReq& req, const std::vector<int32_t>& feas, std::vector<int64_t>& s) const {
  // PodTopologySpread pre_score / score / normalize_score (plugins/spread_affinity.py)
  const size_t F = feas.size();
  s.assign(F, 0);
  std::vector<SpreadC> soft;
  spread_constraints(req, false, &soft);
  if (soft.empty() || F == 0 || spread_soft_constant(soft)) return;
  static const std::string kHostname = "kubernetes.io/hostname";
  auto hit = string_idx_.find(kHostname);
  const int32_t host_key = hit == string_idx_.end() ? -1 : hit->second;
  std::vector<char> ignored(F, 0);
  size_t n_ignored = 0;
  std::unordered_map<uint64_t, int64_t> pairs;   // non-hostname pairs among the scored nodes
  std::vector<int64_t> sizes(soft.size(), 0);
  for (size_t i = 0; i < F; ++i) {
    const Node& n = nodes_[feas[i]];
    bool keys = true;
    for (const SpreadC& c : soft)
      if (!n.labels.count(c.key)) {
        keys = false;
        break;
      }
    if (!keys) {
      ignored[i] = 1;
      ++n_ignored;
      continue;
    }
    for (size_t k = 0; k < soft.size(); ++k) {
      if (soft[k].key == host_key) continue;
      if (pairs.emplace(pair_key(soft[k].key, n.labels.at(soft[k].key)), 0).second) ++sizes[k];
    }
  }
  std::vector<double> w(soft.size());
  for (size_t k = 0; k < soft.size(); ++k)
    w[k] = std::log((double)((soft[k].key == host_key ? (int64_t)(F - n_ignored) : sizes[k]) + 2));
  if (!pairs.empty()) {
    for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i) {
      const Node& n = nodes_[i];
      if (!n.alive) continue;
      bool keys = true;
      for (const SpreadC& c : soft)
        if (!n.labels.count(c.key)) {
          keys = false;
          break;
        }
      if (!keys || !affinity_ok(req, n)) continue;
      for (const SpreadC& c : soft) {
        auto p = pairs.find(pair_key(c.key, n.labels.at(c.key)));
        if (p != pairs.end() && !n.pods.empty()) p->second += count_matching(i, req.ns, c.sel);
      }
    }
  }
  bool any = false;
  int64_t lo = 0, hi = 0;
  for (size_t i = 0; i < F; ++i) {
    if (ignored[i]) continue;
    const Node& n = nodes_[feas[i]];
    double total = 0.0;
    for (size_t k = 0; k < soft.size(); ++k) {
      auto lab = n.labels.find(soft[k].key);
      if (lab == n.labels.end()) continue;
      int64_t cnt;
      if (soft[k].key == host_key) {
        cnt = count_matching(feas[i], req.ns, soft[k].sel);
      } else {
        auto p = pairs.find(pair_key(soft[k].key, lab->second));
        cnt = p == pairs.end() ? 0 : p->second;
      }
      total += (double)cnt * w[k] + (double)(soft[k].max_skew - 1);
    }
    s[i] = (int64_t)total;
    lo = any ? std::min(lo, s[i]) : s[i];
    hi = std::max(hi, s[i]);
    any = true;
  }
  for (size_t i = 0; i < F; ++i) {
    if (ignored[i]) s[i] = 0;
    else if (hi == 0) s[i] = kMaxNodeScore;
    else s[i] = floor_div(kMaxNodeScore * (hi + lo - s[i]), hi);
  }
}

CycleResult Engine::schedule(uint64_t pod, const PodReq& req, bool assume, const std::vector<int32_t>& candidates,
                             const std::vector<int64_t>& extra) {
  ++cycles_;
  CycleResult r;
  // a cycle the device scorer covers scores every feasible node (the kernel filters and scores
  // the whole table in one pass, so percentageOfNodesToScore's early exit saves it nothing);
  // the CPU path of such a cycle (device busy, abandoned or failed) does the same, so both
  // paths choose from the same node set
  const bool dev_covers = dev_ctx_ && candidates.empty() && extra.empty() && live_ >= dev_min_nodes_ &&
                          device_eligible(req);
  if (dev_covers) {
    // a batch may hold the device (its engine lock dropped): then this cycle runs on the
    // CPU path, which is bit-exact with the device
    std::unique_lock<std::mutex> dl(dev_mu_, std::try_to_lock);
    if (dl.owns_lock() && schedule_device(req, &r)) {
      dl.unlock();
      if (r.node >= 0) r.node_gen = nodes_[r.node].gen;
      if (assume && r.node >= 0) reserve(pod, req, r.node, r.cards);
      return r;
    }
    r = CycleResult();
  }
  std::vector<int32_t> feas = feasible_nodes(req, candidates, &r.reason_counts, dev_covers);
  r.feasible = (int32_t)feas.size();
  r.evaluated = candidates.empty() ? live_ : (int32_t)candidates.size();
  if (feas.empty()) return r;
  int32_t chosen;
  if (feas.size() == 1) {
    chosen = feas[0];   // upstream: exactly one feasible node → no scoring
  } else {
    std::vector<int64_t> sc = score_nodes(req, feas);
    if (!extra.empty()) {
      std::unordered_map<int32_t, int64_t> ex;
      for (size_t i = 0; i < candidates.size() && i < extra.size(); ++i) ex[candidates[i]] = extra[i];
      for (size_t i = 0; i < feas.size(); ++i) {
        auto it = ex.find(feas[i]);
        if (it != ex.end()) sc[i] += it->second;
      }
    }
    // selectHost: max score, reservoir-sampled tie break
    int64_t best = sc[0];
    chosen = feas[0];
    uint64_t cnt = 1;
    for (size_t i = 1; i < feas.size(); ++i) {
      if (sc[i] > best) {
        best = sc[i];
        chosen = feas[i];
        cnt = 1;
      } else if (sc[i] == best) {
        ++cnt;
        if (rng_() % cnt == 0) chosen = feas[i];
      }
    }
    r.score = best;
  }
  r.node = chosen;
  r.node_gen = nodes_[chosen].gen;
  if (filters_ & F_YODA) {
    int32_t q = 10000;
    if (!select_gpus(req, chosen, &r.cards, &q) && !compat_) {
      // cannot happen in fixed mode (filter guarantees eligibility); be defensive
      r.node = -1;
      r.reason_counts.assign(RS_NUM, 0);
      r.reason_counts[RS_GPU_FIT] = 1;
      return r;
    }
    r.gang_quality = q;
  }
  if (assume) reserve(pod, req, chosen, r.cards);
  return r;
}

std::vector<CycleResult> Engine::schedule_batch(const std::vector<uint64_t>& pods,
                                                const std::vector<const PodReq*>& reqs) {
  // Maximal runs of batch-eligible pods go to the device as one k_batch dispatch each; the pods
  // between them take per-pod cycles (device per-pod cycle or CPU), in creation order, so each
  // pod still sees every earlier pod's reservation. One pod the device cannot carry no longer
  // sends the whole batch to per-pod cycles (VERDICT r5 next #3a).
  std::vector<CycleResult> out;
  out.reserve(pods.size());
  static const std::vector<int32_t> none;
  static const std::vector<int64_t> nox;
  const size_t n = std::min(pods.size(), reqs.size());
  const bool dev = dev_ctx_ && fn_schedule_batch_ && live_ >= dev_min_nodes_;
  BatchCols cols;
  size_t i = 0;
  while (i < n) {
    size_t j = i;
    cols.spread.clear();
    cols.image.clear();
    cols.pods.clear();
    // a run ends at a pod the device cannot carry, one needing a third column slot, or after
    // one k_batch chunk when it uses columns (the staged columns are the chunk's start)
    if (dev)
      while (j < n && batch_eligible(*reqs[j]) && (j - i) < 256 && assign_cols(*reqs[j], &cols)) ++j;
    const bool use_cols = !cols.spread.empty() || !cols.image.empty();
    if (j - i >= (use_cols ? 1u : 2u) &&
        schedule_batch_device(pods.data() + i, reqs.data() + i, j - i, &out, use_cols ? &cols : nullptr)) {
      ++dev_batches_;
      i = j;
      continue;
    }
    // a lone eligible pod, an ineligible one, or a run the device refused: per-pod cycles
    const size_t end = std::max(j, i + 1);
    for (; i < end; ++i) out.push_back(schedule(pods[i], *reqs[i], true, none, nox));
  }
  return out;
}

bool Engine::batch_eligible(const PodReq& q) const {
  return device_eligible(q, fn_extras_ != nullptr) && !needs_candidates(q) && !(q.has_memory && q.memory > UINT32_MAX);
}

// ============================================================== device scorer (dlopen)
using dev_create_t = void* (*)(int, int, char*, int);
using dev_destroy_t = void (*)(void*);
using dev_upload_t = int (*)(void*, int, const int32_t*, const yoda_dev_node_t*);
using dev_schedule_t = int (*)(void*, int, const yoda_dev_req_t*, const uint8_t*, yoda_dev_result_t*);
using dev_last_us_t = float (*)(void*);

void Engine::mark_dirty(int32_t idx) {
  if (!dev_ctx_ || idx < 0) return;
  if ((int32_t)dirty_.size() <= idx) dirty_.resize(idx + 1, 0);
  if (!dirty_[idx]) {
    dirty_[idx] = 1;
    dirty_list_.push_back(idx);
  }
}

bool Engine::enable_device(const std::string& lib_path, int device, int capacity, int min_nodes, std::string* err) {
  disable_device();
  void* lib = dlopen(lib_path.c_str(), RTLD_NOW | RTLD_GLOBAL);
  if (!lib) {
    if (err) *err = std::string("dlopen: ") + dlerror();
    return false;
  }
  auto create = (dev_create_t)dlsym(lib, "yoda_dev_create");
  fn_destroy_ = dlsym(lib, "yoda_dev_destroy");
  fn_upload_ = dlsym(lib, "yoda_dev_upload");
  fn_schedule_ = dlsym(lib, "yoda_dev_schedule");
  fn_last_us_ = dlsym(lib, "yoda_dev_last_us");
  fn_set_timing_ = dlsym(lib, "yoda_dev_set_timing");
  fn_schedule_batch_ = dlsym(lib, "yoda_dev_schedule_batch");   // optional
  fn_busy_ = dlsym(lib, "yoda_dev_busy");                         // optional
  fn_extras_ = dlsym(lib, "yoda_dev_batch_extras");               // optional
  if (!create || !fn_destroy_ || !fn_upload_ || !fn_schedule_ || !fn_last_us_) {
    if (err) *err = "libyoda_hip.so lacks the yoda_dev_* entry points";
    dlclose(lib);
    return false;
  }
  char buf[256] = {0};
  void* ctx = create(device, capacity, buf, sizeof buf);
  if (!ctx) {
    if (err) *err = buf;
    dlclose(lib);
    return false;
  }
  dev_lib_ = lib;
  dev_ctx_ = ctx;
  dev_cap_ = capacity;
  dev_min_nodes_ = min_nodes;
  // everything is dirty for the first device cycle
  dirty_.assign(nodes_.size(), 0);
  dirty_list_.clear();
  for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i) mark_dirty(i);
  return true;
}

void Engine::disable_device() {
  if (dev_ctx_) ((dev_destroy_t)fn_destroy_)(dev_ctx_);
  if (dev_lib_) dlclose(dev_lib_);
  dev_ctx_ = dev_lib_ = nullptr;
  dirty_.clear();
  dirty_list_.clear();
}

float Engine::device_last_us() const { return dev_ctx_ ? ((dev_last_us_t)fn_last_us_)(dev_ctx_) : 0.f; }

void Engine::device_set_timing(bool on) {
  if (dev_ctx_ && fn_set_timing_) ((void (*)(void*, int))fn_set_timing_)(dev_ctx_, on ? 1 : 0);
}

bool Engine::pack_node(int32_t idx, void* out) const {
  yoda_dev_node_t* row = (yoda_dev_node_t*)out;
  std::memset(row, 0, sizeof(*row));
  const Node& n = nodes_[idx];
  if (!n.alive) return true;   // flags 0 = dead slot
  if (n.cards.size() > YODA_DEV_CARDS || n.nphys > YODA_DEV_CARDS || n.card_number > UINT32_MAX) return false;
  row->flags = YODA_DEV_ALIVE | (n.has_scv ? YODA_DEV_HAS_SCV : 0) | (n.stale ? YODA_DEV_STALE : 0) |
               (n.unschedulable ? YODA_DEV_UNSCHEDULABLE : 0);
  row->ncards = (uint8_t)n.cards.size();
  row->nphys = (uint8_t)n.nphys;
  row->card_number = (uint32_t)n.card_number;
  row->alloc_cpu = n.alloc_cpu_m;
  row->alloc_mem = n.alloc_mem;
  row->alloc_pods = n.alloc_pods;
  row->req_cpu = n.req_cpu_m;
  row->req_mem = n.req_mem;
  row->nz_cpu = n.nz_cpu_m;
  row->nz_mem = n.nz_mem;
  row->ext_alloc = ext_amount(n.ext_alloc, dev_ext_res_);
  row->ext_used = ext_amount(n.ext_used, dev_ext_res_);
  row->pod_count = n.pod_count;
  if (n.alloc_mem > (int64_t)1 << 56 || n.alloc_cpu_m > (int64_t)1 << 56) return false;
  for (size_t c = 0; c < n.cards.size(); ++c) {
    const Card& x = n.cards[c];
    const uint64_t vals[8] = {x.total_mb, x.free_mb, x.reserved_mb, x.pending_mb, x.clock, x.bandwidth, x.core, x.power};
    for (uint64_t v : vals)
      if (v > UINT32_MAX) return false;
    if (x.phys < 0 || x.phys >= YODA_DEV_CARDS) return false;
    row->cards[c] = yoda_dev_card_t{(uint32_t)x.total_mb, (uint32_t)x.free_mb, (uint32_t)x.reserved_mb,
                                    (uint32_t)x.pending_mb, (uint32_t)x.clock, (uint32_t)x.bandwidth,
                                    (uint32_t)x.core, (uint32_t)x.power};
    row->healthy[c] = x.healthy;
    row->phys[c] = (uint8_t)x.phys;
    row->numa[c] = (uint8_t)(x.numa & 63);
    row->occ[c] = (uint16_t)std::min(std::max(x.occ_q, 0), 65535);
  }
  // card-pair link quality, resolved here so the device needs no phys indirection
  // (same rule as gang_objective: same physical GPU or unknown link → 10000)
  for (size_t a = 0; a < n.cards.size(); ++a)
    for (size_t b = 0; b < n.cards.size(); ++b) {
      const int32_t pa = n.cards[a].phys, pb = n.cards[b].phys;
      int32_t q = 10000;
      if (pa != pb && pa < n.nphys && pb < n.nphys) q = n.link_q[(size_t)pa * n.nphys + pb];
      if (q < 0 || q > 65535) return false;   // not representable: CPU path
      row->linkq[a][b] = (uint16_t)q;
    }
  return true;
}

bool Engine::flush_dirty() {
  // the device still drains a call it abandoned (a tenant kernel holds the GPU): refuse
  // before packing rows — after an abandoned batch every row is dirty, and packing them for
  // each refused per-pod attempt cost more than the CPU cycles themselves
  if (fn_busy_ && ((int (*)(void*))fn_busy_)(dev_ctx_)) return false;
  if (dirty_list_.empty()) return true;
  std::vector<yoda_dev_node_t> rows(dirty_list_.size());
  for (size_t i = 0; i < dirty_list_.size(); ++i)
    if (!pack_node(dirty_list_[i], &rows[i])) return false;   // stays dirty; CPU path this cycle
  if (((dev_upload_t)fn_upload_)(dev_ctx_, (int)dirty_list_.size(), dirty_list_.data(), rows.data()) != 0)
    return false;
  for (int32_t i : dirty_list_) dirty_[i] = 0;
  dirty_list_.clear();
  return true;
}

bool Engine::device_eligible(const PodReq& req, bool slots) const {
  if (!dev_ctx_ || compat_) return false;
  if ((int32_t)nodes_.size() > dev_cap_) return false;
  if (wt_.enum_limit < 70) return false;                       // device search is always exhaustive
  if (score_w_[S_NODE_AFFINITY] && !req.preferred_terms.empty()) return false;
  if (score_w_[S_TAINT_TOLERATION] && prefer_taint_nodes_ > 0) return false;
  int64_t wsum = 0;
  for (int i = 0; i < S_NUM; ++i) wsum += score_w_[i] < 0 ? -score_w_[i] : score_w_[i];
  if (wsum * 200 >= ((int64_t)1 << 38)) return false;          // key = (final << 24) | perm
  // the device forms the gang objective with 32×32-bit multiply-adds: |w| ≤ 10^6
  if (wt_.w_minlink < 0 || wt_.w_minlink > 1000000) return false;
  if (wt_.w_link < 0 || wt_.w_link > 1000000 || wt_.w_numa > 1000000 || wt_.w_fit > 1000000 || wt_.w_occ > 1000000 ||
      wt_.w_numa < -1000000 || wt_.w_fit < -1000000 || wt_.w_occ < -1000000)
    return false;
  if (!default_alloc_weights()) return false;                    // device computes (c + m) / 2
  // NodePorts: the device row carries no host ports, and pods placed in one device batch would
  // not see each other's
  if ((filters_ & F_NODE_PORTS) && !req.host_ports.empty()) return false;
  if (!req.vol.empty() || req.count_vols) return false;   // PV node affinity / zones / attach limits: not in the device row
  // default-plugin terms the device row does not carry: only pods for which they are a
  // constant (or nothing) go to the device
  if ((filters_ & F_NODE_RESOURCES_FIT) && !req.ext.empty())
    for (const auto& r : req.ext)   // the device carries one extended resource dimension
      if (r.first != dev_ext_res_ && ext_checked(r.first)) return false;
  int64_t img;
  if (!slots && !image_score_const(req, &img)) return false;   // (k_batch: an image slot)
  if (!interpod_inert(req)) return false;
  if (score_w_[S_PREFER_AVOID] && req.avoid_kind && avoid_nodes_ > 0) return false;
  if (wants_spread_filter(req)) {
    std::vector<SpreadC> hard;
    spread_constraints(req, true, &hard);
    if (!hard.empty()) return false;
  }
  if (score_w_[S_SPREAD] && !slots) {   // (k_batch: a spread slot, assign_cols)
    std::vector<SpreadC> soft;
    spread_constraints(req, false, &soft);
    if (!soft.empty() && !spread_soft_constant(soft)) return false;
  }
  return true;
}

bool Engine::assign_cols(const PodReq& q, BatchCols* cols) const {
  BatchCols::PodCols pc;
  int64_t img_const;
  if (score_w_[S_IMAGE_LOCALITY] && !image_score_const(q, &img_const)) {
    int k = 0;
    while (k < (int)cols->image.size() && !(cols->image[k].first == q.images && cols->image[k].second == q.containers)) ++k;
    if (k == (int)cols->image.size()) {
      if (k >= YODA_DEV_IMAGE_SLOTS) return false;
      cols->image.emplace_back(q.images, q.containers);
    }
    pc.image = (int8_t)k;
  }
  if (score_w_[S_SPREAD]) {
    std::vector<SpreadC> soft;
    spread_constraints(q, false, &soft);
    if (!soft.empty() && !spread_soft_constant(soft)) {
      // representable: ≤ 2 constraints of one selector, at most one on kubernetes.io/hostname
      // and one on another key (the slot's domain key)
      if (soft.size() > 2) return false;
      static const std::string kHostname = "kubernetes.io/hostname";
      auto hit = string_idx_.find(kHostname);
      const int32_t host_key = hit == string_idx_.end() ? -1 : hit->second;
      BatchCols::Spread sp;
      sp.ns = q.ns;
      sp.sel = soft[0].sel;
      for (size_t c = 0; c < soft.size(); ++c) {
        if (!(soft[c].sel == sp.sel)) return false;
        if (soft[c].key == host_key) {
          if (sp.host) return false;
          sp.host = true;
          pc.ckind[c] = 0;
        } else {
          if (sp.dom_key >= 0) return false;
          sp.dom_key = soft[c].key;
          pc.ckind[c] = 1;
        }
        pc.skew[c] = soft[c].max_skew;
      }
      pc.nc = (uint8_t)soft.size();
      int k = 0;
      while (k < (int)cols->spread.size()) {
        const BatchCols::Spread& x = cols->spread[k];
        if (x.ns == sp.ns && x.host == sp.host && x.dom_key == sp.dom_key && x.sel == sp.sel) break;
        ++k;
      }
      if (k == (int)cols->spread.size()) {
        if (k >= YODA_DEV_SPREAD_SLOTS) return false;
        cols->spread.push_back(std::move(sp));
      }
      pc.spread = (int8_t)k;
    }
  }
  cols->pods.push_back(pc);
  return true;
}

bool Engine::stage_cols(const BatchCols& cols, const PodReq* const* reqs, size_t count) {
  const int n = (int)nodes_.size();
  const int ns = (int)cols.spread.size(), ni = (int)cols.image.size();
  if (!ns && !ni) return true;
  if (!fn_extras_) return false;
  std::vector<int32_t> cnt((size_t)ns * n, 0), zc((size_t)ns * YODA_DEV_DOMAINS, 0);
  std::vector<uint8_t> dom((size_t)ns * n, YODA_DEV_DOM_NONE);
  static const std::string kHostname = "kubernetes.io/hostname";
  auto hit = string_idx_.find(kHostname);
  const int32_t host_key = hit == string_idx_.end() ? -1 : hit->second;
  for (int k = 0; k < ns; ++k) {
    const BatchCols::Spread& sp = cols.spread[k];
    std::unordered_map<int32_t, int32_t> ids;   // domain value → id
    int64_t total = 0;
    for (int32_t i = 0; i < n; ++i) {
      const Node& nd = nodes_[i];
      if (!nd.alive) continue;
      if (sp.host && !nd.labels.count(host_key)) continue;
      int32_t d = 0;
      if (sp.dom_key >= 0) {
        auto lab = nd.labels.find(sp.dom_key);
        if (lab == nd.labels.end()) continue;
        auto it = ids.find(lab->second);
        if (it == ids.end()) {
          if ((int)ids.size() >= YODA_DEV_DOMAINS) return false;   // too many domains: per-pod cycles
          it = ids.emplace(lab->second, (int32_t)ids.size()).first;
        }
        d = it->second;
      }
      const int64_t c = nd.pods.empty() ? 0 : count_matching(i, sp.ns, sp.sel);
      if (c > INT32_MAX / 2) return false;
      cnt[(size_t)k * n + i] = (int32_t)c;
      dom[(size_t)k * n + i] = (uint8_t)d;
      zc[(size_t)k * YODA_DEV_DOMAINS + d] += (int32_t)c;
      total += c;
    }
    // the device keeps a spread raw score in 32 bits: (pods + the batch) × log(n + 2) per
    // constraint, plus the skews
    int64_t skew = 0;
    for (size_t j = 0; j < count; ++j) skew = std::max<int64_t>(skew, cols.pods[j].skew[0] + (int64_t)cols.pods[j].skew[1]);
    if ((double)(total + (int64_t)count) * std::log((double)n + 2.0) * 2.0 + (double)skew > 1.0e9) return false;
  }
  std::vector<int32_t> img((size_t)ni * n, 0);
  for (int k = 0; k < ni; ++k) {
    PodReq tmp;
    tmp.images = cols.image[k].first;
    tmp.containers = cols.image[k].second;
    for (int32_t i = 0; i < n; ++i)
      if (nodes_[i].alive) {
        const int64_t v = score_w_[S_IMAGE_LOCALITY] * image_score(tmp, nodes_[i]);
        if (v > INT32_MAX || v < 0) return false;
        img[(size_t)k * n + i] = (int32_t)v;
      }
  }
  using extras_t = int (*)(void*, int, int, const int32_t*, const uint8_t*, const int32_t*, int, const int32_t*);
  return ((extras_t)fn_extras_)(dev_ctx_, n, ns, cnt.data(), dom.data(), zc.data(), ni, img.data()) == 0;
}

Reason Engine::candidate_reason(const PodReq& req, const Node& n) const {
  if ((filters_ & F_NODE_NAME) && req.node_name > 0 && strings_[req.node_name] != n.name) return RS_NODE_NAME;
  if ((filters_ & F_NODE_AFFINITY) && !affinity_ok(req, n)) return RS_AFFINITY;
  if ((filters_ & F_TAINT_TOLERATION) && !taints_ok(req, n)) return RS_TAINT;
  return RS_OK;
}

void Engine::make_dev_req(const PodReq& req, yoda_dev_req_t* out, const BatchCols::PodCols* pc,
                          const BatchCols* cols) {
  yoda_dev_req_t& d = *out;
  d = yoda_dev_req_t{};
  d.spread_slot = -1;
  d.img_slot = -1;
  if (pc) {
    d.img_slot = pc->image;
    d.spread_slot = pc->spread;
    d.spread_w = (int32_t)score_w_[S_SPREAD];
    d.spread_nc = pc->nc;
    for (int c = 0; c < 2; ++c) {
      d.ckind[c] = pc->ckind[c];
      d.cskew[c] = pc->skew[c];
    }
    // which slots' selectors this pod counts for once assumed (upstream countPodsMatchSelector:
    // same namespace, not terminating)
    for (size_t k = 0; k < cols->spread.size(); ++k) {
      const BatchCols::Spread& sp = cols->spread[k];
      if (sp.ns == req.ns && !req.deleting && sp.sel.matches(req.labels)) d.match_mask |= (uint8_t)(1u << k);
    }
  }
  d.number = req.has_number ? req.number : 1;
  d.memory = req.has_memory ? req.memory : 0;
  d.clock = req.has_clock ? req.clock : 0;
  d.clock_min = req.clock_min;
  d.cpu_m = req.cpu_m;
  d.mem = req.mem;
  d.nz_cpu_m = req.nz_cpu_m;
  d.nz_mem = req.nz_mem;
  d.has_number = req.has_number;
  d.has_memory = req.has_memory;
  d.has_clock = req.has_clock;
  d.binpack = wt_.gpu_binpack;
  d.filters = filters_;
  d.w_yoda = score_w_[S_YODA];
  d.w_least = score_w_[S_LEAST_ALLOCATED];
  d.w_balanced = score_w_[S_BALANCED_ALLOCATION];
  d.w_most = score_w_[S_MOST_ALLOCATED];
  // no PreferNoSchedule taints anywhere: TaintToleration normalises every node to 100
  d.w_const = score_w_[S_TAINT_TOLERATION] * kMaxNodeScore;
  // NodePreferAvoidPods scores every node 100 for a device-eligible pod (device_eligible), and
  // ImageLocality scores every node alike (image_score_const)
  d.w_const += score_w_[S_PREFER_AVOID] * kMaxNodeScore;
  int64_t img = 0;
  if (d.img_slot < 0 && image_score_const(req, &img)) d.w_const += img;   // (a slot: the column)
  d.ext = ((filters_ & F_NODE_RESOURCES_FIT) && ext_checked(dev_ext_res_)) ? ext_amount(req.ext, dev_ext_res_) : 0;
  d.w_link = wt_.w_link;
  d.w_numa = wt_.w_numa;
  d.w_fit = wt_.w_fit;
  d.w_occ = wt_.w_occ;
  d.w_gang_score = wt_.w_gang_score;
  d.w_minlink = wt_.w_minlink;
  Taint ut{unsched_key_, 0, kNoSchedule};
  for (const Toleration& x : req.tolerations)
    if (tolerates(x, ut)) d.tolerates_unschedulable = 1;
  // random tie-break: bijective p(i) = (i*mul + add) mod 2^24 and its inverse
  uint32_t mul = (uint32_t)(rng_() | 1u) & 0xFFFFFFu, add = (uint32_t)rng_() & 0xFFFFFFu;
  uint32_t inv = mul;   // Newton: inv = inv * (2 - mul*inv), 5 steps reach 2^24
  for (int i = 0; i < 5; ++i) inv *= 2u - mul * inv;
  d.perm_mul = mul;
  d.perm_add = add;
  d.perm_inv = inv & 0xFFFFFFu;
}

bool Engine::needs_candidates(const PodReq& req) const {
  return ((filters_ & F_NODE_NAME) && req.node_name > 0) ||
         ((filters_ & F_NODE_AFFINITY) && (!req.node_selector.empty() || !req.required_terms.empty())) ||
         ((filters_ & F_TAINT_TOLERATION) && hard_taint_nodes_ > 0);
}

void Engine::fill_result(const yoda_dev_result_t& res, CycleResult* r) const {
  r->node = res.node;
  r->feasible = res.feasible;
  r->evaluated = live_;
  r->score = res.score;
  r->reason_counts.assign(RS_NUM, 0);
  for (int i = 1; i < RS_NUM && i < YODA_DEV_REASONS; ++i)
    if (i != RS_DEAD) r->reason_counts[i] = res.reasons[i];
  r->cards.clear();
  r->gang_quality = 10000;
  if (r->node >= 0 && (filters_ & F_YODA)) {
    for (int c = 0; c < YODA_DEV_CARDS; ++c)
      if ((res.mask >> c) & 1u) r->cards.push_back(c);
    r->gang_quality = res.quality;
  }
}

bool Engine::schedule_device(const PodReq& req, CycleResult* r) {
  if (!flush_dirty()) {
    ++dev_fallbacks_;
    return false;
  }
  const std::mt19937_64 rng_before = rng_;
  yoda_dev_req_t d;
  make_dev_req(req, &d);
  std::vector<uint8_t> cand;
  const bool need_cand = needs_candidates(req);
  if (need_cand) {
    cand.assign(nodes_.size(), 0);
    for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i)
      if (nodes_[i].alive) cand[i] = (uint8_t)candidate_reason(req, nodes_[i]);
    d.use_candidates = 1;
  }
  yoda_dev_result_t res{};
  int rc = ((dev_schedule_t)fn_schedule_)(dev_ctx_, (int)nodes_.size(), &d, need_cand ? cand.data() : nullptr, &res);
  if (rc != 0) {
    // the CPU cycle that follows draws the tie-break exactly as if the device was never tried
    rng_ = rng_before;
    ++dev_fallbacks_;
    return false;
  }
  ++dev_cycles_;
  fill_result(res, r);
  return true;
}

bool Engine::schedule_batch_device(const uint64_t* pods, const PodReq* const* reqs, size_t count,
                                   std::vector<CycleResult>* out, const BatchCols* cols) {
  if (!dev_ctx_ || !fn_schedule_batch_ || live_ < dev_min_nodes_ || count < (cols ? 1u : 2u)) return false;
  std::unique_lock<std::mutex> dl(dev_mu_, std::try_to_lock);
  if (!dl.owns_lock()) return false;
  // the device assumes each winner with its reservation counted as pending (Engine::reserve
  // with is_pending true); that holds for every node whose sample is not from the future
  const double t = now();
  for (const Node& n : nodes_)
    if (n.alive && !(t > n.sample_ts - settle_s_)) return false;
  if (!flush_dirty()) {
    ++dev_fallbacks_;
    return false;
  }
  // the run's score columns, staged for this call (false: the device cannot take them)
  if (cols && !stage_cols(*cols, reqs, count)) return false;
  // rng draws happen in make_dev_req, in pod order — the same sequence as per-pod cycles
  const std::mt19937_64 rng_before = rng_;
  std::vector<yoda_dev_req_t> d(count);
  for (size_t i = 0; i < count; ++i) make_dev_req(*reqs[i], &d[i], cols ? &cols->pods[i] : nullptr, cols);
  std::vector<yoda_dev_result_t> res(count);
  using batch_t = int (*)(void*, int, int, const yoda_dev_req_t*, yoda_dev_result_t*);
  void* ctx = dev_ctx_;
  const int n_nodes = (int)nodes_.size();
  // the device works on this snapshot (flushed rows + its own in-batch assumes) with the
  // engine lock dropped: mutations meanwhile (bind confirmations, releases, Scv samples)
  // mark their rows dirty and reach the device with the next flush, exactly as if they had
  // happened after the batch
  removed_in_flight_.clear();
  batch_in_flight_.store(true, std::memory_order_release);
  if (ext_mu_) ext_mu_->unlock();
  const int rc = ((batch_t)fn_schedule_batch_)(ctx, n_nodes, (int)d.size(), d.data(), res.data());
  if (ext_mu_) ext_mu_->lock();
  batch_in_flight_.store(false, std::memory_order_release);
  dl.unlock();
  if (rc != 0) {
    // the device table may hold partial in-batch assumptions: re-upload every row. The CPU
    // path that places the batch instead draws the same tie-breaks a CPU-only engine would
    // (-8: abandoned at the host deadline; -9: the device is still draining an abandoned call)
    rng_ = rng_before;
    ++dev_fallbacks_;
    for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i) mark_dirty(i);
    return false;
  }
  std::vector<int32_t> diverged;   // device assumed, host refused (duplicate pod, node gone): re-upload
  // rows dirtied while the lock was dropped are before this mark and stay dirty
  const size_t mark = dirty_list_.size();
  for (size_t i = 0; i < count; ++i) {
    ++cycles_;
    ++dev_cycles_;
    CycleResult r;
    fill_result(res[i], &r);
    if (r.node >= 0 && std::find(removed_in_flight_.begin(), removed_in_flight_.end(), r.node) !=
                           removed_in_flight_.end()) {
      // the node was deleted (and its slot maybe reused by another node) while the device
      // placed this pod on the old row: never bind it there — the caller retries the pod
      diverged.push_back(r.node);
      r.stale = true;
      r.node = -1;
      r.cards.clear();
    } else if (r.node >= 0) {
      r.node_gen = nodes_[r.node].gen;
      if (!reserve(pods[i], *reqs[i], r.node, r.cards)) diverged.push_back(r.node);
    }
    out->push_back(std::move(r));
  }
  // a row reserve() just dirtied was clean when the batch started and untouched since, and
  // the device applied the same assumes to it (same fields, same arithmetic as reserve()
  // with the reservation pending): both sides hold the same row, no re-upload
  for (size_t k = mark; k < dirty_list_.size(); ++k) dirty_[dirty_list_[k]] = 0;
  dirty_list_.resize(mark);
  for (int32_t i : diverged) mark_dirty(i);
  removed_in_flight_.clear();
  return true;
}

bool Engine::device_flush() {
  if (!dev_ctx_) return true;
  std::unique_lock<std::mutex> dl(dev_mu_, std::try_to_lock);
  if (!dl.owns_lock()) return false;
  return flush_dirty();
}

bool Engine::device_cycle(const PodReq& req, CycleResult* out) {
  if (!device_eligible(req)) return false;
  std::unique_lock<std::mutex> dl(dev_mu_, std::try_to_lock);
  if (!dl.owns_lock()) return false;
  return schedule_device(req, out);
}

}  // namespace yoda
