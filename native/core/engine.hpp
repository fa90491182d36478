// Native placement + scheduling-cycle engine for the yoda scheduler.
//
// Holds the cluster as struct-of-arrays-ish node records (k8s node facts + sniffed
// MI355X cards + the scheduler's per-GPU HBM reservation ledger) and runs the whole
// hot loop of a scheduling cycle natively: Filter (yoda + the upstream default
// filters that matter for GPU pods) → PreScore (cluster maxima, SURVEY Q1 fix) →
// Score (yoda formula, compat or fixed) → NormalizeScore → weighted sum →
// selectHost → Reserve (k-subset xGMI-aware gang selection on the chosen node).
//
// Reference parity: pkg/yoda/filter/filter.go:11-58, pkg/yoda/score/algorithm.go:28-87,
// pkg/yoda/collection/collection.go:30-78, pkg/yoda/scheduler.go:76-157 (see
// yoda_scheduler_amd/plugins/yoda_policy.py for the executable Python spec).
#pragma once

#include "yoda_dev_abi.h"
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <memory>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace yoda {

constexpr int64_t kMaxNodeScore = 100;
constexpr int kMaxPhys = 64;

enum TaintEffect : int8_t { kNoSchedule = 0, kPreferNoSchedule = 1, kNoExecute = 2, kEffectAny = 3 };
enum TolOp : int8_t { kTolEqual = 0, kTolExists = 1 };
enum SelOp : int8_t { kIn = 0, kNotIn = 1, kExists = 2, kDoesNotExist = 3, kGt = 4, kLt = 5 };

// Plugin bits for the native filter / score sets.
enum FilterBit : uint32_t {
  F_NODE_UNSCHEDULABLE = 1u << 0,
  F_NODE_NAME = 1u << 1,
  F_TAINT_TOLERATION = 1u << 2,
  F_NODE_AFFINITY = 1u << 3,
  F_NODE_RESOURCES_FIT = 1u << 4,
  F_YODA = 1u << 5,
  F_SPREAD = 1u << 6,          // PodTopologySpread DoNotSchedule constraints (explicit or profile defaults)
  F_INTERPOD = 1u << 7,        // InterPodAffinity: required (anti-)affinity, existing pods' anti-affinity
  F_NODE_PORTS = 1u << 8,      // NodePorts: host ports of the pods the ledger holds on the node
};
enum ScoreIdx : int {
  S_YODA = 0,
  S_LEAST_ALLOCATED = 1,
  S_BALANCED_ALLOCATION = 2,
  S_TAINT_TOLERATION = 3,
  S_NODE_AFFINITY = 4,
  S_MOST_ALLOCATED = 5,
  S_IMAGE_LOCALITY = 6,
  S_PREFER_AVOID = 7,          // NodePreferAvoidPods
  S_SPREAD = 8,                // PodTopologySpread ScheduleAnyway constraints (explicit or profile defaults)
  S_INTERPOD = 9,              // InterPodAffinity: preferred terms both ways + hardPodAffinityWeight
  S_NUM = 10,
};

// Why a node was rejected (first failing plugin), reported for FitError diagnosis.
enum Reason : int8_t {
  RS_OK = 0, RS_UNSCHEDULABLE, RS_NODE_NAME, RS_TAINT, RS_AFFINITY, RS_RESOURCES, RS_NO_SCV,
  RS_STALE, RS_GPU_NUMBER, RS_GPU_MEMORY, RS_GPU_CLOCK, RS_GPU_FIT, RS_DEAD,
  RS_EXT_RESOURCES,            // NodeResourcesFit: a resource beyond cpu/memory/pods
  RS_SPREAD,                   // PodTopologySpread: skew
  RS_SPREAD_LABEL,             // PodTopologySpread: the node lacks a constraint's topology key
  RS_EXISTING_ANTI,            // InterPodAffinity: an existing pod's required anti-affinity
  RS_POD_AFFINITY,             // InterPodAffinity: the pod's required affinity
  RS_POD_ANTI,                 // InterPodAffinity: the pod's required anti-affinity
  RS_NODE_PORTS,               // NodePorts: a requested host port is taken
  RS_VOLUME_NODE,              // VolumeBinding: a bound PV's node affinity rejects the node
  RS_VOLUME_ZONE,              // VolumeZone: a bound PV's zone / region labels reject the node
  RS_VOLUME_LIMITS,            // NodeVolumeLimits: a CSI driver's attach limit would be exceeded
  RS_NUM
};

struct Card {
  uint64_t total_mb = 0, free_mb = 0;
  uint64_t clock = 0, bandwidth = 0, core = 0, power = 0;
  bool healthy = true;
  int32_t phys = 0;
  int32_t numa = 0;
  int32_t occ_q = 0;          // CU occupancy in 1e-4 units (0..10000)
  uint64_t reserved_mb = 0;   // ledger: HBM reserved by assumed/bound pods
  uint64_t pending_mb = 0;    // part of reserved_mb the last sample cannot reflect yet
  int32_t pods = 0;           // pods holding a reservation on this card
};

struct Taint { int32_t key, value; int8_t effect; };
struct Toleration { int32_t key; int32_t value; int8_t op; int8_t effect; };  // key -1 = any
struct SelReq {
  int32_t key;
  int8_t op;
  std::vector<int32_t> values;
  int64_t num;
  bool operator==(const SelReq& o) const { return key == o.key && op == o.op && values == o.values && num == o.num; }
};
struct SelTerm {
  std::vector<SelReq> reqs;
  bool operator==(const SelTerm& o) const { return reqs == o.reqs; }
};
struct PrefTerm { int32_t weight; SelTerm term; };

// Interned (key, value) pairs sorted by key: a pod's labels as the ledger keeps them.
using Labels = std::vector<std::pair<int32_t, int32_t>>;

// metav1.LabelSelector over interned strings (models/selectors.py::LabelSelector): every
// requirement must hold — matchLabels k=v become In {v}, matchExpressions In/NotIn/Exists/
// DoesNotExist keep their SelOp — and a nil selector (`nothing`) matches no pod.
struct LReq {
  int32_t key;
  int8_t op;
  std::vector<int32_t> values;
  bool operator==(const LReq& o) const { return key == o.key && op == o.op && values == o.values; }
};
struct LSel {
  bool nothing = false;
  std::vector<LReq> reqs;
  bool empty() const { return !nothing && reqs.empty(); }
  bool matches(const Labels& l) const;
  bool operator==(const LSel& o) const { return nothing == o.nothing && reqs == o.reqs; }
};

// One topology spread constraint (upstream v1.20 podtopologyspread; plugins/spread_affinity.py).
struct SpreadC {
  int32_t key = 0;             // interned topologyKey
  int32_t max_skew = 1;
  bool hard = true;            // DoNotSchedule (filter) vs ScheduleAnyway (score)
  LSel sel;
};
// One pod (anti-)affinity term (plugins/spread_affinity.py InterPodAffinity): topology key, the
// namespaces it selects pods in (the owner's own when the term lists none) and the selector
struct PodTerm {
  int32_t key = 0;
  std::vector<int32_t> ns;
  LSel sel;
  int32_t weight = 1;          // preferred terms
  bool matches(int32_t pod_ns, const Labels& l) const {
    return std::find(ns.begin(), ns.end(), pod_ns) != ns.end() && sel.matches(l);
  }
  bool operator==(const PodTerm& o) const { return key == o.key && ns == o.ns && sel == o.sel && weight == o.weight; }
};
// A pod's inter-pod affinity (shared by its request and its ledger entry)
struct PodAffinity {
  std::vector<PodTerm> req_aff, req_anti, pref_aff, pref_anti;
  bool empty() const { return req_aff.empty() && req_anti.empty() && pref_aff.empty() && pref_anti.empty(); }
  bool operator==(const PodAffinity& o) const {
    return req_aff == o.req_aff && req_anti == o.req_anti && pref_aff == o.pref_aff && pref_anti == o.pref_anti;
  }
  uint64_t hash() const;
};
// The reserved pods that carry one (anti-)affinity term set (pods of one template carry equal
// terms), and how many of them each node holds: the symmetric checks of a new pod (existing
// pods' required anti-affinity, their required / preferred terms in scoring) run once per set
// and node, weighted by that count, instead of once per holder pod
struct AffSet {
  std::shared_ptr<const PodAffinity> aff;          // a representative (content-equal for every holder)
  std::unordered_map<int32_t, int32_t> nodes;      // node index → holders there
  int64_t pods = 0;
};

// A profile's default constraint (PodTopologySpread args: System defaults or a List); its
// selector is the pod's DefaultSelector (Services + controller)
struct DefaultSpread {
  int32_t key = 0;
  int32_t max_skew = 1;
  bool hard = false;
};

// (namespace, label key, label value) of the pods on a node; key = value = -1: the namespace alone
struct LKey {
  int32_t ns, k, v;
  bool operator==(const LKey& o) const { return ns == o.ns && k == o.k && v == o.v; }
};
struct LKeyHash {
  size_t operator()(const LKey& x) const {
    return (size_t)(((uint64_t)(uint32_t)x.ns * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)(uint32_t)x.k * 0xC2B2AE3D27D4EB4Full) ^
                    ((uint64_t)(uint32_t)x.v * 0x165667B19E3779F9ull));
  }
};

// A reserved pod's (namespace, sorted labels), interned once by the engine (Engine::labset_acquire):
// the ledger entry holds its id and a node's label-set groups count pods per id, so reserving or
// releasing a pod of a known template copies no labels and allocates nothing
struct LabSetRec {
  int32_t ns = 0;
  Labels labels;
  uint64_t hash = 0;
  int64_t refs = 0;            // ledger entries holding it; 0: idle (kept for reuse until a sweep)
  int32_t next = -1;           // the next id in its hash chain (labset_by_hash_)
  bool used = false;           // false: on the free list
};
uint64_t labset_hash(int32_t ns, const Labels& l);

// Open-addressing map uint64 → int32 (linear probing, backward-shift deletion): the ledger's
// pod → slab index. Inserting a key into a table below its load limit and erasing one never
// allocate, so a steady reserve / release cycle does not touch the heap.
class U64Map {
 public:
  int32_t find(uint64_t k) const {
    if (cap_ == 0) return -1;
    for (size_t i = slot(k);; i = (i + 1) & (cap_ - 1)) {
      if (!used_[i]) return -1;
      if (keys_[i] == k) return vals_[i];
    }
  }
  bool insert(uint64_t k, int32_t v);   // false if present
  bool erase(uint64_t k);
  size_t size() const { return size_; }

 private:
  size_t slot(uint64_t k) const {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    return (size_t)k & (cap_ - 1);
  }
  void grow();
  std::vector<uint64_t> keys_;
  std::vector<int32_t> vals_;
  std::vector<uint8_t> used_;
  size_t cap_ = 0, size_ = 0;
};

// NodePorts: a container port with hostPort > 0, sanitized as upstream HostPortInfo (hostIP ""
// → "0.0.0.0", protocol "" → "TCP"); hostIP and protocol interned
struct HostPort {
  int32_t ip = 0, proto = 0, port = 0;
  bool operator<(const HostPort& o) const {
    return ip != o.ip ? ip < o.ip : proto != o.proto ? proto < o.proto : port < o.port;
  }
  bool operator==(const HostPort& o) const { return ip == o.ip && proto == o.proto && port == o.port; }
};

struct Node {
  std::string name;
  uint32_t gen = 0;                   // slot generation: bumped when the slot gets a new node or dies
  bool alive = true;
  bool unschedulable = false;
  bool has_scv = false;
  bool stale = false;
  std::vector<Card> cards;
  uint64_t card_number = 0, free_sum = 0, total_sum = 0;   // Scv.Status (sniffed)
  int32_t nphys = 0;
  std::vector<int32_t> link_q;        // nphys*nphys pair quality, 10000 = idle healthy link
  std::unordered_map<int32_t, int32_t> labels;   // interned key → interned value
  std::vector<Taint> taints;
  int64_t alloc_cpu_m = 0, alloc_mem = 0, alloc_pods = 0;
  int64_t req_cpu_m = 0, req_mem = 0, pod_count = 0;
  int64_t nz_cpu_m = 0, nz_mem = 0;     // Σ non-zero requests (upstream NodeInfo.NonZeroRequested)
  uint64_t label_mem_sum = 0;         // Σ scv/memory labels of pods on node (compat Allocate)
  bool hard_taint = false, prefer_taint = false;   // has NoSchedule/NoExecute, PreferNoSchedule taints
  double sample_ts = 0;               // unix time of the Scv sample the cards came from
  std::vector<int32_t> pods;          // ledger slab indices of the pods on this node
  std::vector<std::pair<int32_t, int64_t>> images;     // status.images: (normalized name, bytes), sorted
  std::vector<std::pair<int32_t, int64_t>> ext_alloc;  // allocatable beyond cpu/memory/pods, sorted
  std::vector<std::pair<int32_t, int64_t>> ext_used;   // Σ of the ledger's ext requests, sorted
  std::vector<std::pair<int8_t, int32_t>> avoid;       // preferAvoidPods controllers (kind 1 RC / 2 RS, uid)
  // label index of the reserved pods: (all, not terminating) per (namespace, key, value) and per
  // namespace — a single-label selector's count in O(1) (spread / affinity pre-filters)
  std::unordered_map<LKey, std::pair<int32_t, int32_t>, LKeyHash> lab_idx;
  // the same pods grouped by their exact (namespace, label set) — an interned label-set id — with
  // (all, not terminating) counts: any other selector is matched once per group instead of once
  // per pod (a node's pods come from few templates)
  struct LabGroup {
    int32_t all = 0, live = 0;
    // the group's label-index entries (its namespace's, then one per label): bumped through these
    // pointers (unordered_map references are stable), rebound when the group's count is 0 — a
    // fresh group, or an id the label-set table recycled for another set
    std::vector<std::pair<int32_t, int32_t>*> idx;
  };
  std::unordered_map<int32_t, LabGroup> lab_groups;
  // entries of lab_idx / lab_groups whose count dropped to 0: kept, so a pod of the same template
  // arriving again allocates nothing; swept once they outnumber the live entries
  int32_t lab_idx_zero = 0, lab_groups_zero = 0;
  // NodePorts: host ports of the reserved pods, per (ip, protocol, port) and per (protocol, port)
  // over every ip (a 0.0.0.0 request conflicts with any ip) — counts, as two pods may hold one
  std::map<HostPort, int32_t> ports;
  std::map<std::pair<int32_t, int32_t>, int32_t> ports_any;
  // NodeVolumeLimits: CSI attach limits (driver → count, sorted) and the PVC claims the node's
  // reserved pods mount (claim → pods); a claim's volume is looked up when counting
  std::vector<std::pair<int32_t, int64_t>> vol_limits;
  std::unordered_map<int32_t, int32_t> claims;
};

struct PodReq {
  // scv labels (Go semantics already applied by the caller's parser)
  bool has_number = false, has_memory = false, has_clock = false;
  uint64_t number = 1, memory = 0, clock = 0, clock_min = 0;
  int64_t priority = 0;                  // scv/priority (yoda QueueSort)
  int64_t pod_priority = 0;              // spec.priority (PriorityClass: DefaultPreemption)
  // k8s spec
  int32_t node_name = -1;                // interned spec.nodeName, -1 = none
  int64_t cpu_m = 0, mem = 0;
  int64_t nz_cpu_m = 100, nz_mem = 200LL * 1024 * 1024;   // per-container non-zero defaults applied
  std::vector<std::pair<int32_t, int32_t>> node_selector;
  std::vector<SelTerm> required_terms;   // ORed
  std::vector<PrefTerm> preferred_terms;
  std::vector<Toleration> tolerations;
  // what other pods' spread constraints read of this pod once it holds a reservation (the
  // ledger keeps them): namespace, labels, terminating
  int32_t ns = 0;
  Labels labels;
  bool deleting = false;
  // ImageLocality: normalized images of spec.containers (interned), and their count
  std::vector<int32_t> images;
  int32_t containers = 0;
  // NodeResourcesFit beyond cpu / memory / pods (ephemeral-storage, hugepages-*, amd.com/gpu,
  // other extended resources): (interned resource name, amount), sorted by name
  std::vector<std::pair<int32_t, int64_t>> ext;
  // controllerRef for DefaultSelector (1 v1 ReplicationController, 2 apps/v1 ReplicaSet,
  // 3 apps/v1 StatefulSet; 0 none / another kind) and for NodePreferAvoidPods (the first
  // controller of kind ReplicationController (1) or ReplicaSet (2), any apiVersion, by uid)
  int8_t owner_kind = 0;
  int32_t owner_name = -1;
  int8_t avoid_kind = 0;
  int32_t avoid_uid = -1;
  // PodTopologySpread: spec.topologySpreadConstraints (when non-empty the profile's default
  // constraints do not apply, even for an action none of them has)
  bool spread_explicit = false;
  std::vector<SpreadC> spread;
  // InterPodAffinity: the pod's (anti-)affinity terms (null: none)
  std::shared_ptr<const PodAffinity> aff;
  // NodePorts: its containers' host ports (hostPort > 0), sanitized
  std::vector<HostPort> host_ports;
  // VolumeBinding / VolumeZone for claims bound to PVs with node affinity / zone labels (the
  // native lane's claim table): each entry's terms are OR'ed, every entry must hold; the
  // reason says which plugin rejects a node
  struct VolTerms {
    std::shared_ptr<const std::vector<SelTerm>> terms;
    int8_t reason = RS_VOLUME_NODE;
  };
  std::vector<VolTerms> vol;
  // NodeVolumeLimits: the "namespace/claim" of its persistentVolumeClaim volumes (interned; what
  // the ledger keeps per node), and whether this cycle counts them against the node's limits
  std::vector<int32_t> pvc_claims;
  bool count_vols = false;
};

struct Weights {
  // gang / GPU-level selection objective (lower is better), see gang_objective()
  int64_t w_link = 4, w_numa = 2, w_fit = 1, w_occ = 1;
  // bottleneck term: a ring all-reduce over the set is bound by its slowest xGMI link, so the
  // worst pair counts on top of the mean (minlink_bad = (10000 − min pair q) · 100)
  int64_t w_minlink = 2;
  bool gpu_binpack = false;     // false: worst-fit (spread, default); true: best-fit within node
  int64_t w_gang_score = 3;     // node score bonus × xGMI quality for multi-GPU pods (fixed mode)
  int64_t enum_limit = 5000;    // exhaustive k-subset search up to this many subsets
};

// The node as the yoda filter sees it (Engine::filter_view)
struct FilterView {
  struct C {
    bool healthy;
    uint64_t free, eff_free, clock;
  };
  bool known = false, has_scv = false, stale = false;
  uint64_t card_number = 0;
  std::vector<C> cards;
};

struct Assignment {
  int32_t node = -1;
  std::vector<int32_t> cards;
  uint64_t mb = 0;              // per card
  int64_t cpu_m = 0, mem = 0;
  int64_t nz_cpu_m = 0, nz_mem = 0;
  uint64_t label_mem = 0;
  bool has_label_mem = false;
  double t_res = 0;             // unix time of the reservation
  int32_t slot = -1;            // index in Node::pods
  uint64_t pod = 0;             // the ledger key (the slab entry is free when !live)
  bool live = false;
  int32_t ns = 0;               // the pod as other pods' spread constraints count it
  int32_t labset = -1;          // its interned (namespace, labels) (Engine::labset)
  bool deleting = false;
  std::vector<std::pair<int32_t, int64_t>> ext;   // extended resources it holds on the node
  std::shared_ptr<const PodAffinity> aff;          // its (anti-)affinity terms (symmetric rule, scoring)
  uint64_t aff_hash = 0;                           // its AffSet's bucket (aff_sets_)
  std::vector<HostPort> host_ports;                // NodePorts: the host ports it holds on the node
  std::vector<int32_t> pvc_claims;                 // NodeVolumeLimits: the PVC claims it mounts
  int64_t prio = 0;                                // spec.priority (DefaultPreemption)
  bool detached = false;                           // off its node for a what-if (detach_pod)
};

// DefaultPreemption (upstream v1.20 preemption: FindCandidates → SelectCandidate) on the ledger.
// A PodDisruptionBudget as selectVictimsOnNode reads it: namespace, selector (empty / nil
// selects nothing), status.disruptionsAllowed
struct Pdb {
  int32_t ns = 0;
  LSel sel;
  int64_t allowed = 0;
};
struct PreemptArgs {
  int64_t priority = 0;                 // the preemptor's spec.priority
  std::vector<Pdb> pdbs;
  int32_t min_pct = 10, min_abs = 100;  // DefaultPreemptionArgs minCandidateNodes{Percentage,Absolute}
  int64_t offset = -1;                  // dry-run start in the potential nodes; <0: the engine's rng
};
struct PreemptResult {
  int32_t node = -1;                    // nominated node, -1: no candidate
  std::vector<uint64_t> victims;        // ledger pod ids to evict
  std::vector<int32_t> cards;           // the GPUs the preemptor takes once they are gone
  int32_t violations = 0;               // PDB violations of the chosen victims
  int32_t potential = 0;                // nodes where preemption might help (resolvable status)
  int32_t evaluated = 0;                // nodes dry-run before the candidate quota was met
  int32_t candidates = 0;
};

struct CycleResult {
  int32_t node = -1;                 // selected node, -1 = unschedulable
  uint32_t node_gen = 0;             // generation of that node's slot when it was selected
  bool stale = false;                // the node was removed / its slot reused while the device placed it
  int32_t feasible = 0;
  int32_t evaluated = 0;
  std::vector<int32_t> cards;        // GPU assignment on the selected node
  int64_t score = 0;
  std::vector<int32_t> reason_counts;  // RS_NUM histogram over rejected nodes
  int32_t gang_quality = 0;          // 0..10000
};

class ThreadPool {
 public:
  explicit ThreadPool(int n);
  ~ThreadPool();
  // Runs fn(begin, end) over [0, n) in chunks across workers (+ the caller).
  void parallel_for(int n, int grain, const std::function<void(int, int)>& fn);
  int size() const { return (int)workers_.size() + 1; }

 private:
  void worker();
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int, int)>* job_ = nullptr;
  int job_n_ = 0, job_grain_ = 1;
  std::atomic<int> next_{0};
  int active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Everything a profile configures on the engine (Framework.apply): the native lane keeps one
// per profile and swaps it in around its batches, restoring the caller's afterwards.
struct EngineConfig {
  uint32_t filters = 0;
  int64_t score_w[S_NUM] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int64_t alloc_w[2][3] = {{1, 1, 0}, {1, 1, 0}};
  Weights wt;
  double settle_s = 30.0;
  std::vector<DefaultSpread> spread_defaults;   // PodTopologySpread default constraints
  std::vector<int32_t> ext_ignored;             // NodeResourcesFit ignoredResources
  std::vector<std::string> ext_ignored_groups;  // NodeResourcesFit ignoredResourceGroups
  int64_t hard_pod_affinity_weight = 1;         // InterPodAffinity args
};

class Engine {
 public:
  Engine(bool compat, int threads);
  ~Engine();

  EngineConfig config() const;
  void set_config(const EngineConfig& c);

  // ---- configuration
  bool compat() const { return compat_; }
  void set_compat(bool c) { compat_ = c; }
  void set_filters(uint32_t mask) { filters_ = mask; }
  uint32_t filters() const { return filters_; }
  void set_score_weight(int idx, int64_t w) { score_w_[idx] = w; }
  // Least/MostAllocated `resources` weights (args): cpu, memory, and the summed weight of
  // resources this engine does not track (they score 0 upstream but count in the divisor)
  void set_alloc_weights(bool most, int64_t cpu, int64_t mem, int64_t other) {
    alloc_w_[most ? 1 : 0][0] = cpu;
    alloc_w_[most ? 1 : 0][1] = mem;
    alloc_w_[most ? 1 : 0][2] = other;
  }
  bool default_alloc_weights() const {
    for (int k = 0; k < 2; ++k)
      if (alloc_w_[k][0] != 1 || alloc_w_[k][1] != 1 || alloc_w_[k][2] != 0) return false;
    return true;
  }
  int64_t score_weight(int idx) const { return score_w_[idx]; }
  Weights& weights() { return wt_; }
  void set_percentage_of_nodes_to_score(int p) { pct_nodes_ = p; }
  int32_t num_feasible_to_find(int32_t all) const;   // upstream numFeasibleNodesToFind
  void seed(uint64_t s) { rng_.seed(s); }
  int32_t intern(const std::string& s);
  const std::string& str(int32_t id) const { return strings_[id]; }
  // NodePorts: one requested host port as upstream HostPortInfo keeps it; false for port <= 0
  // (not a host port: never conflicts)
  bool host_port(int64_t port, const std::string& protocol, const std::string& ip, HostPort* out);
  bool ports_free(const PodReq& req, const Node& n) const;
  // NodeVolumeLimits: a claim's volume — (CSI driver, unique volume id) of its bound CSI PV, or
  // (provisioner, "<provisioner>/<namespace>/<claim>") while a provisioning StorageClass binds
  // it; claims without one are absent (plugins/volumes.py::claim_volume)
  void set_claim_volume(int32_t claim, int32_t driver, int32_t handle) { claim_vol_[claim] = {driver, handle}; }
  void clear_claim_volume(int32_t claim) { claim_vol_.erase(claim); }
  void set_node_vol_limits(int32_t idx, std::vector<std::pair<int32_t, int64_t>> limits);
  bool vols_fit(const PodReq& req, const Node& n) const;

  // ---- cluster state
  int32_t upsert_node(const std::string& name);      // returns index (stable)
  int32_t node_index(const std::string& name) const;
  void remove_node(int32_t idx);
  Node& node(int32_t idx) { return nodes_[idx]; }
  const Node& node(int32_t idx) const { return nodes_[idx]; }
  int32_t num_nodes() const { return (int32_t)nodes_.size(); }
  uint32_t node_gen(int32_t idx) const {
    return idx >= 0 && idx < (int32_t)nodes_.size() ? nodes_[idx].gen : 0;
  }
  int32_t live_nodes() const { return live_; }
  // sample_ts: when the Scv sample was taken (unix s). Reservations younger than
  // sample_ts − settle are "pending": the sample cannot contain their HBM use yet, so
  // they are subtracted from the sampled free memory (never double-counted: see eff_free).
  void set_cards(int32_t idx, std::vector<Card> cards, uint64_t card_number, uint64_t free_sum,
                 uint64_t total_sum, bool stale, double sample_ts = 0);
  void set_settle_seconds(double s) { settle_s_ = s; }
  double settle_seconds() const { return settle_s_; }
  // test hook: pin the reservation clock (unix s); <0 = use the system clock
  void set_fixed_now(double t) { fixed_now_ = t; }
  void clear_scv(int32_t idx);
  void set_links(int32_t idx, int32_t nphys, std::vector<int32_t> q);

  // ---- ledger
  bool reserve(uint64_t pod, const PodReq& req, int32_t node, const std::vector<int32_t>& cards);
  bool release(uint64_t pod);
  bool has_pod(uint64_t pod) const { return ledger_.find(pod) >= 0; }
  const Assignment* assignment(uint64_t pod) const;
  size_t ledger_size() const { return ledger_.size(); }
  // the (namespace, labels) of an interned label set (Assignment::labset)
  const LabSetRec& labset(int32_t id) const { return labsets_[id]; }
  size_t labsets_used() const { return labsets_.size() - labset_free_.size(); }

  // ---- policy pieces (exposed for parity tests and for the Python runner)
  Reason filter_node(const PodReq& req, int32_t idx, uint64_t* n, uint64_t* m, uint64_t* c) const;
  Reason yoda_filter(const PodReq& req, int32_t idx, uint64_t* n, uint64_t* m, uint64_t* c) const;
  void collect_max(const PodReq& req, const std::vector<int32_t>& nodes, uint64_t mx[6]) const;
  uint64_t yoda_raw_score(const PodReq& req, int32_t idx, const uint64_t mx[6]) const;
  static void normalize_yoda(std::vector<int64_t>& s);
  // GPU set on node (empty + false if none)
  bool select_gpus(const PodReq& req, int32_t idx, std::vector<int32_t>* out, int32_t* quality) const;
  FilterView filter_view(int32_t idx) const;
  bool select_gpus_small(const Node& n, const std::vector<int32_t>& E, uint64_t k, uint64_t m,
                         std::vector<int32_t>* out, int32_t* quality) const;

  // ---- DefaultPreemption: the pod failed on every node; find the node where evicting the
  // fewest / least important lower-priority pods lets it fit. The ledger is restored exactly.
  bool preempt(const PodReq& req, const PreemptArgs& args, PreemptResult* out);
  std::vector<int32_t> preempt_potential(const PodReq& req) const;
  // the node's first failing filter in upstream v1.20 plugin order is not
  // UnschedulableAndUnresolvable (nodesWherePreemptionMightHelp); a node that passes counts too
  bool preemption_might_help(const PodReq& req, int32_t idx) const;
  // what-if helpers for the Python spec of preemption: a ledger entry's effect on its node off /
  // back on, the entry (and its reservation time) kept; false if the pod is unknown or already so
  bool detach_pod(uint64_t pod);
  bool attach_pod(uint64_t pod);

  // ---- full native cycle
  // candidates: node indices to consider (empty = all). Python filter/score plugins can
  // pre-restrict candidates and add extra per-node scores (extra_scores aligned with
  // candidates, already weighted), so the native fast path and the hybrid runner share
  // one implementation.
  CycleResult schedule(uint64_t pod, const PodReq& req, bool assume,
                       const std::vector<int32_t>& candidates,
                       const std::vector<int64_t>& extra_scores);

  // Batch: schedule pods in order, each seeing the previous ones' reservations.
  std::vector<CycleResult> schedule_batch(const std::vector<uint64_t>& pods,
                                          const std::vector<const PodReq*>& reqs);

  // Filter only → feasible node indices (for the hybrid runner)
  // exhaustive: ignore percentageOfNodesToScore (the caller applies further filters and
  // does its own early exit, so the sample must be taken over nodes passing ALL filters)
  std::vector<int32_t> feasible_nodes(const PodReq& req, const std::vector<int32_t>& candidates,
                                      std::vector<int32_t>* reasons, bool exhaustive = false);
  // Native weighted score of the given feasible nodes (normalized per plugin, summed).
  std::vector<int64_t> score_nodes(const PodReq& req, const std::vector<int32_t>& feasible);

  uint64_t cycles() const { return cycles_; }

  // ---- k8s node facts (keeps the taint census the device path needs)
  void set_node_meta(int32_t idx, bool unschedulable, const std::vector<std::pair<int32_t, int32_t>>& labels,
                     const std::vector<Taint>& taints, int64_t cpu_m, int64_t mem, int64_t pods);
  // status.images (ImageLocality), allocatable beyond cpu/memory/pods (NodeResourcesFit) and the
  // preferAvoidPods annotation's controllers (NodePreferAvoidPods); each list sorted by key
  void set_node_extras(int32_t idx, std::vector<std::pair<int32_t, int64_t>> images,
                       std::vector<std::pair<int32_t, int64_t>> ext_alloc,
                       std::vector<std::pair<int8_t, int32_t>> avoid);
  int32_t image_nodes(int32_t image) const;          // nodes reporting the image
  int32_t avoid_nodes() const { return avoid_nodes_; }

  // ---- DefaultSelector sources (upstream helper.DefaultSelector: Services selecting the pod,
  // its ReplicationController's map selector, its ReplicaSet's / StatefulSet's LabelSelector)
  void set_service(int32_t ns, int32_t name, bool nil_selector, Labels selector);
  void remove_service(int32_t ns, int32_t name);
  // kind 1 RC (the map as In requirements), 2 RS, 3 STS
  void set_controller(int8_t kind, int32_t ns, int32_t name, LSel sel);
  void remove_controller(int8_t kind, int32_t ns, int32_t name);
  // the pod's DefaultSelector; false when it is empty (no default constraints apply)
  bool default_selector(const PodReq& req, LSel* out) const;
  // the pod's constraints of one action (explicit ones, else the profile defaults with the
  // DefaultSelector); empty when the pod has none
  void spread_constraints(const PodReq& req, bool hard, std::vector<SpreadC>* out) const;
  // a reserved pod's labels or deletionTimestamp changed (spread counts read them)
  bool set_pod_meta(uint64_t pod, Labels labels, bool deleting);
  // pods on node idx holding a reservation, in namespace ns, not terminating, matching sel
  int64_t count_matching(int32_t idx, int32_t ns, const LSel& sel) const;

  // ---- InterPodAffinity pieces (exposed for parity tests)
  struct InterPodPF {
    bool active = false;
    std::unordered_map<int32_t, std::unordered_set<int32_t>> existing_anti;   // key → blocked values
    std::unordered_map<uint64_t, int64_t> affinity, anti;                      // (key << 32 | value) → pods
    bool any_aff_match = false, self_match = false;
  };
  void interpod_prefilter(const PodReq& req, InterPodPF* pf) const;
  Reason interpod_filter(const PodReq& req, const Node& n, const InterPodPF& pf) const;
  void interpod_scores(const PodReq& req, const std::vector<int32_t>& feas, std::vector<int64_t>& s) const;
  size_t affinity_holders() const { return aff_holders_.size(); }
  void set_hard_pod_affinity_weight(int64_t w) { hard_aff_w_ = w; }

  // ---- profile configuration of the default plugins beyond the score weights
  void set_spread_defaults(std::vector<DefaultSpread> d) { spread_defaults_ = std::move(d); }
  const std::vector<DefaultSpread>& spread_defaults() const { return spread_defaults_; }
  // the one extended resource the device rows carry (default ephemeral-storage): pods whose only
  // checked extended request is this one stay device-eligible
  void set_device_ext_resource(int32_t res) {
    dev_ext_res_ = res;
    for (int32_t i = 0; i < (int32_t)nodes_.size(); ++i) mark_dirty(i);
  }
  int32_t device_ext_resource() const { return dev_ext_res_; }
  void set_ext_ignored(std::vector<int32_t> res, std::vector<std::string> groups) {
    ext_ignored_ = std::move(res);
    ext_ignored_groups_ = std::move(groups);
  }

  // ---- gfx950 device scorer (libyoda_hip.so, loaded with dlopen; see native/hip/scorer.hip)
  // Offloads whole cycles for clusters of >= min_nodes nodes when the pod/profile is
  // representable on the device (fixed mode, <= 8 GPUs per node, ...); otherwise, or on
  // any device error, the CPU path runs. Device cycles score every feasible node (the
  // adaptive percentageOfNodesToScore sampling exists to bound CPU cost).
  bool enable_device(const std::string& lib_path, int device, int capacity, int min_nodes, std::string* err);
  void disable_device();
  bool device_enabled() const { return dev_ctx_ != nullptr; }
  uintptr_t device_ctx() const { return (uintptr_t)dev_ctx_; }   // for yoda_dev_* debug entry points
  // The caller's engine lock (the Python binding's). schedule_batch drops it while the
  // device places the batch, so other engine calls (informer updates, bind confirmations)
  // proceed meanwhile instead of stalling the event loop for the whole batch; the caller
  // must hold it exactly once. Device use itself is serialised by dev_mu_.
  void set_external_lock(std::recursive_mutex* m) { ext_mu_ = m; }
  bool batch_in_flight() const { return batch_in_flight_.load(std::memory_order_acquire); }
  uint64_t device_cycles() const { return dev_cycles_; }
  uint64_t device_batches() const { return dev_batches_; }   // k_batch dispatches that placed pods
  uint64_t device_fallbacks() const { return dev_fallbacks_; }
  float device_last_us() const;
  void device_set_timing(bool on);   // per-cycle event timing (benchmarks)
  // `slots`: for k_batch, whose score columns carry a non-constant ImageLocality term and
  // PodTopologySpread soft constraints (BatchCols); the per-pod kernels carry neither
  bool device_eligible(const PodReq& req, bool slots = false) const;
  // parity hook: run one device cycle without reserving; false if not eligible/failed
  bool device_cycle(const PodReq& req, CycleResult* out);
  // push the rows changed since the last device call to the device now (an idle scheduler
  // does, so the next batch does not carry them); false if the device is busy or refused
  bool device_flush();

 private:
  void mark_dirty(int32_t idx);
  bool pack_node(int32_t idx, void* row) const;   // row: yoda_dev_node_t*
  bool flush_dirty();
  bool schedule_device(const PodReq& req, CycleResult* r);
  // k_batch score columns of one device run: up to YODA_DEV_SPREAD_SLOTS spread slots (pods
  // counted by one selector in one namespace, over one set of topology keys) and
  // YODA_DEV_IMAGE_SLOTS image slots (one image list); per pod its slots and constraints
  struct BatchCols {
    struct Spread {
      int32_t ns = 0;
      LSel sel;
      bool host = false;       // a kubernetes.io/hostname constraint
      int32_t dom_key = -1;    // the other constraint's key (-1: none)
    };
    struct PodCols {
      int8_t spread = -1, image = -1;
      uint8_t nc = 0, ckind[2] = {0, 0};
      int32_t skew[2] = {0, 0};
    };
    std::vector<Spread> spread;
    std::vector<std::pair<std::vector<int32_t>, int32_t>> image;   // (images, containers)
    std::vector<PodCols> pods;
  };
  // one k_batch dispatch for pods[0, count) (all batch_eligible), results appended to *out;
  // false (nothing appended) when the device refuses or fails
  bool schedule_batch_device(const uint64_t* pods, const PodReq* const* reqs, size_t count,
                             std::vector<CycleResult>* out, const BatchCols* cols = nullptr);
  bool batch_eligible(const PodReq& q) const;   // device_eligible (with slots), no per-node candidate mask
  // the pod's slots in `cols` (adding slots as needed); false when it needs one too many or its
  // soft constraints are not representable
  bool assign_cols(const PodReq& q, BatchCols* cols) const;
  // stage the run's columns on the device (fn_extras_); false: the run takes per-pod cycles
  bool stage_cols(const BatchCols& cols, const PodReq* const* reqs, size_t count);
  void make_dev_req(const PodReq& req, yoda_dev_req_t* out, const BatchCols::PodCols* pc = nullptr,
                    const BatchCols* cols = nullptr);
  bool needs_candidates(const PodReq& req) const;
  // PodTopologySpread PreFilter state of one pod's DoNotSchedule constraints (upstream
  // preFilterState): matching pods per (key, value) over the nodes passing the pod's node
  // affinity that carry every key, and the minimum per key
  struct SpreadPF {
    std::vector<SpreadC> cons;
    std::unordered_map<uint64_t, int64_t> pair_counts;   // (key << 32) | value
    std::unordered_map<int32_t, int64_t> min_count;
  };
  void spread_prefilter(const PodReq& req, SpreadPF* pf) const;
  Reason spread_filter(const PodReq& req, const Node& n, const SpreadPF& pf) const;
  Reason filter_node_pf(const PodReq& req, int32_t idx, uint64_t* n, uint64_t* m, uint64_t* c,
                        const SpreadPF* pf, const InterPodPF* ip = nullptr) const;
  bool wants_spread_filter(const PodReq& req) const;
  int preempt_status(const PodReq& req, int32_t idx, const SpreadPF* spf, const InterPodPF* ipf) const;
  bool preempt_over(const PodReq& req, const PreemptArgs& args, const std::vector<int32_t>& potential,
                    PreemptResult* out);
  bool wants_interpod_filter(const PodReq& req) const;
  // InterPodAffinity is a constant (no filter, equal scores) for this pod: device-eligible
  bool interpod_inert(const PodReq& req) const;
  bool ext_checked(int32_t res) const;
  // normalized PodTopologySpread scores of the feasible nodes (soft constraints)
  void spread_scores(const PodReq& req, const std::vector<int32_t>& feas, std::vector<int64_t>& s) const;
  // the soft constraints score every node 0 (no live node carries one of their keys)
  bool spread_soft_constant(const std::vector<SpreadC>& soft) const;
  bool images_matter(const PodReq& req) const;
  void index_pod(Node& n, const Assignment& a, int sign);
  // pods of node n in namespace ns matching sel from the label index; false when sel needs the walk
  bool indexed_count(const Node& n, int32_t ns, const LSel& sel, bool skip_deleting, int64_t* out) const;
  // pods of node n one affinity term matches: the label index for a single-label (or empty)
  // selector, else a walk of the node's pods
  int64_t term_count(const Node& n, const PodTerm& t) const;
  // pods of node n in namespace ns a selector matches, over the label-set groups
  int64_t group_count(const Node& n, int32_t ns, const LSel& sel, bool skip_deleting) const;
  // ImageLocality scores every live node alike for this pod (each of its images is on no node,
  // or on every node with one size): true and the weighted score in *v
  bool image_score_const(const PodReq& req, int64_t* v) const;
  int64_t image_score(const PodReq& req, const Node& n) const;
  int64_t ext_amount(const std::vector<std::pair<int32_t, int64_t>>& v, int32_t res) const;
  std::unordered_map<int32_t, std::unordered_map<int64_t, int32_t>> image_sizes_;   // image → size → nodes
  void index_node_extras(const Node& n, int sign);
  void fill_result(const yoda_dev_result_t& res, CycleResult* r) const;
  Reason candidate_reason(const PodReq& req, const Node& n) const;
  bool taints_ok(const PodReq& req, const Node& n) const;
  bool affinity_ok(const PodReq& req, const Node& n) const;
  bool term_matches(const SelTerm& t, const Node& n) const;
  bool yoda_card_eligible(const PodReq& req, const Card& c, uint64_t m, uint64_t cl) const;
  uint64_t eff_free(const Card& c) const;
  int64_t gang_objective(const Node& n, const std::vector<int32_t>& set, uint64_t m,
                         int64_t* link_bad) const;

  bool compat_;
  uint32_t filters_ = F_NODE_UNSCHEDULABLE | F_NODE_NAME | F_TAINT_TOLERATION | F_NODE_AFFINITY |
                      F_NODE_RESOURCES_FIT | F_YODA;
  int64_t score_w_[S_NUM] = {300, 1, 1, 1, 1, 0, 0, 0, 0, 0};
  int64_t alloc_w_[2][3] = {{1, 1, 0}, {1, 1, 0}};   // [least, most][cpu, memory, other]
  Weights wt_;
  int pct_nodes_ = 0;
  int32_t unsched_key_ = 0;
  int32_t any_ip_ = 0, tcp_ = 0;      // interned "0.0.0.0" / "TCP" (NodePorts sanitize)
  std::unordered_map<int32_t, std::pair<int32_t, int32_t>> claim_vol_;   // claim → (driver, volume id)
  std::vector<Node> nodes_;
  std::vector<int32_t> free_slots_;
  uint32_t gen_counter_ = 0;
  std::vector<int32_t> removed_in_flight_;   // slots removed while a device batch held no lock
  int32_t live_ = 0;
  std::unordered_map<std::string, int32_t> node_idx_;
  std::vector<std::string> strings_;
  std::unordered_map<std::string, int32_t> string_idx_;
  // the ledger: a slab of entries (free ones reused with their vectors' capacity) and pod → index
  std::vector<Assignment> slab_;
  std::vector<int32_t> slab_free_;
  U64Map ledger_;
  // interned label sets (LabSetRec): id → record, hash → first id of its chain; idle ones (no
  // holder) are reused as they are and recycled by a sweep once they outnumber the held ones
  std::vector<LabSetRec> labsets_;
  std::vector<int32_t> labset_free_;
  std::unordered_map<uint64_t, int32_t> labset_by_hash_;
  int64_t labset_idle_ = 0;
  int32_t labset_acquire(int32_t ns, const Labels& labels);
  void labset_release(int32_t id);
  void labset_sweep();
  void sweep_lab_index(Node& n);
  void free_entry(int32_t si);
  void attach(int32_t si);
  void detach(int32_t si);
  std::mt19937_64 rng_{0x59d4};
  double settle_s_ = 30.0;
  double fixed_now_ = -1.0;
  // device scorer state
  void* dev_lib_ = nullptr;
  void* dev_ctx_ = nullptr;
  int dev_cap_ = 0;
  int dev_min_nodes_ = 256;
  uint64_t dev_cycles_ = 0, dev_fallbacks_ = 0, dev_batches_ = 0;
  std::vector<char> dirty_;
  std::vector<int32_t> dirty_list_;
  int32_t hard_taint_nodes_ = 0, prefer_taint_nodes_ = 0;
  // default-plugin state beyond the node rows
  std::unordered_map<int32_t, int32_t> image_nodes_;      // image → nodes reporting it
  int32_t avoid_nodes_ = 0;                               // nodes with preferAvoidPods controllers
  std::unordered_map<int32_t, int32_t> label_key_nodes_;  // label key → live nodes carrying it
  struct Svc {
    int32_t name;
    bool nil;
    Labels sel;
  };
  std::unordered_map<int32_t, std::vector<Svc>> svcs_;    // namespace → services
  std::unordered_map<uint64_t, LSel> ctrls_;              // (kind, ns, name) → selector
  static uint64_t ctrl_key(int8_t kind, int32_t ns, int32_t name) {
    return ((uint64_t)(uint8_t)kind << 58) ^ ((uint64_t)(uint32_t)ns << 29) ^ (uint64_t)(uint32_t)name;
  }
  std::vector<DefaultSpread> spread_defaults_;
  int32_t field_name_key_ = -1;               // "@metadata.name": a matchFields requirement on the node name
  int32_t dev_ext_res_ = -1;                  // set in the constructor: "ephemeral-storage"
  int64_t hard_aff_w_ = 1;
  std::unordered_set<uint64_t> aff_holders_;  // ledger pods with any (anti-)affinity term
  std::unordered_set<uint64_t> anti_holders_; // ... with a required anti-affinity term
  std::unordered_map<uint64_t, std::vector<AffSet>> aff_sets_;   // term-set hash → sets (collisions)
  void aff_set_add(Assignment& a);
  void aff_set_remove(const Assignment& a, bool whole_node = false);
  std::vector<int32_t> ext_ignored_;
  std::vector<std::string> ext_ignored_groups_;
  void* fn_destroy_ = nullptr;
  void* fn_upload_ = nullptr;
  void* fn_schedule_ = nullptr;
  void* fn_last_us_ = nullptr;
  void* fn_set_timing_ = nullptr;   // optional entry points
  void* fn_schedule_batch_ = nullptr;
  void* fn_busy_ = nullptr;
  void* fn_extras_ = nullptr;   // yoda_dev_batch_extras (k_batch score columns); optional
  std::recursive_mutex* ext_mu_ = nullptr;
  std::mutex dev_mu_;                        // device context (stream, staging buffers)
  std::atomic<bool> batch_in_flight_{false};
  double now() const;
  bool is_pending(const Node& n, const Assignment& a) const { return a.t_res > n.sample_ts - settle_s_; }
  int32_t next_start_ = 0;
  uint64_t cycles_ = 0;
  ThreadPool* pool_ = nullptr;
};

}  // namespace yoda
