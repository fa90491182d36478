// pybind11 bindings of the native scheduling engine (module yoda_scheduler_amd._native._yoda_core).
#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <memory>
#include <sys/eventfd.h>
#include <pthread.h>
#include <unistd.h>
#include <mutex>
#include <thread>
#include <chrono>

#include <pybind11/pybind11.h>

#include "build_id.h"
#include <pybind11/stl.h>

#include "engine.hpp"
#include "lane.hpp"

namespace py = pybind11;
using namespace yoda;

namespace {

// One process-wide engine lock: a batch scheduled on a worker thread (GIL released, see
// schedule_batch) may overlap event-loop calls (informer updates, bind failures) on the
// same engine. Recursive: bound methods never nest today, but a future one may.
std::recursive_mutex g_engine_mu;
std::atomic<uint64_t> g_lock_contended{0}, g_lock_wait_ns{0};
// Uncontended: take the lock with the GIL held (the common case, no GIL round trip). Contended
// — the engine worker is preparing or finishing a batch — wait WITHOUT the GIL, so the event
// loop's other threads (and the worker itself, which needs the GIL to hand its results back)
// keep running. No thread therefore ever waits for the lock while holding the GIL, which is
// what makes re-taking the GIL with the lock held deadlock-free.
struct EngineGuard {
  std::unique_lock<std::recursive_mutex> g{g_engine_mu, std::defer_lock};
  EngineGuard() {
    if (g.try_lock()) return;
    const auto t0 = std::chrono::steady_clock::now();
    if (PyGILState_Check()) {
      py::gil_scoped_release nogil;
      g.lock();
    } else {
      g.lock();
    }
    g_lock_contended.fetch_add(1, std::memory_order_relaxed);
    g_lock_wait_ns.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                 std::chrono::steady_clock::now() - t0).count(), std::memory_order_relaxed);
  }
};

// The engine lock at a moment no device batch is in flight (schedule_batch drops the lock
// while it waits for the device; replacing the device context then must wait for it).
EngineGuard lock_without_batch(Engine& e) {
  for (;;) {
    EngineGuard g;
    if (!e.batch_in_flight()) return g;
    g.g.unlock();
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

int8_t effect_of(const std::string& e) {
  if (e == "NoSchedule") return kNoSchedule;
  if (e == "PreferNoSchedule") return kPreferNoSchedule;
  if (e == "NoExecute") return kNoExecute;
  return kEffectAny;
}

int8_t selop_of(const std::string& op) {
  if (op == "In") return kIn;
  if (op == "NotIn") return kNotIn;
  if (op == "Exists") return kExists;
  if (op == "DoesNotExist") return kDoesNotExist;
  if (op == "Gt") return kGt;
  if (op == "Lt") return kLt;
  throw std::invalid_argument("unknown node selector operator: " + op);
}

SelTerm make_term(Engine& e, const py::list& reqs) {
  SelTerm t;
  for (auto item : reqs) {
    auto tup = item.cast<py::tuple>();   // (key, op, [values])
    SelReq r;
    r.key = e.intern(tup[0].cast<std::string>());
    r.op = selop_of(tup[1].cast<std::string>());
    r.num = 0;
    for (auto v : tup[2].cast<py::list>()) {
      std::string s = v.cast<std::string>();
      r.values.push_back(e.intern(s));
      if (r.op == kGt || r.op == kLt) r.num = std::stoll(s);
    }
    t.reqs.push_back(std::move(r));
  }
  return t;
}

// LabelSelector.native() tuple (namespaces | None, nothing, [(key, value)], [(key, op, [values])]) or
// None (a nil selector) → LSel over interned strings; namespaces are not part of an LSel
LSel lsel_of(Engine& e, const py::handle& h) {
  LSel s;
  if (h.is_none()) {
    s.nothing = true;
    return s;
  }
  auto t = h.cast<py::tuple>();
  s.nothing = t[1].cast<bool>();
  for (auto kv : t[2]) {
    auto p = kv.cast<py::tuple>();
    s.reqs.push_back(LReq{e.intern(p[0].cast<std::string>()), kIn, {e.intern(p[1].cast<std::string>())}});
  }
  for (auto ex : t[3]) {
    auto p = ex.cast<py::tuple>();
    LReq r;
    r.key = e.intern(p[0].cast<std::string>());
    r.op = selop_of(p[1].cast<std::string>());
    if (r.op == kGt || r.op == kLt) throw std::invalid_argument("label selectors take In/NotIn/Exists/DoesNotExist");
    for (auto v : p[2]) r.values.push_back(e.intern(v.cast<std::string>()));
    s.reqs.push_back(std::move(r));
  }
  return s;
}

Labels labels_of(Engine& e, const std::vector<std::pair<std::string, std::string>>& kv) {
  Labels l;
  l.reserve(kv.size());
  for (const auto& x : kv) l.emplace_back(e.intern(x.first), e.intern(x.second));
  std::sort(l.begin(), l.end());
  return l;
}

int8_t owner_kind_of(const std::string& api, const std::string& kind) {
  // plugins/optional.py::_OWNER_KINDS
  if (api == "v1" && kind == "ReplicationController") return 1;
  if (api == "apps/v1" && kind == "ReplicaSet") return 2;
  if (api == "apps/v1" && kind == "StatefulSet") return 3;
  return 0;
}

// (node, feasible, evaluated, cards, score, reason_counts, gang_quality, node_gen, stale)
py::tuple cycle_tuple(const CycleResult& r) {
  return py::make_tuple(r.node, r.feasible, r.evaluated, r.cards, r.score, r.reason_counts, r.gang_quality,
                        r.node_gen, r.stale);
}

// Engine batches on a native thread. The event loop submits a batch (ids + request
// pointers; Python keeps the PodReq objects alive until the result is collected), the
// thread runs Engine::schedule_batch under the engine lock — which the engine itself drops
// while a device batch is on the GPU — and signals an eventfd the loop watches; the loop
// converts the results when it collects them. Unlike an executor thread this one never takes
// the GIL, so a batch costs the event loop no GIL hand-offs (two or more per batch with a
// Python worker, each up to the switch interval).
class BatchWorker {
 public:
  struct Job {
    uint64_t id = 0;
    std::vector<uint64_t> pods;
    std::vector<const PodReq*> reqs;
    std::vector<CycleResult> res;
    std::string err;
    double t0 = 0, t1 = 0;   // CLOCK_MONOTONIC seconds (time.perf_counter's clock on Linux)
  };

  explicit BatchWorker(Engine* e) : e_(e) {
    efd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (efd_ < 0) throw std::runtime_error("eventfd failed");
    th_ = std::thread([this] {
    pthread_setname_np(pthread_self(), "yoda-engine");   // per-thread CPU in bench / top -H
    run();
  });
  }
  ~BatchWorker() { close(); }

  int fileno() const { return efd_; }

  uint64_t submit(std::vector<uint64_t> pods, std::vector<const PodReq*> reqs) {
    if (pods.size() != reqs.size()) throw std::invalid_argument("pods/reqs length mismatch");
    auto j = std::make_unique<Job>();
    j->pods = std::move(pods);
    j->reqs = std::move(reqs);
    std::lock_guard<std::mutex> g(mu_);
    if (stop_) throw std::runtime_error("batch worker closed");
    j->id = ++next_;
    const uint64_t id = j->id;
    q_.push_back(std::move(j));
    cv_.notify_one();
    return id;
  }

  std::vector<std::unique_ptr<Job>> take_done() {
    uint64_t v;
    while (::read(efd_, &v, sizeof v) > 0) {
    }
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::unique_ptr<Job>> out(std::make_move_iterator(done_.begin()), std::make_move_iterator(done_.end()));
    done_.clear();
    return out;
  }

  size_t pending() {
    std::lock_guard<std::mutex> g(mu_);
    return q_.size() + (busy_ ? 1 : 0);
  }

  void close() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stop_ && !th_.joinable()) return;
      stop_ = true;
      cv_.notify_all();
    }
    if (th_.joinable()) th_.join();
    if (efd_ >= 0) {
      ::close(efd_);
      efd_ = -1;
    }
  }

 private:
  static double mono() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  void run() {
    for (;;) {
      std::unique_ptr<Job> j;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;   // stop requested and nothing left
        j = std::move(q_.front());
        q_.pop_front();
        busy_ = true;
      }
      j->t0 = mono();
      try {
        EngineGuard lk;   // this thread never holds the GIL: a plain lock
        j->res = e_->schedule_batch(j->pods, j->reqs);
      } catch (const std::exception& ex) {
        j->err = ex.what();
      } catch (...) {
        j->err = "unknown error in schedule_batch";
      }
      j->t1 = mono();
      {
        std::lock_guard<std::mutex> g(mu_);
        done_.push_back(std::move(j));
        busy_ = false;
      }
      const uint64_t one = 1;
      ssize_t w = ::write(efd_, &one, sizeof one);
      (void)w;
    }
  }

  Engine* e_;
  int efd_ = -1;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::unique_ptr<Job>> q_, done_;
  bool stop_ = false, busy_ = false;
  uint64_t next_ = 0;
};

}  // namespace

// (namespaces | None, nothing, [(key, value)], [(key, op, [values])]) → MatchTerm
MatchTerm match_term(const py::handle& h) {
  auto t = h.cast<py::tuple>();
  MatchTerm m;
  if (!t[0].is_none())
    for (auto ns : t[0]) m.namespaces.push_back(ns.cast<std::string>());
  m.nothing = t[1].cast<bool>();
  for (auto kv : t[2]) {
    auto p = kv.cast<py::tuple>();
    m.labels.emplace_back(p[0].cast<std::string>(), p[1].cast<std::string>());
  }
  for (auto ex : t[3]) {
    auto p = ex.cast<py::tuple>();
    MatchTerm::Expr x;
    x.key = p[0].cast<std::string>();
    const std::string op = p[1].cast<std::string>();
    x.op = op == "In" ? 0 : op == "NotIn" ? 1 : op == "Exists" ? 2 : op == "DoesNotExist" ? 3 : -1;
    if (x.op < 0) throw std::invalid_argument("unknown selector operator " + op);
    for (auto v : p[2]) x.values.push_back(v.cast<std::string>());
    m.exprs.push_back(std::move(x));
  }
  return m;
}

namespace yoda_sampler {
void start(const std::vector<int>& tids, int period_us, bool stacks);
std::pair<std::vector<std::tuple<uintptr_t, int, std::vector<uintptr_t>>>, size_t> stop();
}  // namespace yoda_sampler

PYBIND11_MODULE(_yoda_core, m) {
  m.def("sampler_start", &yoda_sampler::start, py::arg("tids"), py::arg("period_us") = 200,
        py::arg("stacks") = false,
        "sample the program counter of these threads every period_us of their own CPU time (sampler.cpp)");
  m.def("sampler_stop", &yoda_sampler::stop, "stop sampling: ([(pc, tid | overrun << 24, [return addresses])], dropped)");
  m.def("build_id", [] { return std::string(YODA_BUILD_ID); }, "hash of the sources this module was built from");
  m.doc() = "Native placement / scheduling-cycle engine (C++17)";
  m.def("engine_lock_stats", [] {
    return py::make_tuple(g_lock_contended.load(), g_lock_wait_ns.load() / 1000);
  }, "(contended acquisitions, total wait in us) of the process-wide engine lock");
  m.attr("F_NODE_UNSCHEDULABLE") = (uint32_t)F_NODE_UNSCHEDULABLE;
  m.attr("F_NODE_NAME") = (uint32_t)F_NODE_NAME;
  m.attr("F_TAINT_TOLERATION") = (uint32_t)F_TAINT_TOLERATION;
  m.attr("F_NODE_AFFINITY") = (uint32_t)F_NODE_AFFINITY;
  m.attr("F_NODE_RESOURCES_FIT") = (uint32_t)F_NODE_RESOURCES_FIT;
  m.attr("F_YODA") = (uint32_t)F_YODA;
  m.attr("S_YODA") = (int)S_YODA;
  m.attr("S_LEAST_ALLOCATED") = (int)S_LEAST_ALLOCATED;
  m.attr("S_BALANCED_ALLOCATION") = (int)S_BALANCED_ALLOCATION;
  m.attr("S_TAINT_TOLERATION") = (int)S_TAINT_TOLERATION;
  m.attr("S_NODE_AFFINITY") = (int)S_NODE_AFFINITY;
  m.attr("S_MOST_ALLOCATED") = (int)S_MOST_ALLOCATED;
  m.attr("S_IMAGE_LOCALITY") = (int)S_IMAGE_LOCALITY;
  m.attr("S_PREFER_AVOID") = (int)S_PREFER_AVOID;
  m.attr("S_SPREAD") = (int)S_SPREAD;
  m.attr("S_NUM") = (int)S_NUM;
  m.attr("F_SPREAD") = (uint32_t)F_SPREAD;
  m.attr("F_INTERPOD") = (uint32_t)F_INTERPOD;
  m.attr("F_NODE_PORTS") = (uint32_t)F_NODE_PORTS;
  m.attr("S_INTERPOD") = (int)S_INTERPOD;
  m.attr("REASONS") = py::make_tuple("OK", "NodeUnschedulable", "NodeName", "TaintToleration", "NodeAffinity",
                                     "NodeResourcesFit", "NoScv", "ScvStale", "GpuNumber", "GpuMemory",
                                     "GpuClock", "GpuFit", "NodeGone", "NodeResourcesFitExtended",
                                     "PodTopologySpread", "PodTopologySpreadLabel", "InterPodAffinityExisting",
                                     "InterPodAffinity", "InterPodAntiAffinity", "NodePorts", "VolumeBinding",
                                     "VolumeZone", "NodeVolumeLimits");

  py::class_<PodReq>(m, "PodReq")
      .def_readonly("has_number", &PodReq::has_number)
      .def_readonly("number", &PodReq::number)
      .def_readonly("has_memory", &PodReq::has_memory)
      .def_readonly("memory", &PodReq::memory)
      .def_readonly("has_clock", &PodReq::has_clock)
      .def_readonly("clock", &PodReq::clock)
      .def_readonly("cpu_m", &PodReq::cpu_m)
      .def_readonly("mem", &PodReq::mem)
      .def_readonly("containers", &PodReq::containers)
      .def_readonly("spread_explicit", &PodReq::spread_explicit)
      .def_readwrite("pod_priority", &PodReq::pod_priority)
      .def_property_readonly("n_ext", [](const PodReq& r) { return r.ext.size(); })
      .def_property_readonly("n_spread", [](const PodReq& r) { return r.spread.size(); });

  py::class_<Engine>(m, "Engine")
      .def(py::init([](bool compat, int threads) {
             auto* e = new Engine(compat, threads);
             e->set_external_lock(&g_engine_mu);   // schedule_batch drops it during device batches
             return e;
           }),
           py::arg("compat") = false, py::arg("threads") = 1)
      .def_property("compat", &Engine::compat, &Engine::set_compat)
      .def_property("filters", &Engine::filters, &Engine::set_filters)
      .def("set_score_weight", &Engine::set_score_weight, py::call_guard<EngineGuard>())
      .def("set_alloc_weights", &Engine::set_alloc_weights, py::arg("most"), py::arg("cpu"), py::arg("mem"),
           py::arg("other"), py::call_guard<EngineGuard>())
      .def("score_weight", &Engine::score_weight, py::call_guard<EngineGuard>())
      .def("set_gang_weights",
           [](Engine& e, int64_t link, int64_t numa, int64_t fit, int64_t occ, bool binpack, int64_t gang_score,
              int64_t enum_limit, int64_t minlink) {
             auto& w = e.weights();
             w.w_link = link; w.w_numa = numa; w.w_fit = fit; w.w_occ = occ;
             w.gpu_binpack = binpack; w.w_gang_score = gang_score; w.enum_limit = enum_limit;
             w.w_minlink = minlink;
           },
           py::arg("link") = 4, py::arg("numa") = 2, py::arg("fit") = 1, py::arg("occ") = 1,
           py::arg("binpack") = false, py::arg("gang_score") = 3, py::arg("enum_limit") = 5000,
           py::arg("minlink") = 2, py::call_guard<EngineGuard>())
      .def("set_percentage_of_nodes_to_score", &Engine::set_percentage_of_nodes_to_score, py::call_guard<EngineGuard>())
      .def("seed", &Engine::seed, py::call_guard<EngineGuard>())
      .def("intern", &Engine::intern, py::call_guard<EngineGuard>())
      .def("upsert_node", &Engine::upsert_node, py::call_guard<EngineGuard>())
      .def("node_index", &Engine::node_index, py::call_guard<EngineGuard>())
      .def("remove_node", &Engine::remove_node, py::call_guard<EngineGuard>())
      .def_property_readonly("num_nodes", &Engine::num_nodes)
      .def_property_readonly("live_nodes", &Engine::live_nodes)
      .def_property_readonly("cycles", &Engine::cycles)
      .def_property_readonly("ledger_size", &Engine::ledger_size)
      .def_property_readonly("labsets_used", &Engine::labsets_used)
      .def("node_name", [](Engine& e, int32_t i) { return e.node(i).name; }, py::call_guard<EngineGuard>())
      .def("node_gen", &Engine::node_gen, py::call_guard<EngineGuard>(),
           "generation of a node slot (changes when the slot's node is removed or replaced)")
      .def("set_node_meta",
           [](Engine& e, int32_t idx, bool unsched, const std::vector<std::pair<std::string, std::string>>& labels,
              const std::vector<std::tuple<std::string, std::string, std::string>>& taints, int64_t cpu_m,
              int64_t mem, int64_t pods) {
             std::vector<std::pair<int32_t, int32_t>> lab;
             for (auto& kv : labels) lab.emplace_back(e.intern(kv.first), e.intern(kv.second));
             std::vector<Taint> ts;
             for (auto& t : taints)
               ts.push_back(Taint{e.intern(std::get<0>(t)), e.intern(std::get<1>(t)), effect_of(std::get<2>(t))});
             e.set_node_meta(idx, unsched, lab, ts, cpu_m, mem, pods);
           }, py::call_guard<EngineGuard>())
      .def("enable_device",
           [](Engine& e, const std::string& path, int device, int capacity, int min_nodes) {
             std::string err;
             bool ok = false;
             {
               py::gil_scoped_release nogil;
               EngineGuard g = lock_without_batch(e);
               ok = e.enable_device(path, device, capacity, min_nodes, &err);
             }
             return py::make_tuple(ok, err);
           },
           py::arg("lib_path"), py::arg("device") = 0, py::arg("capacity") = 65536, py::arg("min_nodes") = 256)
      .def("disable_device",
           [](Engine& e) {
             py::gil_scoped_release nogil;
             EngineGuard g = lock_without_batch(e);
             e.disable_device();
           })
      .def_property_readonly("device_enabled", &Engine::device_enabled)
      .def_property_readonly("device_ctx", &Engine::device_ctx)
      .def_property_readonly("device_cycles", &Engine::device_cycles)
      .def_property_readonly("device_fallbacks", &Engine::device_fallbacks)
      .def_property_readonly("device_batches", &Engine::device_batches)
      .def("device_last_us", &Engine::device_last_us, py::call_guard<EngineGuard>())
      .def("device_set_timing", &Engine::device_set_timing, py::arg("on"), py::call_guard<EngineGuard>())
      .def("device_eligible", &Engine::device_eligible, py::arg("req"), py::arg("slots") = false,
           py::call_guard<EngineGuard>())
      .def("device_flush", &Engine::device_flush, py::call_guard<EngineGuard>())
      .def("device_cycle",
           [](Engine& e, const PodReq& r) -> py::object {
             CycleResult c;
             if (!e.device_cycle(r, &c)) return py::none();
             return cycle_tuple(c);
           }, py::call_guard<EngineGuard>())
      // cards: list of (total, free, clock, bandwidth, core, power, healthy, phys, numa, occ_q)
      .def("set_cards",
           [](Engine& e, int32_t idx,
              const std::vector<std::tuple<uint64_t, uint64_t, uint64_t, uint64_t, uint64_t, uint64_t, bool, int32_t,
                                           int32_t, int32_t>>& cs,
              uint64_t card_number, uint64_t free_sum, uint64_t total_sum, bool stale, double sample_ts) {
             std::vector<Card> cards;
             cards.reserve(cs.size());
             for (auto& t : cs) {
               Card c;
               std::tie(c.total_mb, c.free_mb, c.clock, c.bandwidth, c.core, c.power, c.healthy, c.phys, c.numa,
                        c.occ_q) = t;
               if (c.phys < 0 || c.phys >= kMaxPhys) throw std::invalid_argument("physical id out of range");
               cards.push_back(c);
             }
             e.set_cards(idx, std::move(cards), card_number, free_sum, total_sum, stale, sample_ts);
           },
           py::arg("idx"), py::arg("cards"), py::arg("card_number"), py::arg("free_sum"), py::arg("total_sum"),
           py::arg("stale"), py::arg("sample_ts") = 0.0, py::call_guard<EngineGuard>())
      .def_property("settle_seconds", &Engine::settle_seconds, &Engine::set_settle_seconds)
      .def("set_fixed_now", &Engine::set_fixed_now, py::call_guard<EngineGuard>())
      .def("clear_scv", &Engine::clear_scv, py::call_guard<EngineGuard>())
      .def("set_links", &Engine::set_links, py::call_guard<EngineGuard>())
      .def("node_cards",
           [](Engine& e, int32_t idx) {
             py::list out;
             for (auto& c : e.node(idx).cards)
               out.append(py::make_tuple(c.total_mb, c.free_mb, c.reserved_mb, c.pods, c.clock, c.healthy, c.phys,
                                         c.pending_mb));
             return out;
           }, py::call_guard<EngineGuard>())
      // (has_scv, stale, card_number, [(healthy, free, effective free, clock)]) — the yoda
      // filter's inputs for the Scv queueing hint; None for an unknown / removed node
      .def("filter_view",
           [](Engine& e, int32_t idx) -> py::object {
             const FilterView v = e.filter_view(idx);
             if (!v.known) return py::none();
             py::list cards;
             for (const auto& c : v.cards) cards.append(py::make_tuple(c.healthy, c.free, c.eff_free, c.clock));
             return py::make_tuple(v.has_scv, v.stale, v.card_number, cards);
           }, py::call_guard<EngineGuard>())
      .def("node_usage",
           [](Engine& e, int32_t idx) {
             const Node& n = e.node(idx);
             return py::make_tuple(n.req_cpu_m, n.req_mem, n.pod_count, n.label_mem_sum, n.nz_cpu_m, n.nz_mem);
           }, py::call_guard<EngineGuard>())
      .def("make_req",
           [](Engine& e, bool has_number, uint64_t number, bool has_memory, uint64_t memory, bool has_clock,
              uint64_t clock, uint64_t clock_min, int64_t priority, const std::string& node_name, int64_t cpu_m,
              int64_t mem, const std::vector<std::pair<std::string, std::string>>& node_selector,
              const py::list& required, const py::list& preferred, const py::list& tolerations,
              int64_t nz_cpu_m, int64_t nz_mem) {
             PodReq r;
             r.has_number = has_number;
             r.number = has_number ? number : 1;
             r.has_memory = has_memory;
             r.memory = memory;
             r.has_clock = has_clock;
             r.clock = clock;
             r.clock_min = clock_min;
             r.priority = priority;
             r.node_name = node_name.empty() ? -1 : e.intern(node_name);
             r.cpu_m = cpu_m;
             r.mem = mem;
             // -1: derive at pod level (one container); PodInfo passes per-container values
             r.nz_cpu_m = nz_cpu_m >= 0 ? nz_cpu_m : (cpu_m > 0 ? cpu_m : 100);
             r.nz_mem = nz_mem >= 0 ? nz_mem : (mem > 0 ? mem : 200LL * 1024 * 1024);
             for (auto& kv : node_selector) r.node_selector.emplace_back(e.intern(kv.first), e.intern(kv.second));
             for (auto t : required) r.required_terms.push_back(make_term(e, t.cast<py::list>()));
             for (auto p : preferred) {
               auto tup = p.cast<py::tuple>();
               r.preferred_terms.push_back(PrefTerm{tup[0].cast<int32_t>(), make_term(e, tup[1].cast<py::list>())});
             }
             for (auto t : tolerations) {
               auto tup = t.cast<py::tuple>();   // (key|None, value, op, effect)
               Toleration x;
               x.key = tup[0].is_none() ? -1 : e.intern(tup[0].cast<std::string>());
               if (x.key == 0) x.key = -1;   // empty key
               x.value = e.intern(tup[1].cast<std::string>());
               x.op = tup[2].cast<std::string>() == "Exists" ? kTolExists : kTolEqual;
               x.effect = effect_of(tup[3].cast<std::string>());
               r.tolerations.push_back(x);
             }
             return r;
           },
           py::arg("has_number"), py::arg("number"), py::arg("has_memory"), py::arg("memory"), py::arg("has_clock"),
           py::arg("clock"), py::arg("clock_min") = 0, py::arg("priority") = 0, py::arg("node_name") = "",
           py::arg("cpu_m") = 0, py::arg("mem") = 0,
           py::arg("node_selector") = std::vector<std::pair<std::string, std::string>>{},
           py::arg("required") = py::list(), py::arg("preferred") = py::list(), py::arg("tolerations") = py::list(),
           py::arg("nz_cpu_m") = -1, py::arg("nz_mem") = -1, py::call_guard<EngineGuard>())
      // the default-plugin inputs of a PodReq (ImageLocality, NodeResourcesFit beyond cpu/memory,
      // NodePreferAvoidPods, PodTopologySpread and what other pods' spread counts read of it)
      // NodeVolumeLimits: the "namespace/claim" of the pod's persistentVolumeClaim volumes (the
      // ledger keeps them per node); count_vols: count them against CSI limits in this cycle
      .def("set_req_claims",
           [](Engine& e, PodReq& r, const std::vector<std::string>& claims, bool count_vols) {
             r.pvc_claims.clear();
             for (const auto& c : claims) r.pvc_claims.push_back(e.intern(c));
             r.count_vols = count_vols && !r.pvc_claims.empty();
           },
           py::arg("req"), py::arg("claims"), py::arg("count_vols") = false, py::call_guard<EngineGuard>())
      // claim volumes: [(claim, driver, volume id)] set, [claim] removed (plugins/volumes.py::claim_volume)
      .def("set_claim_volumes",
           [](Engine& e, const std::vector<std::tuple<std::string, std::string, std::string>>& add,
              const std::vector<std::string>& remove) {
             for (const auto& c : remove) e.clear_claim_volume(e.intern(c));
             for (const auto& t : add)
               e.set_claim_volume(e.intern(std::get<0>(t)), e.intern(std::get<1>(t)), e.intern(std::get<2>(t)));
           },
           py::arg("add"), py::arg("remove"), py::call_guard<EngineGuard>())
      .def("set_node_vol_limits",
           [](Engine& e, int32_t idx, const std::vector<std::pair<std::string, int64_t>>& limits) {
             std::vector<std::pair<int32_t, int64_t>> v;
             for (const auto& l : limits) v.emplace_back(e.intern(l.first), l.second);
             e.set_node_vol_limits(idx, std::move(v));
           },
           py::arg("idx"), py::arg("limits"), py::call_guard<EngineGuard>())
      // NodePorts: the pod's containers' host ports [(hostPort, protocol, hostIP)]
      .def("set_req_ports",
           [](Engine& e, PodReq& r, const std::vector<std::tuple<int64_t, std::string, std::string>>& ports) {
             r.host_ports.clear();
             HostPort h;
             for (const auto& t : ports)
               if (e.host_port(std::get<0>(t), std::get<1>(t), std::get<2>(t), &h)) r.host_ports.push_back(h);
           },
           py::arg("req"), py::arg("ports"), py::call_guard<EngineGuard>())
      .def("set_req_extras",
           [](Engine& e, PodReq& r, const std::string& ns, const std::vector<std::pair<std::string, std::string>>& labels,
              bool deleting, const std::vector<std::string>& images, int32_t containers,
              const std::vector<std::pair<std::string, int64_t>>& ext, const py::object& owner,
              const py::object& avoid, const py::object& spread, const py::object& pod_aff) {
             r.ns = e.intern(ns);
             r.labels = labels_of(e, labels);
             r.deleting = deleting;
             r.images.clear();
             for (const auto& im : images) r.images.push_back(e.intern(im));
             r.containers = containers;
             r.ext.clear();
             for (const auto& x : ext)
               if (x.second) r.ext.emplace_back(e.intern(x.first), x.second);
             std::sort(r.ext.begin(), r.ext.end());
             r.owner_kind = 0;
             r.owner_name = -1;
             if (!owner.is_none()) {
               auto t = owner.cast<py::tuple>();   // (apiVersion, kind, name, uid)
               r.owner_kind = owner_kind_of(t[0].cast<std::string>(), t[1].cast<std::string>());
               if (r.owner_kind) r.owner_name = e.intern(t[2].cast<std::string>());
             }
             r.avoid_kind = 0;
             r.avoid_uid = -1;
             if (!avoid.is_none()) {
               auto t = avoid.cast<py::tuple>();   // (kind, uid)
               const std::string k = t[0].cast<std::string>();
               r.avoid_kind = k == "ReplicationController" ? 1 : k == "ReplicaSet" ? 2 : 0;
               if (r.avoid_kind) r.avoid_uid = e.intern(t[1].cast<std::string>());
             }
             r.spread.clear();
             r.spread_explicit = false;
             if (!spread.is_none()) {
               for (auto c : spread) {
                 auto t = c.cast<py::tuple>();     // (topologyKey, maxSkew, whenUnsatisfiable, selector | None)
                 r.spread_explicit = true;
                 const std::string when = t[2].cast<std::string>();
                 if (when != "DoNotSchedule" && when != "ScheduleAnyway") continue;   // in neither list
                 SpreadC x;
                 x.key = e.intern(t[0].cast<std::string>());
                 x.max_skew = t[1].cast<int32_t>();
                 x.hard = when == "DoNotSchedule";
                 x.sel = lsel_of(e, t[3]);
                 r.spread.push_back(std::move(x));
               }
             }
             // (required affinity, required anti-affinity, preferred affinity, preferred anti-affinity),
             // each [(topologyKey, namespaces | None, LabelSelector.native() | None, weight)]
             r.aff.reset();
             if (!pod_aff.is_none()) {
               auto pa = std::make_shared<PodAffinity>();
               auto t4 = pod_aff.cast<py::tuple>();
               std::vector<PodTerm>* dst[4] = {&pa->req_aff, &pa->req_anti, &pa->pref_aff, &pa->pref_anti};
               for (int k = 0; k < 4; ++k)
                 for (auto term : t4[k]) {
                   auto t = term.cast<py::tuple>();
                   PodTerm x;
                   x.key = e.intern(t[0].cast<std::string>());
                   if (t[1].is_none() || py::len(t[1]) == 0) x.ns.push_back(r.ns);
                   else
                     for (auto n : t[1]) x.ns.push_back(e.intern(n.cast<std::string>()));
                   x.sel = lsel_of(e, t[2]);
                   x.weight = t[3].cast<int32_t>();
                   dst[k]->push_back(std::move(x));
                 }
               if (!pa->empty()) r.aff = std::move(pa);
             }
           },
           py::arg("req"), py::arg("ns"), py::arg("labels"), py::arg("deleting") = false,
           py::arg("images") = std::vector<std::string>{}, py::arg("containers") = 0,
           py::arg("ext") = std::vector<std::pair<std::string, int64_t>>{}, py::arg("owner") = py::none(),
           py::arg("avoid") = py::none(), py::arg("spread") = py::none(), py::arg("pod_aff") = py::none(),
           py::call_guard<EngineGuard>())
      .def("set_hard_pod_affinity_weight", &Engine::set_hard_pod_affinity_weight, py::call_guard<EngineGuard>())
      .def_property_readonly("affinity_holders", &Engine::affinity_holders)
      .def("set_node_extras",
           [](Engine& e, int32_t idx, const std::vector<std::pair<std::string, int64_t>>& images,
              const std::vector<std::pair<std::string, int64_t>>& ext_alloc,
              const std::vector<std::pair<std::string, std::string>>& avoid) {
             std::vector<std::pair<int32_t, int64_t>> im, ea;
             for (const auto& x : images) im.emplace_back(e.intern(x.first), x.second);
             for (const auto& x : ext_alloc) ea.emplace_back(e.intern(x.first), x.second);
             std::vector<std::pair<int8_t, int32_t>> av;
             for (const auto& x : avoid) {
               const int8_t k = x.first == "ReplicationController" ? 1 : x.first == "ReplicaSet" ? 2 : 0;
               if (k) av.emplace_back(k, e.intern(x.second));
             }
             e.set_node_extras(idx, std::move(im), std::move(ea), std::move(av));
           },
           py::arg("idx"), py::arg("images"), py::arg("ext_alloc"), py::arg("avoid"), py::call_guard<EngineGuard>())
      .def("image_nodes", [](Engine& e, const std::string& im) { return e.image_nodes(e.intern(im)); },
           py::call_guard<EngineGuard>())
      .def_property_readonly("avoid_nodes", &Engine::avoid_nodes)
      .def("set_service",
           [](Engine& e, const std::string& ns, const std::string& name, const py::object& selector) {
             if (selector.is_none()) {
               e.set_service(e.intern(ns), e.intern(name), true, {});
               return;
             }
             e.set_service(e.intern(ns), e.intern(name), false,
                           labels_of(e, selector.cast<std::vector<std::pair<std::string, std::string>>>()));
           },
           py::arg("ns"), py::arg("name"), py::arg("selector"), py::call_guard<EngineGuard>())
      .def("remove_service",
           [](Engine& e, const std::string& ns, const std::string& name) {
             e.remove_service(e.intern(ns), e.intern(name));
           }, py::call_guard<EngineGuard>())
      // kind: "replicationcontrollers" (selector: [(key, value)]) | "replicasets" | "statefulsets"
      // (selector: LabelSelector.native() tuple, or None when nil)
      .def("set_controller",
           [](Engine& e, const std::string& kind, const std::string& ns, const std::string& name,
              const py::object& selector) {
             const int8_t k = kind == "replicationcontrollers" ? 1 : kind == "replicasets" ? 2 : kind == "statefulsets" ? 3 : 0;
             if (!k) throw std::invalid_argument("unknown controller kind " + kind);
             LSel s;
             if (k == 1) {
               if (!selector.is_none())
                 for (const auto& kv : labels_of(e, selector.cast<std::vector<std::pair<std::string, std::string>>>()))
                   s.reqs.push_back(LReq{kv.first, kIn, {kv.second}});
             } else {
               s = lsel_of(e, selector);
             }
             e.set_controller(k, e.intern(ns), e.intern(name), std::move(s));
           },
           py::arg("kind"), py::arg("ns"), py::arg("name"), py::arg("selector"), py::call_guard<EngineGuard>())
      .def("remove_controller",
           [](Engine& e, const std::string& kind, const std::string& ns, const std::string& name) {
             const int8_t k = kind == "replicationcontrollers" ? 1 : kind == "replicasets" ? 2 : kind == "statefulsets" ? 3 : 0;
             if (k) e.remove_controller(k, e.intern(ns), e.intern(name));
           }, py::call_guard<EngineGuard>())
      // [(key, op, [values])] of the pod's DefaultSelector, or None when it is empty
      .def("default_selector",
           [](Engine& e, const PodReq& r) -> py::object {
             LSel s;
             if (!e.default_selector(r, &s)) return py::none();
             py::list out;
             static const char* kOps[] = {"In", "NotIn", "Exists", "DoesNotExist"};
             for (const auto& q : s.reqs) {
               py::list vals;
               for (int32_t v : q.values) vals.append(e.str(v));
               out.append(py::make_tuple(e.str(q.key), kOps[q.op], vals));
             }
             return out;
           }, py::call_guard<EngineGuard>())
      .def("set_pod_meta",
           [](Engine& e, uint64_t pod, const std::vector<std::pair<std::string, std::string>>& labels, bool deleting) {
             return e.set_pod_meta(pod, labels_of(e, labels), deleting);
           }, py::arg("pod"), py::arg("labels"), py::arg("deleting"), py::call_guard<EngineGuard>())
      .def("count_matching",
           [](Engine& e, int32_t idx, const std::string& ns, const py::object& selector) {
             return e.count_matching(idx, e.intern(ns), lsel_of(e, selector));
           }, py::call_guard<EngineGuard>())
      // PodTopologySpread args: [(topologyKey, maxSkew, whenUnsatisfiable)]
      .def("set_spread_defaults",
           [](Engine& e, const std::vector<std::tuple<std::string, int32_t, std::string>>& d) {
             std::vector<DefaultSpread> v;
             for (const auto& x : d) {
               const std::string& w = std::get<2>(x);
               if (w != "DoNotSchedule" && w != "ScheduleAnyway") continue;
               v.push_back(DefaultSpread{e.intern(std::get<0>(x)), std::get<1>(x), w == "DoNotSchedule"});
             }
             e.set_spread_defaults(std::move(v));
           }, py::call_guard<EngineGuard>())
      .def("set_ext_ignored",
           [](Engine& e, const std::vector<std::string>& res, const std::vector<std::string>& groups) {
             std::vector<int32_t> r;
             for (const auto& x : res) r.push_back(e.intern(x));
             e.set_ext_ignored(std::move(r), groups);
           }, py::call_guard<EngineGuard>())
      // DefaultPreemption on the ledger: pdbs [(namespace, LabelSelector.native() | None,
      // disruptionsAllowed)] → (node | -1, [victim ids], [cards], PDB violations, potential
      // nodes, nodes dry-run, candidates)
      .def("preempt",
           [](Engine& e, const PodReq& r, int64_t priority, const py::list& pdbs, int32_t min_pct, int32_t min_abs,
              int64_t offset) {
             PreemptArgs a;
             a.priority = priority;
             a.min_pct = min_pct;
             a.min_abs = min_abs;
             a.offset = offset;
             for (auto t : pdbs) {
               auto tup = t.cast<py::tuple>();
               Pdb d;
               d.ns = e.intern(tup[0].cast<std::string>());
               d.sel = lsel_of(e, tup[1]);
               d.allowed = tup[2].cast<int64_t>();
               a.pdbs.push_back(std::move(d));
             }
             PreemptResult o;
             e.preempt(r, a, &o);
             return py::make_tuple(o.node, o.victims, o.cards, o.violations, o.potential, o.evaluated, o.candidates);
           },
           py::arg("req"), py::arg("priority"), py::arg("pdbs"), py::arg("min_pct") = 10, py::arg("min_abs") = 100,
           py::arg("offset") = -1, py::call_guard<EngineGuard>())
      // nodes where preemption might help (first failing filter in upstream order is not
      // UnschedulableAndUnresolvable), in node-index order
      .def("preempt_potential",
           [](Engine& e, const PodReq& r) { return e.preempt_potential(r); }, py::call_guard<EngineGuard>())
      .def("detach_pod", &Engine::detach_pod, py::call_guard<EngineGuard>())
      .def("attach_pod", &Engine::attach_pod, py::call_guard<EngineGuard>())
      // (node, cards, mb per card, reservation time, spec.priority) or None
      .def("assignment_info",
           [](Engine& e, uint64_t pod) -> py::object {
             const Assignment* a = e.assignment(pod);
             if (!a) return py::none();
             return py::make_tuple(a->node, a->cards, a->mb, a->t_res, a->prio);
           }, py::call_guard<EngineGuard>())
      .def("reserve", &Engine::reserve, py::call_guard<EngineGuard>())
      .def("release", &Engine::release, py::call_guard<EngineGuard>())
      .def("has_pod", &Engine::has_pod, py::call_guard<EngineGuard>())
      .def("assignment",
           [](Engine& e, uint64_t pod) -> py::object {
             const Assignment* a = e.assignment(pod);
             if (!a) return py::none();
             return py::make_tuple(a->node, a->cards, a->mb);
           }, py::call_guard<EngineGuard>())
      .def("filter_node",
           [](Engine& e, const PodReq& r, int32_t idx) { return (int)e.filter_node(r, idx, nullptr, nullptr, nullptr); }, py::call_guard<EngineGuard>())
      .def("collect_max",
           [](Engine& e, const PodReq& r, const std::vector<int32_t>& idxs) {
             uint64_t mx[6];
             e.collect_max(r, idxs, mx);
             return py::make_tuple(mx[0], mx[1], mx[2], mx[3], mx[4], mx[5]);
           }, py::call_guard<EngineGuard>())
      .def("yoda_raw_score",
           [](Engine& e, const PodReq& r, int32_t idx, const std::array<uint64_t, 6>& mx) {
             return e.yoda_raw_score(r, idx, mx.data());
           }, py::call_guard<EngineGuard>())
      .def_static("normalize_yoda",
                  [](std::vector<int64_t> s) {
                    Engine::normalize_yoda(s);
                    return s;
                  })
      .def("select_gpus",
           [](Engine& e, const PodReq& r, int32_t idx) {
             std::vector<int32_t> out;
             int32_t q = 0;
             bool ok = e.select_gpus(r, idx, &out, &q);
             return py::make_tuple(ok, out, q);
           }, py::call_guard<EngineGuard>())
      .def("feasible_nodes",
           [](Engine& e, const PodReq& r, const std::vector<int32_t>& cand, bool exhaustive) {
             std::vector<int32_t> reasons;
             auto f = e.feasible_nodes(r, cand, &reasons, exhaustive);
             return py::make_tuple(f, reasons);
           },
           py::arg("req"), py::arg("candidates"), py::arg("exhaustive") = false, py::call_guard<EngineGuard>())
      .def("num_feasible_to_find", &Engine::num_feasible_to_find, py::call_guard<EngineGuard>())
      .def("score_nodes", &Engine::score_nodes, py::call_guard<EngineGuard>())
      // the six per-metric maxima (bandwidth, clock, core, free, power, total) over `nodes` —
      // what k_batch's record 1 exchanges (scripts/record1_reuse.py)
      .def("maxima",
           [](const Engine& e, const PodReq& r, const std::vector<int32_t>& nodes) {
             uint64_t mx[6];
             e.collect_max(r, nodes, mx);
             return std::vector<uint64_t>(mx, mx + 6);
           },
           py::call_guard<EngineGuard>())
      .def("schedule",
           [](Engine& e, uint64_t pod, const PodReq& r, bool assume, const std::vector<int32_t>& cand,
              const std::vector<int64_t>& extra) { return cycle_tuple(e.schedule(pod, r, assume, cand, extra)); },
           py::arg("pod"), py::arg("req"), py::arg("assume") = true,
           py::arg("candidates") = std::vector<int32_t>{}, py::arg("extra") = std::vector<int64_t>{}, py::call_guard<EngineGuard>())
      .def("schedule_batch",
           [](Engine& e, const std::vector<uint64_t>& pods, const std::vector<PodReq*>& reqs) {
             if (pods.size() != reqs.size()) throw std::invalid_argument("pods/reqs length mismatch");
             std::vector<const PodReq*> rr(reqs.begin(), reqs.end());
             std::vector<CycleResult> res;
             {
               // GIL first, then the engine lock: the lock is dropped before the GIL is
               // re-taken, so an event-loop thread waiting on the lock (holding the GIL)
               // cannot deadlock against this call
               py::gil_scoped_release nogil;
               EngineGuard g;
               res = e.schedule_batch(pods, rr);
             }
             py::list out;
             for (auto& r : res) out.append(cycle_tuple(r));
             return out;
           });

  // ---- native pod lane (lane.hpp). PodEvent objects are the _yoda_kube module's type
  // (pybind11 shares registered types across modules built with the same headers).
  py::class_<Lane>(m, "Lane")
      .def(py::init([](Engine& e, int batch, double bind_timeout, int sort_kind, bool events, bool events_v1,
                       double event_qps, int event_burst, int event_buffer, const std::string& host,
                       const std::string& name_prefix, int async_mode, int engine_delay_us, int spin_us,
                       double initial_backoff, double max_backoff, double unschedulable_flush) {
             LaneOptions o;
             o.initial_backoff_s = initial_backoff;
             o.max_backoff_s = max_backoff;
             o.unsched_flush_s = unschedulable_flush;
             o.async_mode = async_mode;
             o.engine_delay_us = engine_delay_us;
             o.spin_us = spin_us;
             o.batch = batch;
             o.bind_timeout_s = bind_timeout;
             o.sort_kind = sort_kind;
             o.events = events;
             o.events_v1 = events_v1;
             o.event_qps = event_qps;
             o.event_burst = event_burst;
             o.event_buffer = event_buffer;
             o.host = host;
             o.name_prefix = name_prefix;
             return std::make_unique<Lane>(&e, &g_engine_mu, std::move(o));
           }),
           py::arg("engine"), py::arg("batch") = 256, py::arg("bind_timeout") = 30.0, py::arg("sort_kind") = 0,
           py::arg("events") = true, py::arg("events_v1") = true, py::arg("event_qps") = 50.0,
           py::arg("event_burst") = 300, py::arg("event_buffer") = 1000, py::arg("host") = "localhost",
           py::arg("name_prefix") = "00000000", py::arg("async_mode") = 1,
           py::arg("engine_delay_us") = 0, py::arg("spin_us") = 0, py::arg("initial_backoff") = 1.0,
           py::arg("max_backoff") = 10.0, py::arg("unschedulable_flush") = 60.0, py::keep_alive<1, 2>())
      .def("sink_ptr", [](Lane& l) { return (uintptr_t) static_cast<yk::PodSink*>(&l); })
      .def("set_port", [](Lane& l, uintptr_t p) { l.set_port(reinterpret_cast<yk::PodPort*>(p)); })
      // the profile's engine configuration is the engine's current one (the caller applied it)
      .def("set_profile",
           [](Lane& l, Engine& e, const std::string& name, bool enabled, int flag_mask, bool annotate,
              int64_t preempt_above, const py::list& gate_terms, bool claims_ok, bool vol_node, bool vol_zone,
              bool vol_limits) {
             Lane::Profile p;
             p.vol_limits = vol_limits;
             p.preempt_above = preempt_above;
             p.claims_ok = claims_ok;
             p.vol_node = vol_node;
             p.vol_zone = vol_zone;
             for (auto t : gate_terms) p.gate_terms.push_back(match_term(t));
             p.name = name;
             p.enabled = enabled;
             p.flag_mask = flag_mask;
             p.annotate = annotate;
             {
               EngineGuard g;
               p.cfg = e.config();
             }
             l.set_profile(p);
           },
           py::arg("engine"), py::arg("name"), py::arg("enabled"), py::arg("flag_mask"), py::arg("annotate"),
           py::arg("preempt_above") = INT64_MIN, py::arg("gate_terms") = py::list(), py::arg("claims_ok") = false,
           py::arg("vol_node") = false, py::arg("vol_zone") = false, py::arg("vol_limits") = false)
      // [(key, node terms | None, zone terms | None)], each terms [[(key, op, [values])]]
      .def("update_claims",
           [](Lane& l, Engine& e, bool reset, const py::list& add, const std::vector<std::string>& remove) {
             std::vector<std::pair<std::string, Lane::ClaimConsP>> a;
             {
               EngineGuard g;                  // interning
               for (auto item : add) {
                 auto t = item.cast<py::tuple>();
                 Lane::ClaimConsP cons;
                 if (!t[1].is_none() || !t[2].is_none()) {
                   auto c = std::make_shared<Lane::ClaimCons>();
                   if (!t[1].is_none()) {
                     c->has_node = true;
                     for (auto term : t[1]) c->node.push_back(make_term(e, term.cast<py::list>()));
                   }
                   if (!t[2].is_none()) {
                     c->has_zone = true;
                     for (auto term : t[2]) c->zone.push_back(make_term(e, term.cast<py::list>()));
                   }
                   cons = std::move(c);
                 }
                 a.emplace_back(t[0].cast<std::string>(), std::move(cons));
               }
             }
             l.update_claims(reset, std::move(a), remove);
           },
           py::arg("engine"), py::arg("reset"), py::arg("add"), py::arg("remove"))
      .def("set_inert_claims", &Lane::set_inert_claims, py::arg("keys"),
           "PersistentVolumeClaims (namespace/name) whose pods the profiles with claims_ok may run")
      .def("update_inert_claims", &Lane::update_inert_claims, py::arg("add"), py::arg("remove"),
           "add / remove claims of the inert set")
      .def("set_gates",
           [](Lane& l, const std::string& name, const py::list& gate_terms) {
             std::vector<MatchTerm> v;
             for (auto t : gate_terms) v.push_back(match_term(t));
             return l.set_gates(name, std::move(v));
           },
           py::arg("name"), py::arg("gate_terms"),
           "replace a declared profile's selector gates only (no engine-config snapshot)")
      .def("set_active", &Lane::set_active)
      .def("move", &Lane::move, py::arg("node") = -1,
           "move request: -1 moves every parked lane pod; a node index is a queueing hint for that node")
      .def("set_node_cards", &Lane::set_node_cards, py::arg("node"), py::arg("vis"))
      .def("remove_node_cards", &Lane::remove_node_cards)
      .def("fileno", &Lane::fileno)
      // ([(type, PodEvent, old PodEvent | None)], [handoff], moves)
      // handoff = (kind, PodEvent, profile, cycle tuple, status, message, t_enqueue, t_cycle, attempts)
      .def("drain",
           [](Lane& l) {
             std::vector<Lane::Fwd> fwd;
             std::vector<Lane::Handoff> hand;
             uint64_t moves = 0;
             l.drain(&fwd, &hand, &moves);
             static py::object* types = new py::object[3]{py::str("ADDED"), py::str("MODIFIED"), py::str("DELETED")};
             py::list f;
             for (auto& x : fwd)
               f.append(py::make_tuple(types[x.type == 'A' ? 0 : x.type == 'M' ? 1 : 2], py::cast(x.ev),
                                       x.old ? py::cast(x.old) : py::none()));
             py::list h;
             for (auto& x : hand)
               h.append(py::make_tuple(x.kind, py::cast(x.ev), x.profile, cycle_tuple(x.res), x.status,
                                       py::bytes(x.msg), x.t_enqueue, x.t_cycle, x.attempts));
             return py::make_tuple(f, h, moves);
           })
      .def("relist",
           [](Lane& l, std::vector<std::shared_ptr<yk::PodEv>> items) {
             std::vector<Lane::Fwd> fwd;
             {
               py::gil_scoped_release nogil;
               fwd = l.relist(std::move(items));
             }
             static py::object* types = new py::object[3]{py::str("ADDED"), py::str("MODIFIED"), py::str("DELETED")};
             py::list f;
             for (auto& x : fwd)
               f.append(py::make_tuple(types[x.type == 'A' ? 0 : x.type == 'M' ? 1 : 2], py::cast(x.ev),
                                       x.old ? py::cast(x.old) : py::none()));
             return f;
           })
      .def("lookup",
           [](Lane& l, const std::string& key) -> py::object {
             bool owned = false;
             std::shared_ptr<yk::PodEv> ev;
             {
               py::gil_scoped_release nogil;
               ev = l.lookup(key, &owned);
             }
             if (!ev) return py::none();
             return py::make_tuple(py::cast(ev), owned);
           })
      .def("keys", &Lane::keys, py::call_guard<py::gil_scoped_release>())
      // a lane-owned pod by its engine ledger id: (event, node name) or None
      .def("lookup_id",
           [](Lane& l, uint64_t id) -> py::object {
             std::string node;
             std::shared_ptr<yk::PodEv> ev;
             {
               py::gil_scoped_release nogil;
               ev = l.lookup_id(id, &node);
             }
             if (!ev) return py::none();
             return py::make_tuple(py::cast(ev), node);
           })
      .def("__len__", &Lane::store_size, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("scheduled", [](Lane& l) { return l.scheduled_.load(std::memory_order_relaxed); })
      .def("set_watermark", &Lane::set_watermark, "signal the eventfd once this many Bindings are acknowledged")
      .def("stats",
           [](Lane& l) {
             LaneStats s = l.stats();
             py::dict d;
             d["admitted"] = s.admitted;
             d["scheduled"] = s.scheduled;
             d["unschedulable"] = s.unschedulable;
             d["bind_errors"] = s.bind_errors;
             d["stale_retries"] = s.stale_retries;
             d["forwarded"] = s.forwarded;
             d["released"] = s.released;
             d["batches"] = s.batches;
             d["confirmed"] = s.confirmed;
             d["events_recorded"] = s.events_recorded;
             d["events_dropped"] = s.events_dropped;
             d["events_written"] = s.events_written;
             d["event_errors"] = s.event_errors;
             d["lost_answers_kept"] = s.lost_answers_kept;
             d["queued"] = s.queued;
             d["inflight"] = s.inflight;
             d["binding"] = s.binding;
             d["owned"] = s.owned;
             d["parked"] = s.parked;
             d["backoff"] = s.backoff;
             d["native_failed"] = s.native_failed;
             d["moved"] = s.moved;
             d["retried"] = s.retried;
             d["status_patches"] = s.status_patches;
             d["status_patch_errors"] = s.status_patch_errors;
             d["status_patches_skipped"] = s.status_patches_skipped;
             d["census_calls"] = s.census_calls;
             d["census_entries"] = s.census_entries;
             d["census_s"] = s.census_s;
             d["engine_s"] = s.engine_s;
             d["left_in_flight"] = s.left_in_flight;
             d["engine_pods"] = s.engine_pods;
             d["engine_cpu_s"] = s.engine_cpu_s;
             d["lock_wait_s"] = s.lock_wait_s;
             d["handoff_s"] = s.handoff_s;
             d["return_s"] = s.return_s;
             d["idle_queued_s"] = s.idle_queued_s;
             d["async_runs"] = s.async_runs;
             py::dict bp;
             for (const auto& kv : s.by_profile) bp[py::str(kv.first)] = py::make_tuple(kv.second.first, kv.second.second);
             d["by_profile"] = bp;
             return d;
           })
      // [(t_pick, t_worker_start, t_worker_end, t_done, pods)] of the runs since the last call
      // (monotonic seconds; worker times 0 for runs the lane thread ran itself)
      .def("run_log",
           [](Lane& l) {
             py::list out;
             for (const auto& r : l.run_log()) out.append(py::make_tuple(r.t_pick, r.t_wstart, r.t_wend, r.t_done, r.pods));
             return out;
           })
      .def("pause", &Lane::pause, py::call_guard<py::gil_scoped_release>())
      // (full, [(id, add, PodEvent | None, node, cards)])
      .def("changes",
           [](Lane& l) {
             bool full = false;
             std::vector<Lane::Change> ch;
             {
               py::gil_scoped_release nogil;
               ch = l.changes(&full);
             }
             py::list out;
             for (auto& c : ch)
               out.append(py::make_tuple(c.id, c.add, c.ev ? py::cast(c.ev) : py::none(), c.node, c.cards));
             return py::make_tuple(full, out);
           })
      .def("stop_log", &Lane::stop_log, "turn the change log off (the Python mirror was dropped)",
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("log_on", [](Lane& l) {
        py::gil_scoped_release nogil;
        return l.log_on();
      })
      // queries: [[term, ...], ...] (a pod counts for a query when it matches all its terms);
      // term = (namespaces | None, nothing, [(key, value)], [(key, op, [values])]) → [{node: count}]
      .def("count_matching",
           [](Lane& l, const py::list& queries, bool skip_deleting) {
             std::vector<std::vector<MatchTerm>> qs;
             for (auto q : queries) {
               std::vector<MatchTerm> terms;
               for (auto t : q) terms.push_back(match_term(t));
               qs.push_back(std::move(terms));
             }
             std::vector<std::unordered_map<std::string, int32_t>> out;
             {
               py::gil_scoped_release nogil;
               out = l.count_matching(qs, skip_deleting);
             }
             py::list res;
             for (auto& m : out) {
               py::dict d;
               for (auto& kv : m) d[py::str(kv.first)] = kv.second;
               res.append(d);
             }
             return res;
           },
           py::arg("queries"), py::arg("skip_deleting") = false)
      .def("stop_census", &Lane::stop_census, "drop the selector census (no Python cycle queries it now)",
           py::call_guard<py::gil_scoped_release>())
      .def("take_e2e", &Lane::take_e2e)
      .def("take_pod_latency", &Lane::take_pod_latency)
      .def("wait_idle", &Lane::wait_idle, py::arg("timeout") = 5.0, py::call_guard<py::gil_scoped_release>())
      .def("close", &Lane::close, py::call_guard<py::gil_scoped_release>());

  py::class_<BatchWorker>(m, "BatchWorker")
      .def(py::init([](Engine& e) { return std::make_unique<BatchWorker>(&e); }), py::keep_alive<1, 2>())
      .def("fileno", &BatchWorker::fileno)
      .def("submit",
           [](BatchWorker& w, std::vector<uint64_t> pods, const std::vector<PodReq*>& reqs) {
             return w.submit(std::move(pods), std::vector<const PodReq*>(reqs.begin(), reqs.end()));
           },
           "queue a batch (the caller keeps the PodReq objects alive until it is collected); returns its id")
      .def("collect",
           [](BatchWorker& w) {
             auto jobs = w.take_done();
             py::list out;
             for (auto& j : jobs) {
               if (!j->err.empty()) {
                 out.append(py::make_tuple(j->id, py::none(), j->err, j->t0, j->t1));
                 continue;
               }
               py::list res;
               for (auto& r : j->res) res.append(cycle_tuple(r));
               out.append(py::make_tuple(j->id, res, py::none(), j->t0, j->t1));
             }
             return out;
           },
           "finished batches: [(id, results | None, error | None, t_start, t_end)]")
      .def_property_readonly("pending", &BatchWorker::pending)
      .def("close", [](BatchWorker& w) {
        py::gil_scoped_release nogil;
        w.close();
      });
}
