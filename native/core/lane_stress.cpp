// Stress / profiling driver for the native pod lane (lane.hpp), standalone: a fake
// transport port answers every Binding and feeds back the watch echo, a producer thread plays
// the transport I/O thread (ADDED bursts, echoes, DELETED), and the driver checks the ledger
// after every burst. Built with sanitizers by scripts/sanitize.py (TSan: lane thread vs I/O
// thread vs the caller) and used for per-pod cost measurements (lane thread CPU / pod).
//
//   lane_stress [bursts] [pods_per_burst] [batch]
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <time.h>

#include "engine.hpp"
#include "lane.hpp"
#include "project.hpp"

using namespace yoda;

namespace {

std::string pod_json(const std::string& name, const std::string& uid, const std::string& node, int i, int rv) {
  std::string labels = "\"scv/memory\":\"" + std::to_string(64 * (1 + i % 8)) + "\"";
  if (i % 3 == 0) labels += ",\"scv/number\":\"" + std::to_string(1 + i % 4) + "\"";
  std::string s = "{\"apiVersion\":\"v1\",\"kind\":\"Pod\",\"metadata\":{\"name\":\"" + name +
                  "\",\"namespace\":\"default\",\"uid\":\"" + uid + "\",\"resourceVersion\":\"" + std::to_string(rv) +
                  "\",\"labels\":{" + labels + "}},\"spec\":{\"schedulerName\":\"yoda-scheduler\",";
  if (!node.empty()) s += "\"nodeName\":\"" + node + "\",";
  // every pod mounts the claim "data" (inert: the profile admits it, see run_mode)
  s += "\"volumes\":[{\"name\":\"d\",\"persistentVolumeClaim\":{\"claimName\":\"data\"}}],";
  // and a host port of its own (NodePorts: the ledger's per-node port maps grow and drain)
  s += "\"containers\":[{\"name\":\"main\",\"image\":\"x\",\"ports\":[{\"containerPort\":80,\"hostPort\":" +
       std::to_string(10000 + i) + "}],\"resources\":{\"requests\":{\"cpu\":\"100m\","
       "\"memory\":\"128Mi\"}}}]},\"status\":{\"phase\":\"Pending\"}}";
  return s;
}

std::shared_ptr<yk::PodEv> ev_of(const std::string& json) {
  auto pe = std::make_shared<yk::PodEv>();
  yk::project_pod_text(json, pe->p);
  pe->raw = json;
  return pe;
}

// The "apiserver + I/O thread": answers Bindings 201 and queues the echo.
class FakePort : public yk::PodPort {
 public:
  void bind_native(std::vector<yk::BindSpec>&& binds, const std::vector<uint64_t>& tags, double,
                   yk::PodSink* sink) override {
    std::lock_guard<std::mutex> g(mu);
    for (size_t k = 0; k < binds.size(); ++k) q.push_back({tags[k], sink, std::move(binds[k])});
    cv.notify_one();
  }
  void request_native(const std::string&, const std::string&, std::string&&, bool, double, uint64_t tag,
                      yk::PodSink* sink, const char*) override {
    std::lock_guard<std::mutex> g(mu);
    events.push_back({tag, sink});
    cv.notify_one();
  }
  // as the transport: the events the lane is done with are dropped on the I/O thread
  void recycle(std::vector<std::shared_ptr<yk::PodEv>>&& d) override {
    std::lock_guard<std::mutex> g(mu);
    for (auto& x : d) dead.push_back(std::move(x));
    d.clear();
  }
  std::vector<std::shared_ptr<yk::PodEv>> dead;
  struct B {
    uint64_t tag;
    yk::PodSink* sink;
    yk::BindSpec spec;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::deque<B> q;
  std::deque<std::pair<uint64_t, yk::PodSink*>> events;
  uint64_t bound = 0;
  int rv = 1000000;
};

double cpu_of(pthread_t) { return 0; }

}  // namespace

// One lane over `bursts` bursts of `per` pods; async_mode / spin_us as in LaneOptions (2 = every
// run on the engine worker, the device-scorer path's threading without a device).
int run_mode(int bursts, int per, int batch, int async_mode, int spin_us) {
  std::recursive_mutex emu;
  Engine e(false, 1);
  {
    int idx = e.upsert_node("node-0");
    e.set_node_meta(idx, false, {}, {}, 192000, (int64_t)2 << 40, 100000);
    std::vector<Card> cs(8);
    for (int g = 0; g < 8; ++g) {
      cs[g].total_mb = cs[g].free_mb = 294912;
      cs[g].clock = 2400;
      cs[g].bandwidth = 8000;
      cs[g].core = 256;
      cs[g].power = 1400;
      cs[g].phys = g;
      cs[g].numa = g >= 4;
    }
    e.set_cards(idx, cs, 8, 8 * 294912, 8 * 294912, false, 0);
  }
  e.set_filters(e.filters() | F_NODE_PORTS);
  EngineConfig cfg = e.config();
  LaneOptions o;
  o.batch = batch;
  o.async_mode = async_mode;
  o.spin_us = spin_us;
  Lane lane(&e, &emu, o);
  FakePort port;
  lane.set_port(&port);
  Lane::Profile pr;
  pr.name = "yoda-scheduler";
  pr.enabled = true;
  pr.cfg = cfg;
  pr.flag_mask = yk::PF_CLAIMS;
  pr.claims_ok = true;
  lane.set_profile(pr);
  lane.set_inert_claims({"default/data"});
  lane.set_node_cards("node-0", {{"0", "u0"}, {"1", "u1"}, {"2", "u2"}, {"3", "u3"},
                                 {"4", "u4"}, {"5", "u5"}, {"6", "u6"}, {"7", "u7"}});
  lane.set_active(true);

  // the fake I/O thread: answers and echoes
  std::atomic<bool> stop{false};
  std::thread io([&] {
    for (;;) {
      std::deque<FakePort::B> q;
      std::deque<std::pair<uint64_t, yk::PodSink*>> evs;
      {
        std::unique_lock<std::mutex> lk(port.mu);
        port.cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(5),
                           [&] { return stop.load() || !port.q.empty() || !port.events.empty(); });
        if (stop.load() && port.q.empty()) return;
        q.swap(port.q);
        evs.swap(port.events);
        port.dead.clear();                 // freed here, off the lane thread
      }
      std::vector<yk::PodSink::Answer> ans;
      for (auto& x : evs) ans.push_back({x.first, 201, std::string()});
      for (auto& b : q) ans.push_back({b.tag, 201, std::string()});
      if (!ans.empty()) lane.on_answers(ans);
      std::vector<yk::WatchEvent> echo;
      for (auto& b : q) {
        yk::WatchEvent w;
        w.type = 'M';
        const int rv = ++port.rv;
        w.rv = std::to_string(rv);
        w.pod = ev_of(pod_json(b.spec.name, b.spec.uid, b.spec.node, 0, rv));
        echo.push_back(std::move(w));
        port.bound++;
      }
      if (!echo.empty()) lane.on_pod_events(1, echo);
    }
  });

  // the Python thread re-sending the inert-claims set while the lane admits (TSan: prof_mu_ and
  // the lane thread's kClaims apply); "default/data" stays in it, so every pod stays admissible
  std::thread churn([&] {
    for (int k = 0; !stop.load(); ++k) {
      if (k % 2) lane.set_inert_claims({"default/data", "default/x" + std::to_string(k % 4)});
      else lane.update_inert_claims({"default/y" + std::to_string(k % 3)}, {"default/y" + std::to_string((k + 1) % 3)});
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  });

  // pre-build the bursts' ADDED / DELETED events (the transport's decode cost is not the lane's)
  std::vector<std::vector<yk::WatchEvent>> adds(bursts), dels(bursts);
  int rv = 1;
  for (int b = 0; b < bursts; ++b) {
    for (int i = 0; i < per; ++i) {
      const std::string name = "b" + std::to_string(b) + "-" + std::to_string(i);
      const std::string uid = "uid-" + name;
      yk::WatchEvent a;
      a.type = 'A';
      a.rv = std::to_string(++rv);
      a.pod = ev_of(pod_json(name, uid, "", i, rv));
      adds[b].push_back(std::move(a));
      yk::WatchEvent d;
      d.type = 'D';
      d.rv = std::to_string(++rv);
      d.pod = ev_of(pod_json(name, uid, "node-0", i, rv));
      dels[b].push_back(std::move(d));
    }
  }
  clockid_t lane_clock;
  int fails = 0;
  double lane_cpu = 0, wall = 0;
  for (int b = 0; b < bursts; ++b) {
    const auto t0 = std::chrono::steady_clock::now();
    // chunks of 128 events, as the transport hands them over
    for (size_t k = 0; k < adds[b].size(); k += 128) {
      std::vector<yk::WatchEvent> chunk(std::make_move_iterator(adds[b].begin() + k),
                                        std::make_move_iterator(adds[b].begin() + std::min(adds[b].size(), k + 128)));
      lane.on_pod_events(1, chunk);
    }
    while (lane.scheduled_.load() < (uint64_t)per * (b + 1)) std::this_thread::sleep_for(std::chrono::microseconds(50));
    lane.wait_idle(10);
    wall += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    {
      std::lock_guard<std::recursive_mutex> g(emu);
      if (e.ledger_size() != (size_t)per) {
        fprintf(stderr, "burst %d: ledger %zu != %d\n", b, e.ledger_size(), per);
        fails++;
      }
    }
    for (size_t k = 0; k < dels[b].size(); k += 128) {
      std::vector<yk::WatchEvent> chunk(std::make_move_iterator(dels[b].begin() + k),
                                        std::make_move_iterator(dels[b].begin() + std::min(dels[b].size(), k + 128)));
      lane.on_pod_events(1, chunk);
    }
    lane.wait_idle(10);
    for (int spin = 0; spin < 2000; ++spin) {
      {
        std::lock_guard<std::recursive_mutex> g(emu);
        if (e.ledger_size() == 0) break;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    std::lock_guard<std::recursive_mutex> g(emu);
    if (e.ledger_size() != 0) {
      fprintf(stderr, "burst %d: ledger %zu after deletes\n", b, e.ledger_size());
      fails++;
    }
  }
  (void)lane_clock;
  (void)lane_cpu;
  LaneStats st = lane.stats();
  stop = true;
  port.cv.notify_all();
  io.join();
  churn.join();
  lane.close();
  printf("{\"async_mode\": %d, \"spin_us\": %d, \"bursts\": %d, \"pods\": %d, \"scheduled\": %llu, "
         "\"confirmed\": %llu, \"released\": %llu, \"batches\": %llu, \"async_runs\": %llu, "
         "\"us_per_pod_wall\": %.2f, \"fails\": %d}\n",
         async_mode, spin_us, bursts, per, (unsigned long long)st.scheduled, (unsigned long long)st.confirmed,
         (unsigned long long)st.released, (unsigned long long)st.batches, (unsigned long long)st.async_runs,
         wall / (bursts * per) * 1e6, fails);
  if (async_mode == 2 && st.async_runs == 0) fails++;
  return fails;
}

int main(int argc, char** argv) {
  const int bursts = argc > 1 ? atoi(argv[1]) : 20;
  const int per = argc > 2 ? atoi(argv[2]) : 1000;
  const int batch = argc > 3 ? atoi(argv[3]) : 256;
  // the lane thread placing inline, then runs on the engine worker with both threads spinning
  int fails = run_mode(bursts, per, batch, 1, 0);
  fails += run_mode(bursts, per, batch, 2, 50);
  return fails ? 1 : 0;
}
