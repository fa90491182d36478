// Allocation guard for the engine ledger: counts every operator new the
// engine makes while pods of known templates are reserved and released. Built and run by
// tests/test_engine_alloc.py; prints one JSON line.
//
// Phases, each after a warm-up that lets the ledger, slab, label-set table and node indices
// reach their steady-state size:
//   churn  — one pod at a time: reserve then release, 10 000 fresh pod ids
//   burst  — the bench pattern: 1000 pods of a few templates reserved, then all released, ×10
// Both must allocate nothing: the slab reuses entries (and their vectors' capacity), label sets
// are interned once per template, zero-count node index entries stay until a sweep.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <new>
#include <string>
#include <vector>

#include "engine.hpp"

static std::atomic<long> g_news{0};
static std::atomic<bool> g_count{false};

void* operator new(std::size_t n) {
  if (g_count.load(std::memory_order_relaxed)) g_news.fetch_add(1, std::memory_order_relaxed);
  if (void* p = std::malloc(n ? n : 1)) return p;
  throw std::bad_alloc();
}
void* operator new[](std::size_t n) { return operator new(n); }
void operator delete(void* p) noexcept { std::free(p); }
void operator delete[](void* p) noexcept { std::free(p); }
void operator delete(void* p, std::size_t) noexcept { std::free(p); }
void operator delete[](void* p, std::size_t) noexcept { std::free(p); }

using namespace yoda;

int main(int argc, char** argv) {
  const int churn = argc > 1 ? atoi(argv[1]) : 10000;
  const int bursts = argc > 2 ? atoi(argv[2]) : 10;
  Engine e(false, 1);
  e.set_fixed_now(1000.0);
  const int32_t node = e.upsert_node("n0");
  e.set_node_meta(node, false, {{e.intern("kubernetes.io/hostname"), e.intern("n0")}}, {}, 192000,
                  (int64_t)2 << 40, 100000);
  std::vector<Card> cards(8);
  for (int g = 0; g < 8; ++g) {
    cards[g].total_mb = cards[g].free_mb = 294912;
    cards[g].clock = 2400;
    cards[g].phys = g;
  }
  e.set_cards(node, cards, 8, 8 * 294912, 8 * 294912, false, 0);

  // templates: the bench mix (scv/memory, scv/number) plus an app / pod-template-hash pair
  std::vector<PodReq> tmpl(4);
  for (int t = 0; t < 4; ++t) {
    PodReq& r = tmpl[t];
    r.ns = e.intern("default");
    r.has_memory = true;
    r.memory = 1024 * (t + 1);
    r.has_number = t == 3;
    r.number = t == 3 ? 2 : 1;
    r.cpu_m = 100;
    r.mem = 128 << 20;
    r.labels = {{e.intern("app"), e.intern("web" + std::to_string(t))},
                {e.intern("pod-template-hash"), e.intern("5d8f7c9b4" + std::to_string(t))},
                {e.intern("scv/memory"), e.intern(std::to_string(1024 * (t + 1)))}};
    std::sort(r.labels.begin(), r.labels.end());
  }
  const std::vector<int32_t> one = {0}, two = {0, 1};
  uint64_t pid = 1;
  auto reserve = [&](int t) { return e.reserve(pid++, tmpl[t], node, t == 3 ? two : one); };

  // ---- churn
  for (int t = 0; t < 4; ++t) {
    reserve(t);
    e.release(pid - 1);
  }
  g_news = 0;
  g_count = true;
  for (int i = 0; i < churn; ++i) {
    if (!reserve(i & 3)) return 2;
    if (!e.release(pid - 1)) return 3;
  }
  g_count = false;
  const long churn_news = g_news.load();

  // ---- bursts
  std::vector<uint64_t> held;
  held.reserve(1000);
  auto burst = [&]() {
    held.clear();
    for (int i = 0; i < 1000; ++i) {
      held.push_back(pid);
      if (!reserve(i % 4)) return false;
    }
    for (uint64_t p : held)
      if (!e.release(p)) return false;
    return true;
  };
  if (!burst() || !burst()) return 4;   // warm-up: the ledger map and the slab reach 1000 entries
  g_news = 0;
  g_count = true;
  for (int b = 0; b < bursts; ++b)
    if (!burst()) return 5;
  g_count = false;
  const long burst_news = g_news.load();
  printf("{\"churn_cycles\": %d, \"churn_allocs\": %ld, \"bursts\": %d, \"burst_allocs\": %ld, \"ledger\": %zu, "
         "\"labsets\": %zu}\n",
         churn, churn_news, bursts, burst_news, e.ledger_size(), e.labsets_used());
  return 0;
}
