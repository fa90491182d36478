// Randomised stress driver for the native engine, built with sanitizers by
// scripts/sanitize.py (ASan+UBSan and TSan variants; SURVEY §5 race detection row).
// Exercises node churn, Scv updates, schedule/reserve/release and the parallel filter
// (ThreadPool) and checks the ledger invariants after every step.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "engine.hpp"

using namespace yoda;

static int fail(const char* what, int step) {
  fprintf(stderr, "invariant violated at step %d: %s\n", step, what);
  return 1;
}

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? atoi(argv[1]) : 600;
  const int steps = argc > 2 ? atoi(argv[2]) : 6000;
  const int threads = argc > 3 ? atoi(argv[3]) : 4;
  std::mt19937_64 rng(12345);
  Engine e(false, threads);
  e.set_percentage_of_nodes_to_score(100);
  auto make_cards = [&](int n) {
    std::vector<Card> cs(n);
    for (int g = 0; g < n; ++g) {
      cs[g].total_mb = 294912;
      cs[g].free_mb = 294912 - rng() % 100000;
      cs[g].clock = (rng() & 1) ? 2400 : 2200;
      cs[g].bandwidth = 8000;
      cs[g].core = 256;
      cs[g].power = 1400;
      cs[g].healthy = (rng() % 50) != 0;
      cs[g].phys = g;
      cs[g].numa = g >= n / 2;
      cs[g].occ_q = rng() % 10000;
    }
    return cs;
  };
  for (int i = 0; i < nodes; ++i) {
    int idx = e.upsert_node("n" + std::to_string(i));
    e.set_node_meta(idx, false, {}, {}, 192000, (int64_t)2 << 40, 100000);
    auto cs = make_cards(8);
    e.set_cards(idx, cs, 8, 0, 8 * 294912, false, 0);
  }
  std::vector<uint64_t> live;
  uint64_t next_pod = 1;
  for (int s = 0; s < steps; ++s) {
    const int op = rng() % 100;
    if (op < 60) {
      PodReq r;
      r.has_number = rng() % 3 == 0;
      r.number = r.has_number ? 1 + rng() % 8 : 1;
      r.has_memory = true;
      r.memory = 1024 * (1 + rng() % 32);
      r.cpu_m = 100;
      r.mem = 1 << 28;
      r.pod_priority = (int64_t)(rng() % 4);
      CycleResult res = e.schedule(next_pod, r, true, {}, {});
      if (res.node >= 0) live.push_back(next_pod);
      ++next_pod;
    } else if (op < 85 && !live.empty()) {
      size_t k = rng() % live.size();
      if (!e.release(live[k])) return fail("release of a live pod failed", s);
      live[k] = live.back();
      live.pop_back();
    } else if (op < 88) {
      // DefaultPreemption what-if: detaches / re-attaches victims on many nodes; the ledger
      // invariants below must hold exactly afterwards
      PodReq r;
      r.has_number = true;
      r.number = 1 + rng() % 8;
      r.has_memory = true;
      r.memory = 100000 + rng() % 190000;
      r.pod_priority = 5;
      PreemptArgs a;
      a.priority = 5;
      a.min_abs = 1 + (int32_t)(rng() % 50);
      PreemptResult out;
      e.preempt(r, a, &out);
      if (out.node >= 0 && out.victims.empty()) return fail("preemption without victims", s);
    } else if (op < 95) {
      int idx = (int)(rng() % e.num_nodes());
      if (e.node(idx).alive) e.set_cards(idx, make_cards(8), 8, 0, 8 * 294912, false, (double)s);
    } else {
      int idx = (int)(rng() % e.num_nodes());
      if (e.node(idx).alive && rng() % 4 == 0) {
        // node removal drops its reservations
        std::vector<uint64_t> keep;
        for (uint64_t p : live) {
          const Assignment* a = e.assignment(p);
          if (a && a->node != idx) keep.push_back(p);
        }
        e.remove_node(idx);
        live.swap(keep);
        int ni = e.upsert_node("r" + std::to_string(s));
        e.set_node_meta(ni, false, {}, {}, 192000, (int64_t)2 << 40, 100000);
        e.set_cards(ni, make_cards(8), 8, 0, 8 * 294912, false, 0);
      }
    }
    // invariants: ledger size, per-card reserved == Σ assignments, pending <= reserved
    if (e.ledger_size() != live.size()) return fail("ledger size", s);
    if (s % 97 == 0) {
      std::vector<std::vector<uint64_t>> want(e.num_nodes());
      for (int i = 0; i < e.num_nodes(); ++i) want[i].assign(e.node(i).cards.size(), 0);
      for (uint64_t p : live) {
        const Assignment* a = e.assignment(p);
        if (!a) return fail("missing assignment", s);
        for (int c : a->cards) want[a->node][c] += a->mb;
      }
      for (int i = 0; i < e.num_nodes(); ++i) {
        const Node& n = e.node(i);
        if (!n.alive) continue;
        for (size_t c = 0; c < n.cards.size(); ++c) {
          if (n.cards[c].reserved_mb != want[i][c]) return fail("reserved_mb mismatch", s);
          if (n.cards[c].pending_mb > n.cards[c].reserved_mb) return fail("pending > reserved", s);
        }
      }
    }
  }
  printf("stress ok: %d nodes, %d steps, %zu live pods, %llu cycles\n", nodes, steps, live.size(),
         (unsigned long long)e.cycles());
  return 0;
}
