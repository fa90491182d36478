// Sanitizer driver for the sniffer's host code (SURVEY §5 race/sanitizer row): fuzzes
// to_json with random samples (hostile strings: quotes, backslashes, control and
// invalid UTF-8 bytes, NaN/Inf rates) and, when a driver is present, runs a few real
// amd-smi sample rounds. Prints the last JSON document so the caller can parse it.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

#include "collector.hpp"

static std::string rand_str(std::mt19937_64& rng) {
  static const char alpha[] = "abcXYZ0123456789:._-\"\\ /";
  std::string s;
  int n = (int)(rng() % 24);
  for (int i = 0; i < n; ++i) {
    uint64_t r = rng() % 10;
    if (r == 0) s += (char)(rng() % 0x20);              // control
    else if (r == 1) s += (char)(0x80 + rng() % 0x80);  // stray high byte
    else if (r == 2) s += "\xc3\xa9";                   // valid 2-byte UTF-8
    else s += alpha[rng() % (sizeof(alpha) - 1)];
  }
  return s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  std::mt19937_64 rng(42);
  std::string last;
  for (int it = 0; it < iters; ++it) {
    std::vector<yoda::GpuSample> v(it == iters - 1 ? 8 : (size_t)(rng() % 9));
    for (size_t g = 0; g < v.size(); ++g) {
      yoda::GpuSample& s = v[g];
      s.index = (int)g;
      s.bdf = rand_str(rng);
      s.model = rand_str(rng);
      s.vram_total_mb = (uint32_t)rng();
      s.ecc_uncorrectable = rng();
      s.t = (rng() % 7 == 0) ? NAN : 1.7e9 + (double)(rng() % 1000000) / 1e3;
      s.compute_partition = rand_str(rng);
      s.errors.assign(rng() % 3, rand_str(rng));
      for (int l = 0, nl = (int)(rng() % 8); l < nl; ++l) {
        yoda::LinkSample x;
        x.peer_bdf = rand_str(rng);
        x.read_kbps = (rng() % 5 == 0) ? INFINITY : (double)(rng() % 100000);
        x.load = (rng() % 5 == 0) ? NAN : 0.5;
        s.links.push_back(x);
      }
    }
    last = yoda::to_json(v);
  }
  yoda::Collector c;
  std::string err;
  int sampled = 0;
  if (c.init(&err)) {
    for (int r = 0; r < rounds; ++r) {
      std::string js = yoda::to_json(c.sample());
      if (js.size() < 2) return 3;
      ++sampled;
    }
    c.shutdown();
  }
  fprintf(stderr, "sniffer stress: %d fuzz iterations, %d amd-smi rounds (%s)\n", iters, sampled,
          sampled ? "driver present" : err.c_str());
  printf("%s\n", last.c_str());
  return 0;
}
