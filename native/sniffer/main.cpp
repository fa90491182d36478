// yoda-sniffer: standalone amd-smi collector. Prints one JSON array of per-GPU samples per
// line on stdout (`--interval S` repeats; `--count N` stops after N samples). The Python
// publisher (yoda_scheduler_amd.sniffer) turns samples into Scv status updates; this
// binary is also what the DaemonSet runs for ad-hoc inspection.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "build_id.h"
#include "collector.hpp"

int main(int argc, char** argv) {
  double interval = 0;
  long count = 1;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--interval") && i + 1 < argc) {
      interval = atof(argv[++i]);
      count = -1;
    } else if (!strcmp(argv[i], "--count") && i + 1 < argc) {
      count = atol(argv[++i]);
    } else if (!strcmp(argv[i], "--build-id")) {
      printf("%s\n", YODA_BUILD_ID);
      return 0;
    } else if (!strcmp(argv[i], "-h") || !strcmp(argv[i], "--help")) {
      printf("usage: yoda-sniffer [--interval SECONDS] [--count N]\n");
      return 0;
    }
  }
  yoda::Collector c;
  std::string err;
  if (!c.init(&err)) {
    fprintf(stderr, "yoda-sniffer: %s\n", err.c_str());
    return 2;
  }
  for (long n = 0; count < 0 || n < count; ++n) {
    if (n) std::this_thread::sleep_for(std::chrono::duration<double>(interval > 0 ? interval : 1.0));
    std::string js = yoda::to_json(c.sample());
    printf("%s\n", js.c_str());
    fflush(stdout);
  }
  return 0;
}
