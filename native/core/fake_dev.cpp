// A stand-in for libyoda_hip.so in CPU tests: the yoda_dev_* entry points the engine resolves,
// recording what it asks for and refusing every schedule call (rc -1), so the engine's CPU path
// places the pods exactly as without a device. tests/test_engine_batch_split.py builds it to
// check how Engine::schedule_batch splits a batch into k_batch dispatches (VERDICT r5 #3a).
#include <cstdint>
#include <cstring>
#include <vector>

#include "yoda_dev_abi.h"

namespace {
std::vector<int> g_batches;   // B of every yoda_dev_schedule_batch call, in order
int g_singles = 0;            // yoda_dev_schedule calls
int g_ctx = 0;
}  // namespace

extern "C" {
__attribute__((visibility("default"))) void* yoda_dev_create(int, int, char*, int) { return &g_ctx; }
__attribute__((visibility("default"))) void yoda_dev_destroy(void*) {}
__attribute__((visibility("default"))) int yoda_dev_capacity(void*) { return 65536; }
__attribute__((visibility("default"))) int yoda_dev_upload(void*, int, const int32_t*, const yoda_dev_node_t*) {
  return 0;
}
__attribute__((visibility("default"))) int yoda_dev_schedule(void*, int, const yoda_dev_req_t*, const uint8_t*,
                                                             yoda_dev_result_t*) {
  ++g_singles;
  return -1;
}
__attribute__((visibility("default"))) int yoda_dev_schedule_batch(void*, int, int B, const yoda_dev_req_t*,
                                                                   yoda_dev_result_t*) {
  g_batches.push_back(B);
  return -1;
}
__attribute__((visibility("default"))) float yoda_dev_last_us(void*) { return 0.f; }
__attribute__((visibility("default"))) void yoda_dev_set_timing(void*, int) {}
__attribute__((visibility("default"))) int yoda_dev_busy(void*) { return 0; }
// test accessors: the recorded batch sizes (returns how many), single-cycle calls; reset
__attribute__((visibility("default"))) int yoda_fake_batches(int* out, int max) {
  const int n = (int)g_batches.size();
  for (int i = 0; i < n && i < max; ++i) out[i] = g_batches[i];
  return n;
}
__attribute__((visibility("default"))) int yoda_fake_singles() { return g_singles; }
__attribute__((visibility("default"))) void yoda_fake_reset() {
  g_batches.clear();
  g_singles = 0;
}
}
