// Per-thread block caches under this module's operator new / delete.
//
// The scheduler's native threads hand objects to each other: the I/O thread decodes pod events
// that the lane thread drops, the lane builds Bindings that the I/O thread sends and frees. The
// native-thread profiles (profiles/bench/r6/natprof/) had 40-60 % of the lane and I/O threads in
// glibc malloc / free, much of it waiting on an arena lock or refilling a 7-entry tcache bin.
// Raising glibc's tcache (GLIBC_TUNABLES=glibc.malloc.tcache_count=2048) measured +5.6 % pods/s
// and p99 1.01 -> 0.67 ms on config 3 (profiles/bench/r6/tcache_ab/), but tunables are read at
// process start, and the scheduler runs inside processes it does not start (bench.py under the
// driver, an operator's container). This is the same mechanism inside the module: a freed block
// goes to the freeing thread's list for its size class (up to kCap blocks), and an allocation of
// that class takes one from the list before calling malloc.
//
// Every block is a plain malloc block and its class is read from malloc_usable_size, so blocks
// may cross modules and threads freely: one allocated by libstdc++'s own operator new and freed
// here is cached; one allocated here and freed elsewhere goes to free(). The modules link with
// -Bsymbolic-functions, so their own calls bind to these definitions whatever else the process
// has loaded. Sanitizer builds (YODA_NO_FASTALLOC) and the allocation-counting probe keep the
// default operators.
#ifndef YODA_NO_FASTALLOC
#include <malloc.h>

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <new>

namespace {

constexpr size_t kGranule = 16;
constexpr size_t kClasses = 64;   // usable sizes up to 64 * 16 - 8 = 1016 bytes
constexpr uint32_t kCap = 2048;   // blocks kept per class and thread

// glibc chunks have usable sizes 16k - 8 (k >= 2): class k holds blocks of that usable size
inline size_t class_of_request(size_t n) { return (n + 8 + kGranule - 1) / kGranule; }
inline size_t usable_of_class(size_t k) { return k * kGranule - 8; }

struct Cache {
  void* head[kClasses] = {};
  uint32_t n[kClasses] = {};
  bool dead = false;
  ~Cache() {
    dead = true;
    for (size_t k = 0; k < kClasses; ++k)
      while (void* p = head[k]) {
        head[k] = *static_cast<void**>(p);
        std::free(p);
      }
  }
};

thread_local Cache tc;

inline void* take(size_t n) {
  const size_t k = class_of_request(n);
  if (k < kClasses && !tc.dead) {
    if (void* p = tc.head[k]) {
      tc.head[k] = *static_cast<void**>(p);
      --tc.n[k];
      return p;
    }
    return std::malloc(usable_of_class(k));   // exactly this class's usable size
  }
  return std::malloc(n ? n : 1);
}

inline void give(void* p) {
  if (!p) return;
  const size_t us = malloc_usable_size(p);
  const size_t k = (us + 8) / kGranule;
  if (k < kClasses && usable_of_class(k) == us && !tc.dead && tc.n[k] < kCap) {
    *static_cast<void**>(p) = tc.head[k];
    tc.head[k] = p;
    ++tc.n[k];
    return;
  }
  std::free(p);
}

inline void* take_or_throw(size_t n) {
  void* p = take(n);
  if (!p) throw std::bad_alloc();
  return p;
}

}  // namespace

void* operator new(size_t n) { return take_or_throw(n); }
void* operator new[](size_t n) { return take_or_throw(n); }
void* operator new(size_t n, const std::nothrow_t&) noexcept { return take(n); }
void* operator new[](size_t n, const std::nothrow_t&) noexcept { return take(n); }
void operator delete(void* p) noexcept { give(p); }
void operator delete[](void* p) noexcept { give(p); }
void operator delete(void* p, size_t) noexcept { give(p); }
void operator delete[](void* p, size_t) noexcept { give(p); }
void operator delete(void* p, const std::nothrow_t&) noexcept { give(p); }
void operator delete[](void* p, const std::nothrow_t&) noexcept { give(p); }
#endif  // YODA_NO_FASTALLOC
