// Floor of k_batch's cross-workgroup all-gather on gfx950, without any compute around it:
// G resident blocks exchange K-granule {tag, value} records N times back to back, exactly as
// native/hip/scorer.hip does (relaxed agent-scope atomic stores, thread t < G polls record t
// with relaxed agent-scope atomic loads, records double-buffered by tag parity). Variants:
//   mode 0  poll one granule per record until every record's has landed, then load the rest
//           (scorer.hip's gather)
//   mode 1  load all K granules of the record on every poll
//   mode 2  mode 1 without the s_sleep between polls
// Every spin is bounded (s_memrealtime deadline + abort word), so a non-resident grid ends.
//   hipcc --offload-arch=gfx950 -O3 gather_bench.hip -o gather_bench && ./gather_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                      \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
constexpr int kStride = 16;     // granules per record slot
constexpr int kMaxG = 256;

template <int K, int MODE>
__global__ __launch_bounds__(256) void k_gather(unsigned long long* slots, unsigned int* abort_word, int iters,
                                                unsigned tag0, long long deadline, unsigned long long* ticks) {
  __shared__ int s_fail;
  const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
  if (t == 0) s_fail = 0;
  __syncthreads();
  const long long t_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long sink = 0;
  for (int e = 0; e < iters; ++e) {
    const unsigned tag = tag0 + (unsigned)e;
    gu64* mine = (gu64*)(slots + ((size_t)(tag & 1u) * kMaxG + g) * kStride);
    if (t < K) __hip_atomic_store(mine + t, ((unsigned long long)tag << 32) | (unsigned)(g + t), __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
    bool failed = false;
    if (__builtin_amdgcn_readfirstlane(t & ~63) < G) {
      const gu64* p = (const gu64*)(slots + ((size_t)(tag & 1u) * kMaxG + (t < G ? t : 0)) * kStride);
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      for (unsigned spins = 0;; ++spins) {
        bool ok = true;
        unsigned long long acc = 0;
        if (MODE == 0) {
          const unsigned long long x0 = t < G ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                              : ((unsigned long long)tag << 32);
          ok = (unsigned)(x0 >> 32) == tag;
          if (__all(ok)) {
#pragma unroll
            for (int k = 1; k < K; ++k) {
              const unsigned long long x = t < G ? __hip_atomic_load(p + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                 : ((unsigned long long)tag << 32);
              ok &= (unsigned)(x >> 32) == tag;
              acc += (unsigned)x;
            }
            if (__all(ok)) {
              sink += acc + (unsigned)x0;
              break;
            }
          }
        } else {
#pragma unroll
          for (int k = 0; k < K; ++k) {
            const unsigned long long x = t < G ? __hip_atomic_load(p + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                               : ((unsigned long long)tag << 32);
            ok &= (unsigned)(x >> 32) == tag;
            acc += (unsigned)x;
          }
          if (__all(ok)) {
            sink += acc;
            break;
          }
        }
        if (MODE != 2) __builtin_amdgcn_s_sleep(1);
        if ((spins & 63) == 63) {
          if (__hip_atomic_load((gu32*)abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            failed = true;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > deadline) {
            __hip_atomic_store((gu32*)abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            failed = true;
            break;
          }
        }
      }
    }
    if (failed && (t & 63) == 0) s_fail = 1;
    __syncthreads();
    if (s_fail) break;
  }
  if (g == 0 && t == 0) {
    ticks[0] = (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t_start);
    ticks[1] = (unsigned long long)s_fail;
  }
  if (sink == 0x1234567ull) ticks[2] = sink;   // keeps the loads alive
}

// XCD-local exchange (round 5): the same all-gather, but each group is the
// set of blocks that actually run on one XCD. A block reads its XCC id (hwreg XCC_ID) and takes
// a rank in that XCD's group with an agent-scope atomic add; once every block registered (bounded
// spin) the group size is that XCD's final count. Groups are therefore formed from the real
// placement, never assumed from blockIdx % 8 (that guess is only checked: `mismatch`). The 8
// groups exchange independently; each record is polled only by blocks sharing its L2.
//   STORE 0  agent-scope relaxed atomic stores (write-through: the line leaves the L2)
//   STORE 1  plain stores + vmcnt(0) (the line stays in the XCD's L2), agent-scope (L1-bypassing)
//            loads on the consumer side — same-L2 reads only, which is what makes this valid
constexpr int kMaxPer = 128;   // blocks per XCD group
__device__ __forceinline__ unsigned xcc_id() {
  // s_getreg_b32 hwreg(HW_REG_XCC_ID, 0, 4): id 20, offset 0, size 4 → simm16 = (3 << 11) | 20
  return (unsigned)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xFu;
}

template <int K, int STORE>
__global__ __launch_bounds__(256) void k_gather_xcd(unsigned long long* slots, unsigned int* reg,
                                                    unsigned int* abort_word, int iters, unsigned tag0,
                                                    long long deadline, unsigned long long* ticks) {
  __shared__ int s_fail, s_rank, s_size, s_xcc;
  const int G = gridDim.x, g = blockIdx.x, t = threadIdx.x;
  // reg[0..7]: per-XCD counts, reg[8]: total registered, reg[9]: blockIdx % 8 != XCC mismatches
  if (t == 0) {
    s_fail = 0;
    const unsigned x = xcc_id();
    s_xcc = (int)x;
    s_rank = (int)__hip_atomic_fetch_add(reg + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(g & 7) != x) __hip_atomic_fetch_add(reg + 9, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(reg + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(reg + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)G) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > deadline) {
        s_fail = 1;
        __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    s_size = (int)__hip_atomic_load(reg + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s_size > kMaxPer || s_rank >= kMaxPer) s_fail = 1;
  }
  __syncthreads();
  const int rank = s_rank, size = s_size, xcc = s_xcc;
  const long long t_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long sink = 0;
  for (int e = 0; e < iters && !s_fail; ++e) {
    const unsigned tag = tag0 + (unsigned)e;
    const size_t base = ((size_t)(tag & 1u) * 8 + xcc) * kMaxPer;
    unsigned long long* mine = slots + (base + rank) * kStride;
    if (t < K) {
      const unsigned long long v = ((unsigned long long)tag << 32) | (unsigned)(g + t);
      if (STORE == 0) {
        __hip_atomic_store((gu64*)(mine + t), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        *(gu64*)(mine + t) = v;   // plain global store (no volatile: that would be sc0 sc1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    bool failed = false;
    if (__builtin_amdgcn_readfirstlane(t & ~63) < size) {
      const gu64* p = (const gu64*)(slots + (base + (t < size ? t : 0)) * kStride);
      const long long t0 = __builtin_amdgcn_s_memrealtime();
      for (unsigned spins = 0;; ++spins) {
        const unsigned long long x0 = t < size ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                               : ((unsigned long long)tag << 32);
        bool ok = (unsigned)(x0 >> 32) == tag;
        if (__all(ok)) {
          unsigned long long acc = 0;
#pragma unroll
          for (int k = 1; k < K; ++k) {
            const unsigned long long x = t < size ? __hip_atomic_load(p + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                  : ((unsigned long long)tag << 32);
            ok &= (unsigned)(x >> 32) == tag;
            acc += (unsigned)x;
          }
          if (__all(ok)) {
            sink += acc + (unsigned)x0;
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
        if ((spins & 63) == 63) {
          if (__hip_atomic_load((gu32*)abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            failed = true;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > deadline) {
            __hip_atomic_store((gu32*)abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            failed = true;
            break;
          }
        }
      }
    }
    if (failed && (t & 63) == 0) s_fail = 1;
    __syncthreads();
  }
  if (t == 0 && rank == 0) {
    // one timing per XCD group: slot xcc
    ticks[4 + xcc] = (unsigned long long)(__builtin_amdgcn_s_memrealtime() - t_start);
  }
  if (g == 0 && t == 0) ticks[1] = (unsigned long long)s_fail;
  if (sink == 0x1234567ull) ticks[2] = sink;
}

template <int K, int STORE>
int run_xcd(int G, int iters, unsigned long long* d_slots, unsigned int* d_reg, unsigned int* d_abort,
            unsigned long long* d_ticks, unsigned& tag) {
  CK(hipMemset(d_abort, 0, 4));
  CK(hipMemset(d_reg, 0, 64));
  CK(hipMemset(d_ticks, 0, 16 * 8));
  hipLaunchKernelGGL((k_gather_xcd<K, STORE>), dim3(G), dim3(256), 0, 0, d_slots, d_reg, d_abort, iters, tag,
                     200000000ll / 100, d_ticks);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  tag += (unsigned)iters + 2;
  unsigned long long h[16];
  unsigned int r[16];
  CK(hipMemcpy(h, d_ticks, sizeof(h), hipMemcpyDeviceToHost));
  CK(hipMemcpy(r, d_reg, sizeof(r), hipMemcpyDeviceToHost));
  double mx = 0, mn = 1e30;
  for (int x = 0; x < 8; ++x) {
    const double us = (double)h[4 + x] / 100.0 / iters;
    if (r[x]) {
      mx = us > mx ? us : mx;
      mn = us < mn ? us : mn;
    }
  }
  printf("{\"G\": %d, \"K\": %d, \"mode\": \"xcd_%s\", \"per_xcd\": [%u,%u,%u,%u,%u,%u,%u,%u], "
         "\"mismatch_blockidx_mod8\": %u, \"us_per_exchange_min\": %.3f, \"us_per_exchange_max\": %.3f, "
         "\"aborted\": %llu}\n",
         G, K, STORE ? "plain_store" : "atomic_store", r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7], r[9], mn, mx,
         h[1]);
  return 0;
}

template <int K, int MODE>
int run(int G, int iters, unsigned long long* d_slots, unsigned int* d_abort, unsigned long long* d_ticks,
        unsigned& tag) {
  CK(hipMemset(d_abort, 0, 4));
  hipLaunchKernelGGL((k_gather<K, MODE>), dim3(G), dim3(256), 0, 0, d_slots, d_abort, iters, tag, 200000000ll / 100,
                     d_ticks);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  tag += (unsigned)iters + 2;
  unsigned long long h[3];
  CK(hipMemcpy(h, d_ticks, sizeof(h), hipMemcpyDeviceToHost));
  printf("{\"G\": %d, \"K\": %d, \"mode\": %d, \"us_per_exchange\": %.3f, \"aborted\": %llu}\n", G, K, MODE,
         (double)h[0] / 100.0 / iters, h[1]);
  return 0;
}

int main(int argc, char** argv) {
  unsigned long long *d_slots, *d_ticks;
  unsigned int *d_abort, *d_reg;
  const size_t slot_bytes = (size_t)2 * 8 * kMaxPer * kStride * 8;   // ≥ the global mode's 2 × kMaxG slots
  CK(hipMalloc(&d_slots, slot_bytes));
  CK(hipMemset(d_slots, 0, slot_bytes));
  CK(hipMalloc(&d_ticks, 16 * 8));
  CK(hipMalloc(&d_abort, 4));
  CK(hipMalloc(&d_reg, 64));
  unsigned tag = 1;
  const int iters = 2000;
  if (argc > 1 && argv[1][0] == 'x') {
    // XCD-local groups vs the same group size spread over the chip (global mode 0)
    for (int G : {32, 64, 128}) {
      if (run<2, 0>(G, iters, d_slots, d_abort, d_ticks, tag) || run<4, 0>(G, iters, d_slots, d_abort, d_ticks, tag) ||
          run<11, 0>(G, iters, d_slots, d_abort, d_ticks, tag))
        return 1;
    }
    for (int G : {64, 128, 256, 512}) {
      CK(hipMemset(d_slots, 0, slot_bytes));
      tag = 1;
      if (run_xcd<2, 0>(G, iters, d_slots, d_reg, d_abort, d_ticks, tag) ||
          run_xcd<2, 1>(G, iters, d_slots, d_reg, d_abort, d_ticks, tag) ||
          run_xcd<4, 0>(G, iters, d_slots, d_reg, d_abort, d_ticks, tag) ||
          run_xcd<4, 1>(G, iters, d_slots, d_reg, d_abort, d_ticks, tag) ||
          run_xcd<11, 0>(G, iters, d_slots, d_reg, d_abort, d_ticks, tag) ||
          run_xcd<11, 1>(G, iters, d_slots, d_reg, d_abort, d_ticks, tag))
        return 1;
    }
    return 0;
  }
  for (int G : {64, 128, 256}) {
    if (run<2, 0>(G, iters, d_slots, d_abort, d_ticks, tag) || run<2, 1>(G, iters, d_slots, d_abort, d_ticks, tag) ||
        run<2, 2>(G, iters, d_slots, d_abort, d_ticks, tag) || run<4, 0>(G, iters, d_slots, d_abort, d_ticks, tag) ||
        run<4, 1>(G, iters, d_slots, d_abort, d_ticks, tag) || run<11, 0>(G, iters, d_slots, d_abort, d_ticks, tag) ||
        run<11, 1>(G, iters, d_slots, d_abort, d_ticks, tag))
      return 1;
  }
  return 0;
}
