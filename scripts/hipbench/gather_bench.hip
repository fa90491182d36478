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

int main() {
  unsigned long long *d_slots, *d_ticks;
  unsigned int* d_abort;
  CK(hipMalloc(&d_slots, 2 * kMaxG * kStride * 8));
  CK(hipMemset(d_slots, 0, 2 * kMaxG * kStride * 8));
  CK(hipMalloc(&d_ticks, 64));
  CK(hipMalloc(&d_abort, 4));
  unsigned tag = 1;
  const int iters = 2000;
  for (int G : {64, 128, 256}) {
    if (run<2, 0>(G, iters, d_slots, d_abort, d_ticks, tag) || run<2, 1>(G, iters, d_slots, d_abort, d_ticks, tag) ||
        run<2, 2>(G, iters, d_slots, d_abort, d_ticks, tag) || run<4, 0>(G, iters, d_slots, d_abort, d_ticks, tag) ||
        run<4, 1>(G, iters, d_slots, d_abort, d_ticks, tag) || run<11, 0>(G, iters, d_slots, d_abort, d_ticks, tag) ||
        run<11, 1>(G, iters, d_slots, d_abort, d_ticks, tag))
      return 1;
  }
  return 0;
}
