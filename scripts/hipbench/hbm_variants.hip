// Standalone sweep of HBM read-kernel shapes on gfx950 (used to pick the probe's shape).
// hipcc --offload-arch=gfx950 -O3 hbm_variants.hip -o hbm_variants && ./hbm_variants
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void k_read_gs(const float4* __restrict__ src, size_t n4, float* __restrict__ sink) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (; i + (UNROLL - 1) * stride < n4; i += UNROLL * stride) {
    float4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (NT) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(&src[i + u * stride]));
        v[u] = make_float4(t.x, t.y, t.z, t.w);
      } else {
        v[u] = src[i + u * stride];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
  }
  for (; i < n4; i += stride) { float4 a = src[i]; acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w; }
  float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 1234.5f) sink[blockIdx.x] = s;
}

// each block sweeps one contiguous slab; lanes read consecutive 16-B words
template <int UNROLL>
__global__ __launch_bounds__(256) void k_read_slab(const float4* __restrict__ src, size_t n4, float* __restrict__ sink) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t beg = (size_t)blockIdx.x * per, end = beg + per < n4 ? beg + per : n4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  size_t i = beg + threadIdx.x;
  for (; i + (UNROLL - 1) * 256 < end; i += UNROLL * 256) {
    float4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = src[i + u * 256];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) { acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w; }
  }
  for (; i < end; i += 256) { float4 a = src[i]; acc.x += a.x; acc.y += a.y; acc.z += a.z; acc.w += a.w; }
  float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 1234.5f) sink[blockIdx.x] = s;
}

template <int UNROLL>
__global__ __launch_bounds__(256) void k_copy_gs(const float4* __restrict__ src, float4* __restrict__ dst, size_t n4) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n4; i += UNROLL * stride) {
    float4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) dst[i + u * stride] = v[u];
  }
  for (; i < n4; i += stride) dst[i] = src[i];
}

template <int UNROLL>
__global__ __launch_bounds__(256) void k_copy_nt(const float4* __restrict__ src, float4* __restrict__ dst, size_t n4) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4* s = reinterpret_cast<const f4*>(src);
  f4* d = reinterpret_cast<f4*>(dst);
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (UNROLL - 1) * stride < n4; i += UNROLL * stride) {
    f4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = __builtin_nontemporal_load(&s[i + u * stride]);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) __builtin_nontemporal_store(v[u], &d[i + u * stride]);
  }
  for (; i < n4; i += stride) d[i] = s[i];
}

template <int UNROLL>
__global__ __launch_bounds__(256) void k_copy_slab(const float4* __restrict__ src, float4* __restrict__ dst, size_t n4) {
  const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
  const size_t beg = (size_t)blockIdx.x * per, end = beg + per < n4 ? beg + per : n4;
  size_t i = beg + threadIdx.x;
  for (; i + (UNROLL - 1) * 256 < end; i += UNROLL * 256) {
    float4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = src[i + u * 256];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) dst[i + u * 256] = v[u];
  }
  for (; i < end; i += 256) dst[i] = src[i];
}

template <typename F>
double time_it(F launch, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  launch(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < iters; ++i) launch();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a); hipEventDestroy(b);
  return ms / iters;
}

int main() {
  int cus = 256; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t maxb = 4ull << 30;
  float4 *a, *b; float* sink;
  CK(hipMalloc(&a, maxb)); CK(hipMalloc(&b, maxb)); CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(a, 0, maxb)); CK(hipMemset(b, 0, maxb));
  for (size_t bytes : {1ull << 30, 4ull << 30}) {
    const size_t n4 = bytes / 16;
    for (int mult : {8, 16, 32, 64}) {
      const int grid = cus * mult;
      auto gbps = [&](double ms, double factor) { return bytes * factor / (ms * 1e-3) / 1e9; };
      double r8n = time_it([&] { hipLaunchKernelGGL((k_read_gs<8, true>), dim3(grid), dim3(256), 0, 0, a, n4, sink); }, 10);
      double r4n = time_it([&] { hipLaunchKernelGGL((k_read_gs<4, true>), dim3(grid), dim3(256), 0, 0, a, n4, sink); }, 10);
      double c4n = time_it([&] { hipLaunchKernelGGL((k_copy_nt<4>), dim3(grid), dim3(256), 0, 0, a, b, n4); }, 10);
      double c8n = time_it([&] { hipLaunchKernelGGL((k_copy_nt<8>), dim3(grid), dim3(256), 0, 0, a, b, n4); }, 10);
      double cs4 = time_it([&] { hipLaunchKernelGGL((k_copy_slab<4>), dim3(grid), dim3(256), 0, 0, a, b, n4); }, 10);
      printf("{\"bytes\": %zu, \"blocks_per_cu\": %d, \"read_gs8_nt\": %.0f, \"read_gs4_nt\": %.0f, "
             "\"copy_nt4\": %.0f, \"copy_nt8\": %.0f, \"copy_slab4\": %.0f}\n",
             bytes, mult, gbps(r8n, 1), gbps(r4n, 1), gbps(c4n, 2), gbps(c8n, 2), gbps(cs4, 2));
      fflush(stdout);
    }
  }
  return 0;
}
