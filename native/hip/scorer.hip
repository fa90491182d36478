// gfx950 device placement scorer: one scheduling cycle of the yoda profile over every node
// of a large MI355X cluster, bit-exact with the CPU engine (native/core/engine.cpp, fixed
// mode) — Filter → PreScore maxima → yoda Score + xGMI gang search → NormalizeScore →
// weighted sum → selectHost.
//
// Mapping to CDNA4: a 64-lane wave owns one node; lanes 0..7 own its GPU slots (card
// eligibility via one 64-bit __ballot), and for the gang search all 64 lanes enumerate
// the 256 GPU subsets of the node (4 per lane) and reduce the best one with __shfl_xor.
// Blocks are 4 waves and grid-stride over nodes; per-block LDS reductions cut the
// cross-workgroup atomics to a few per block (maxima, min/max raw score, argmax key),
// keeping them off the single-address serialisation cliff (cdna guide G12).
// Four launches per pod; cluster-global accumulators are re-armed by the last kernel so no
// memset sits between pods. No MFMA: the work is integer compare/reduce, not matmul-shaped.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "yoda_dev_abi.h"

namespace {

// engine FilterBit / Reason values (native/core/engine.hpp)
constexpr uint32_t F_NODE_UNSCHEDULABLE = 1u << 0;
constexpr uint32_t F_NODE_RESOURCES_FIT = 1u << 4;
constexpr uint32_t F_YODA = 1u << 5;
constexpr int RS_UNSCHEDULABLE = 1, RS_RESOURCES = 5, RS_NO_SCV = 6, RS_STALE = 7, RS_GPU_NUMBER = 8,
              RS_GPU_FIT = 11, RS_DEAD = 12;

constexpr int kWaves = 4;
constexpr int kBlock = 64 * kWaves;

struct Globals {
  unsigned long long maxima[6];   // seeded 1 (collection.go:31-38)
  unsigned long long raw_lo;      // seeded ULLONG_MAX
  unsigned long long raw_hi;      // seeded 0 (scheduler.go:134 `highest := 0`)
  unsigned long long best_key;    // (final << 24) | perm(node)
  int reasons[YODA_DEV_REASONS];
  int feasible;
  int pad[3];
};

__host__ __device__ inline void globals_reset(Globals* g) {
  for (int k = 0; k < 6; ++k) g->maxima[k] = 1;
  g->raw_lo = ULLONG_MAX;
  g->raw_hi = 0;
  g->best_key = 0;
  for (int k = 0; k < YODA_DEV_REASONS; ++k) g->reasons[k] = 0;
  g->feasible = 0;
}

__device__ __forceinline__ uint64_t eff_free(const yoda_dev_card_t& c) {
  uint64_t sampled = c.free > c.pending ? (uint64_t)(c.free - c.pending) : 0;
  uint64_t cap = c.total > c.reserved ? (uint64_t)(c.total - c.reserved) : 0;
  return sampled < cap ? sampled : cap;
}

__device__ __forceinline__ bool card_ok(const yoda_dev_req_t& r, const yoda_dev_node_t* nd, int c) {
  const yoda_dev_card_t& cd = nd->cards[c];
  if (!nd->healthy[c]) return false;
  if (eff_free(cd) < r.memory) return false;
  if (r.has_clock && (uint64_t)cd.clock != r.clock) return false;
  if (r.clock_min && (uint64_t)cd.clock < r.clock_min) return false;
  return true;
}

__device__ __forceinline__ unsigned long long wave_max8(unsigned long long v) {
  // lanes 0..7 hold the values of one node (others 0); reduce within each 8-lane group
  for (int off = 4; off > 0; off >>= 1) {
    unsigned long long o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ unsigned long long wave_sum8(unsigned long long v) {
  for (int off = 4; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ------------------------------------------------------------------ K1: filter + maxima
__global__ __launch_bounds__(kBlock) void k_filter(const yoda_dev_node_t* __restrict__ nodes, int n,
                                                   const yoda_dev_req_t* __restrict__ req_p,
                                                   const uint8_t* __restrict__ cand, uint8_t* __restrict__ feas,
                                                   uint8_t* __restrict__ elig, Globals* __restrict__ g) {
  __shared__ unsigned long long s_max[kWaves][6];
  __shared__ int s_reason[YODA_DEV_REASONS];
  __shared__ int s_feas;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (threadIdx.x < YODA_DEV_REASONS) s_reason[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_feas = 0;
  if (lane < 6) s_max[wave][lane] = 1;
  __syncthreads();
  const yoda_dev_req_t r = *req_p;
  const bool yoda = (r.filters & F_YODA) != 0;
  for (int i = blockIdx.x * kWaves + wave; i < n; i += gridDim.x * kWaves) {
    const yoda_dev_node_t* nd = nodes + i;
    const uint8_t flags = nd->flags;
    int reason = 0;
    if (!(flags & YODA_DEV_ALIVE)) {
      reason = RS_DEAD;
    } else if ((r.filters & F_NODE_UNSCHEDULABLE) && (flags & YODA_DEV_UNSCHEDULABLE) && !r.tolerates_unschedulable) {
      reason = RS_UNSCHEDULABLE;
    } else if (r.filters & F_NODE_RESOURCES_FIT) {
      if (nd->pod_count + 1 > nd->alloc_pods) reason = RS_RESOURCES;
      else if (r.cpu_m > 0 && nd->alloc_cpu < r.cpu_m + nd->req_cpu) reason = RS_RESOURCES;
      else if (r.mem > 0 && nd->alloc_mem < r.mem + nd->req_mem) reason = RS_RESOURCES;
    }
    if (!reason && r.use_candidates && cand[i]) reason = cand[i];
    uint32_t emask = 0;
    if (!reason && yoda) {
      if (!(flags & YODA_DEV_HAS_SCV)) {
        reason = RS_NO_SCV;
      } else if (r.has_number ? !(r.number <= (uint64_t)nd->card_number) : !(nd->card_number > 0)) {
        reason = RS_GPU_NUMBER;
      } else if (flags & YODA_DEV_STALE) {
        reason = RS_STALE;
      } else {
        const bool e = lane < nd->ncards && card_ok(r, nd, lane);
        emask = (uint32_t)(__ballot(e) & 0xFFu);
        if ((uint64_t)__popc(emask) < r.number) reason = RS_GPU_FIT;
      }
    }
    if (lane == 0) {
      feas[i] = reason == 0;
      elig[i] = (uint8_t)emask;
      if (reason) atomicAdd(&s_reason[reason], 1);
      else atomicAdd(&s_feas, 1);
    }
    if (!reason && yoda) {
      unsigned long long v[6] = {0, 0, 0, 0, 0, 0};
      if (lane < 8 && ((emask >> lane) & 1u)) {
        const yoda_dev_card_t& cd = nd->cards[lane];
        v[0] = cd.bandwidth; v[1] = cd.clock; v[2] = cd.core; v[3] = eff_free(cd); v[4] = cd.power; v[5] = cd.total;
      }
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        unsigned long long m = wave_max8(v[k]);
        if (lane == 0 && m > s_max[wave][k]) s_max[wave][k] = m;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    unsigned long long m = 1;
    for (int w = 0; w < kWaves; ++w) m = s_max[w][threadIdx.x] > m ? s_max[w][threadIdx.x] : m;
    if (m > 1) atomicMax(&g->maxima[threadIdx.x], m);
  }
  if (threadIdx.x < YODA_DEV_REASONS && s_reason[threadIdx.x]) atomicAdd(&g->reasons[threadIdx.x], s_reason[threadIdx.x]);
  if (threadIdx.x == 0 && s_feas) atomicAdd(&g->feasible, s_feas);
}

// gang objective of subset `m` (bit i = card i) — engine.cpp Engine::gang_objective
__device__ __forceinline__ int64_t gang_obj(const yoda_dev_req_t& r, const yoda_dev_node_t* nd, uint32_t m,
                                            const uint64_t* ef, int64_t* link_bad_out) {
  const int64_t k = __popc(m);
  const int64_t P = k * (k - 1) / 2;
  int64_t qsum = 0, free_after = 0, total = 0, occ = 0;
  uint64_t numa_mask = 0;
  for (int a = 0; a < YODA_DEV_CARDS; ++a) {
    if (!((m >> a) & 1u)) continue;
    numa_mask |= 1ull << (nd->numa[a] & 63);
    free_after += (int64_t)(ef[a] - r.memory);
    total += (int64_t)nd->cards[a].total;
    occ += nd->occ[a];
    for (int b = a + 1; b < YODA_DEV_CARDS; ++b) {
      if (!((m >> b) & 1u)) continue;
      int32_t q = 10000;
      const int pa = nd->phys[a], pb = nd->phys[b];
      if (pa != pb && pa < nd->nphys && pb < nd->nphys) q = nd->linkq[pa][pb];
      qsum += q;
    }
  }
  const int64_t link_bad = P ? (P * 10000 - qsum) * 100 / P : 0;
  const int64_t d = __popcll(numa_mask);
  const int64_t numa_bad = k > 1 ? (d - 1) * 1000000 / (k - 1) : 0;
  const int64_t leftover = total ? free_after * 1000000 / total : 0;
  const int64_t fit = r.binpack ? leftover : 1000000 - leftover;
  const int64_t occ_bad = k ? occ * 100 / k : 0;
  *link_bad_out = link_bad;
  return r.w_link * link_bad + r.w_numa * numa_bad + r.w_fit * fit + r.w_occ * occ_bad;
}

// (obj, mask) a better than b: smaller objective, then lexicographically smaller subset
__device__ __forceinline__ bool better(int64_t oa, uint32_t ma, int64_t ob, uint32_t mb) {
  if (oa != ob) return oa < ob;
  const uint32_t d = ma ^ mb;
  return d && ((d & (0u - d)) & ma);
}

// ------------------------------------------------------------------ K2: scores + gang search
__global__ __launch_bounds__(kBlock) void k_score(const yoda_dev_node_t* __restrict__ nodes, int n,
                                                  const yoda_dev_req_t* __restrict__ req_p,
                                                  const uint8_t* __restrict__ feas, const uint8_t* __restrict__ elig,
                                                  int64_t* __restrict__ raw, int64_t* __restrict__ total_out,
                                                  uint32_t* __restrict__ mask_out, int32_t* __restrict__ quality_out,
                                                  Globals* __restrict__ g) {
  __shared__ unsigned long long s_lo[kWaves], s_hi[kWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_lo[wave] = ULLONG_MAX;
    s_hi[wave] = 0;
  }
  const yoda_dev_req_t r = *req_p;
  const bool yoda_f = (r.filters & F_YODA) != 0;
  const bool yoda_s = yoda_f && r.w_yoda != 0;
  const unsigned long long* mx = g->maxima;
  const unsigned long long mx0 = mx[0], mx1 = mx[1], mx2 = mx[2], mx3 = mx[3], mx4 = mx[4], mx5 = mx[5];
  const uint64_t k = r.has_number ? r.number : 1;
  for (int i = blockIdx.x * kWaves + wave; i < n; i += gridDim.x * kWaves) {
    if (!feas[i]) continue;     // wave-uniform
    const yoda_dev_node_t* nd = nodes + i;
    const uint32_t emask = elig[i];
    // ---- per-GPU data every lane needs for the subset search
    uint64_t ef[YODA_DEV_CARDS];
#pragma unroll
    for (int c = 0; c < YODA_DEV_CARDS; ++c) ef[c] = eff_free(nd->cards[c]);
    // ---- gang / GPU-set selection (also the Reserve choice for the winning node)
    uint32_t best_m = 0;
    int64_t best_o = LLONG_MAX, best_lb = 0;
    bool found = false;
    if (yoda_f && k >= 1 && k <= YODA_DEV_CARDS) {
      for (int j = 0; j < 4; ++j) {
        const uint32_t m = (uint32_t)(lane + 64 * j);
        if ((uint64_t)__popc(m) != k || (m & ~emask)) continue;
        int64_t lb;
        const int64_t o = gang_obj(r, nd, m, ef, &lb);
        if (!found || better(o, m, best_o, best_m)) {
          best_o = o; best_m = m; best_lb = lb; found = true;
        }
      }
      for (int off = 32; off > 0; off >>= 1) {
        const int64_t oo = __shfl_xor(best_o, off, 64);
        const uint32_t om = __shfl_xor(best_m, off, 64);
        const int64_t ol = __shfl_xor(best_lb, off, 64);
        const int of = __shfl_xor((int)found, off, 64);
        if (of && (!found || better(oo, om, best_o, best_m))) {
          best_o = oo; best_m = om; best_lb = ol; found = true;
        }
      }
    }
    const int32_t quality = found ? (int32_t)(10000 - best_lb / 100) : 10000;
    // ---- yoda raw score (algorithm.go:28-87 with the Q1/Q2/Q3/Q4 fixes)
    unsigned long long basic = 0, tot = 0, fre = 0, alloc = 0;
    if (lane < nd->ncards) {
      const yoda_dev_card_t& cd = nd->cards[lane];
      tot = cd.total;
      fre = ef[lane];
      alloc = cd.reserved;
      if ((emask >> lane) & 1u) {
        const uint64_t bw = (uint64_t)cd.bandwidth * 100 / mx0;
        const uint64_t clk = (uint64_t)cd.clock * 100 / mx1;
        const uint64_t core = (uint64_t)cd.core * 100 / mx2;
        const uint64_t pw = (uint64_t)cd.power * 100 / mx4;
        const uint64_t fm = ef[lane] * 100 / mx3;
        const uint64_t tm = (uint64_t)cd.total * 100 / mx5;
        basic = (bw + clk + core + pw) + fm * 2 + tm;
      }
    }
    basic = wave_sum8(basic);
    tot = wave_sum8(tot);
    fre = wave_sum8(fre);
    alloc = wave_sum8(alloc);
    if (lane == 0) {
      int64_t s_out = 0;
      if (yoda_s) {
        const uint64_t actual = tot ? (fre * 100 / tot) * 2 : 0;
        const uint64_t allocate = (tot == 0 || tot < alloc) ? 0 : (tot - alloc) * 100 / tot * 3;
        uint64_t s = basic + allocate + actual;
        if (r.has_number && r.number > 1 && r.number <= nd->ncards && found)
          s += (uint64_t)(quality / 100) * (uint64_t)r.w_gang_score;
        s_out = s > (uint64_t)LLONG_MAX ? 0 : (int64_t)s;
        const unsigned long long us = (unsigned long long)s_out;
        if (us < s_lo[wave]) s_lo[wave] = us;
        if (us > s_hi[wave]) s_hi[wave] = us;
      }
      // upstream default scores (engine.cpp Engine::score_nodes)
      const int64_t nz_cpu = r.cpu_m > 0 ? r.cpu_m : 100;
      const int64_t nz_mem = r.mem > 0 ? r.mem : 200LL * 1024 * 1024;
      const int64_t rc = nd->req_cpu + nz_cpu, rm = nd->req_mem + nz_mem;
      int64_t least = 0, most = 0, extra = r.w_const;
      if (nd->alloc_cpu > 0 && rc <= nd->alloc_cpu) least += (nd->alloc_cpu - rc) * 100 / nd->alloc_cpu;
      if (nd->alloc_mem > 0 && rm <= nd->alloc_mem) least += (nd->alloc_mem - rm) * 100 / nd->alloc_mem;
      if (nd->alloc_cpu > 0) most += (rc < nd->alloc_cpu ? rc : nd->alloc_cpu) * 100 / nd->alloc_cpu;
      if (nd->alloc_mem > 0) most += (rm < nd->alloc_mem ? rm : nd->alloc_mem) * 100 / nd->alloc_mem;
      extra += r.w_least * (least / 2) + r.w_most * (most / 2);
      if (r.w_balanced) {
        const double cf = nd->alloc_cpu > 0 ? (double)rc / (double)nd->alloc_cpu : 1.0;
        const double mf = nd->alloc_mem > 0 ? (double)rm / (double)nd->alloc_mem : 1.0;
        const int64_t b = (cf >= 1 || mf >= 1) ? 0 : (int64_t)((1.0 - fabs(cf - mf)) * 100);
        extra += r.w_balanced * b;
      }
      raw[i] = s_out;
      total_out[i] = extra;
      mask_out[i] = best_m;
      quality_out[i] = quality;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && yoda_s) {
    unsigned long long lo = ULLONG_MAX, hi = 0;
    for (int w = 0; w < kWaves; ++w) {
      lo = s_lo[w] < lo ? s_lo[w] : lo;
      hi = s_hi[w] > hi ? s_hi[w] : hi;
    }
    if (lo != ULLONG_MAX) atomicMin(&g->raw_lo, lo);
    if (hi) atomicMax(&g->raw_hi, hi);
  }
}

// ------------------------------------------------------------------ K3: normalize + argmax
__global__ __launch_bounds__(kBlock) void k_select(int n, const yoda_dev_req_t* __restrict__ req_p,
                                                   const uint8_t* __restrict__ feas, const int64_t* __restrict__ raw,
                                                   const int64_t* __restrict__ total, Globals* __restrict__ g) {
  __shared__ unsigned long long s_key[kBlock / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const yoda_dev_req_t r = *req_p;
  const bool yoda_s = (r.filters & F_YODA) && r.w_yoda != 0;
  // scheduler.go:132-157: highest seeded 0, lowest = min; equal → lowest − 1
  const int64_t hi = (int64_t)g->raw_hi;
  int64_t lo = (int64_t)g->raw_lo;
  if (hi == lo) --lo;
  const int64_t den = (int64_t)((uint64_t)hi - (uint64_t)lo);
  unsigned long long best = 0;
  for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
    if (!feas[i]) continue;
    int64_t f = total[i];
    if (yoda_s) {
      const int64_t num = (int64_t)(((uint64_t)raw[i] - (uint64_t)lo) * 100ull);
      f += (num / den) * r.w_yoda;
    }
    const uint32_t p = ((uint32_t)i * r.perm_mul + r.perm_add) & 0xFFFFFFu;
    const unsigned long long key = ((unsigned long long)f << 24) | p;
    best = key > best ? key : best;
  }
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(best, off, 64);
    best = o > best ? o : best;
  }
  if (lane == 0) s_key[wave] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (int w = 0; w < kBlock / 64; ++w) b = s_key[w] > b ? s_key[w] : b;
    if (b) atomicMax(&g->best_key, b);
  }
}

// ------------------------------------------------------------------ K4: result + re-arm
__global__ void k_finish(const yoda_dev_req_t* __restrict__ req_p, const uint32_t* __restrict__ mask,
                         const int32_t* __restrict__ quality, Globals* __restrict__ g,
                         yoda_dev_result_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const yoda_dev_req_t r = *req_p;
  out->feasible = g->feasible;
  if (g->feasible == 0) {
    out->node = -1;
    out->score = 0;
    out->mask = 0;
    out->quality = 0;
  } else {
    const unsigned long long key = g->best_key;
    const uint32_t p = (uint32_t)(key & 0xFFFFFFull);
    const int32_t node = (int32_t)(((p - r.perm_add) * r.perm_inv) & 0xFFFFFFu);
    out->node = node;
    out->score = g->feasible == 1 ? 0 : (int64_t)(key >> 24);
    out->mask = mask[node];
    out->quality = quality[node];
  }
  for (int k = 0; k < YODA_DEV_REASONS; ++k) out->reasons[k] = g->reasons[k];
  for (int k = 0; k < 6; ++k) out->maxima[k] = g->maxima[k];
  out->raw_lo = (int64_t)g->raw_lo;
  out->raw_hi = (int64_t)g->raw_hi;
  globals_reset(g);
}

__global__ void k_scatter(const yoda_dev_node_t* __restrict__ stage, const int32_t* __restrict__ idx, int n,
                          yoda_dev_node_t* __restrict__ nodes) {
  // one 512-byte record per 32 lanes (16 B each)
  const int rec = blockIdx.x * (blockDim.x / 32) + (threadIdx.x >> 5);
  if (rec >= n) return;
  const uint4* src = reinterpret_cast<const uint4*>(stage + rec);
  uint4* dst = reinterpret_cast<uint4*>(nodes + idx[rec]);
  dst[threadIdx.x & 31] = src[threadIdx.x & 31];
}

struct Ctx {
  int device = 0, cap = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  yoda_dev_node_t *d_nodes = nullptr, *d_stage = nullptr, *h_stage = nullptr;
  int32_t *d_idx = nullptr, *h_idx = nullptr;
  uint8_t *d_feas = nullptr, *d_elig = nullptr, *d_cand = nullptr, *h_cand = nullptr;
  int64_t *d_raw = nullptr, *d_total = nullptr;
  uint32_t* d_mask = nullptr;
  int32_t* d_quality = nullptr;
  yoda_dev_req_t *d_req = nullptr, *h_req = nullptr;
  yoda_dev_result_t *d_res = nullptr, *h_res = nullptr;
  Globals* d_g = nullptr;
  float last_us = 0;
  int grid = 1024;
};

#define CK(x)                            \
  do {                                   \
    hipError_t e__ = (x);                \
    if (e__ != hipSuccess) return (int)e__; \
  } while (0)

int grid_for(const Ctx* c, int n) {
  int g = (n + kWaves - 1) / kWaves;
  return g < c->grid ? (g > 0 ? g : 1) : c->grid;
}

}  // namespace

extern "C" {

void* yoda_dev_create(int device, int capacity, char* err, int err_len) {
  Ctx* c = new Ctx();
  c->device = device;
  c->cap = capacity;
  auto fail = [&](const char* what, hipError_t e) -> void* {
    if (err) snprintf(err, err_len, "%s: %s", what, hipGetErrorString(e));
    delete c;
    return nullptr;
  };
  hipError_t e;
  if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
  int cus = 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess) c->grid = cus * 4;
  if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
  if ((e = hipEventCreate(&c->e0)) != hipSuccess) return fail("event", e);
  if ((e = hipEventCreate(&c->e1)) != hipSuccess) return fail("event", e);
  const size_t N = (size_t)capacity;
  if ((e = hipMalloc(&c->d_nodes, N * sizeof(yoda_dev_node_t))) != hipSuccess) return fail("nodes", e);
  if ((e = hipMemset(c->d_nodes, 0, N * sizeof(yoda_dev_node_t))) != hipSuccess) return fail("memset", e);
  if ((e = hipMalloc(&c->d_stage, N * sizeof(yoda_dev_node_t))) != hipSuccess) return fail("stage", e);
  if ((e = hipHostMalloc(&c->h_stage, N * sizeof(yoda_dev_node_t), hipHostMallocDefault)) != hipSuccess)
    return fail("pinned stage", e);
  if ((e = hipMalloc(&c->d_idx, N * sizeof(int32_t))) != hipSuccess) return fail("idx", e);
  if ((e = hipHostMalloc(&c->h_idx, N * sizeof(int32_t), hipHostMallocDefault)) != hipSuccess) return fail("idx", e);
  if ((e = hipMalloc(&c->d_feas, N)) != hipSuccess) return fail("feas", e);
  if ((e = hipMalloc(&c->d_elig, N)) != hipSuccess) return fail("elig", e);
  if ((e = hipMalloc(&c->d_cand, N)) != hipSuccess) return fail("cand", e);
  if ((e = hipHostMalloc(&c->h_cand, N, hipHostMallocDefault)) != hipSuccess) return fail("cand", e);
  if ((e = hipMalloc(&c->d_raw, N * sizeof(int64_t))) != hipSuccess) return fail("raw", e);
  if ((e = hipMalloc(&c->d_total, N * sizeof(int64_t))) != hipSuccess) return fail("total", e);
  if ((e = hipMalloc(&c->d_mask, N * sizeof(uint32_t))) != hipSuccess) return fail("mask", e);
  if ((e = hipMalloc(&c->d_quality, N * sizeof(int32_t))) != hipSuccess) return fail("quality", e);
  if ((e = hipMalloc(&c->d_req, sizeof(yoda_dev_req_t))) != hipSuccess) return fail("req", e);
  if ((e = hipHostMalloc(&c->h_req, sizeof(yoda_dev_req_t), hipHostMallocDefault)) != hipSuccess) return fail("req", e);
  if ((e = hipMalloc(&c->d_res, sizeof(yoda_dev_result_t))) != hipSuccess) return fail("res", e);
  if ((e = hipHostMalloc(&c->h_res, sizeof(yoda_dev_result_t), hipHostMallocDefault)) != hipSuccess)
    return fail("res", e);
  if ((e = hipMalloc(&c->d_g, sizeof(Globals))) != hipSuccess) return fail("globals", e);
  Globals init;
  globals_reset(&init);
  if ((e = hipMemcpy(c->d_g, &init, sizeof(Globals), hipMemcpyHostToDevice)) != hipSuccess) return fail("init", e);
  return c;
}

void yoda_dev_destroy(void* p) {
  Ctx* c = (Ctx*)p;
  if (!c) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  hipFree(c->d_nodes); hipFree(c->d_stage); hipHostFree(c->h_stage); hipFree(c->d_idx); hipHostFree(c->h_idx);
  hipFree(c->d_feas); hipFree(c->d_elig); hipFree(c->d_cand); hipHostFree(c->h_cand); hipFree(c->d_raw);
  hipFree(c->d_total); hipFree(c->d_mask); hipFree(c->d_quality); hipFree(c->d_req); hipHostFree(c->h_req);
  hipFree(c->d_res); hipHostFree(c->h_res); hipFree(c->d_g);
  hipEventDestroy(c->e0); hipEventDestroy(c->e1);
  hipStreamDestroy(c->stream);
  delete c;
}

int yoda_dev_capacity(void* p) { return p ? ((Ctx*)p)->cap : 0; }

int yoda_dev_upload(void* p, int n, const int32_t* idx, const yoda_dev_node_t* rows) {
  Ctx* c = (Ctx*)p;
  if (n <= 0) return 0;
  if (n > c->cap) return -1;
  for (int i = 0; i < n; ++i)
    if (idx[i] < 0 || idx[i] >= c->cap) return -2;   // never scatter outside the node table
  CK(hipSetDevice(c->device));
  memcpy(c->h_stage, rows, (size_t)n * sizeof(yoda_dev_node_t));
  memcpy(c->h_idx, idx, (size_t)n * sizeof(int32_t));
  CK(hipMemcpyAsync(c->d_stage, c->h_stage, (size_t)n * sizeof(yoda_dev_node_t), hipMemcpyHostToDevice, c->stream));
  CK(hipMemcpyAsync(c->d_idx, c->h_idx, (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  const int per_block = 8;   // 8 records × 32 lanes = 256 threads
  hipLaunchKernelGGL(k_scatter, dim3((n + per_block - 1) / per_block), dim3(256), 0, c->stream, c->d_stage, c->d_idx, n,
                     c->d_nodes);
  CK(hipGetLastError());
  // the staging buffers are reused by the next upload: wait for the copies
  CK(hipStreamSynchronize(c->stream));
  return 0;
}

int yoda_dev_schedule(void* p, int n, const yoda_dev_req_t* req, const uint8_t* cand, yoda_dev_result_t* out) {
  Ctx* c = (Ctx*)p;
  if (n <= 0 || n > c->cap) return -1;
  if (req->use_candidates && !cand) return -3;
  CK(hipSetDevice(c->device));
  *c->h_req = *req;
  CK(hipMemcpyAsync(c->d_req, c->h_req, sizeof(yoda_dev_req_t), hipMemcpyHostToDevice, c->stream));
  if (req->use_candidates) {
    memcpy(c->h_cand, cand, (size_t)n);
    CK(hipMemcpyAsync(c->d_cand, c->h_cand, (size_t)n, hipMemcpyHostToDevice, c->stream));
  }
  const int grid = grid_for(c, n);
  const int grid_sel = (n + kBlock - 1) / kBlock < c->grid ? (n + kBlock - 1) / kBlock : c->grid;
  CK(hipEventRecord(c->e0, c->stream));
  hipLaunchKernelGGL(k_filter, dim3(grid), dim3(kBlock), 0, c->stream, c->d_nodes, n, c->d_req, c->d_cand, c->d_feas,
                     c->d_elig, c->d_g);
  hipLaunchKernelGGL(k_score, dim3(grid), dim3(kBlock), 0, c->stream, c->d_nodes, n, c->d_req, c->d_feas, c->d_elig,
                     c->d_raw, c->d_total, c->d_mask, c->d_quality, c->d_g);
  hipLaunchKernelGGL(k_select, dim3(grid_sel > 0 ? grid_sel : 1), dim3(kBlock), 0, c->stream, n, c->d_req, c->d_feas,
                     c->d_raw, c->d_total, c->d_g);
  hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, c->stream, c->d_req, c->d_mask, c->d_quality, c->d_g, c->d_res);
  CK(hipGetLastError());
  CK(hipEventRecord(c->e1, c->stream));
  CK(hipMemcpyAsync(c->h_res, c->d_res, sizeof(yoda_dev_result_t), hipMemcpyDeviceToHost, c->stream));
  CK(hipStreamSynchronize(c->stream));
  float ms = 0;
  if (hipEventElapsedTime(&ms, c->e0, c->e1) == hipSuccess) c->last_us = ms * 1000.0f;
  *out = *c->h_res;
  return 0;
}

int yoda_dev_debug(void* p, int n, uint8_t* feas, int64_t* raw, int64_t* total, uint32_t* mask, int32_t* quality) {
  Ctx* c = (Ctx*)p;
  if (n <= 0 || n > c->cap) return -1;
  CK(hipSetDevice(c->device));
  if (feas) CK(hipMemcpy(feas, c->d_feas, (size_t)n, hipMemcpyDeviceToHost));
  if (raw) CK(hipMemcpy(raw, c->d_raw, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (total) CK(hipMemcpy(total, c->d_total, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (mask) CK(hipMemcpy(mask, c->d_mask, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (quality) CK(hipMemcpy(quality, c->d_quality, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}

float yoda_dev_last_us(void* p) { return p ? ((Ctx*)p)->last_us : 0.f; }

}  // extern "C"
