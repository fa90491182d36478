// gfx950 device placement scorer: one scheduling cycle of the yoda profile over every node
// of a large MI355X cluster, bit-exact with the CPU engine (native/core/engine.cpp, fixed
// mode) — Filter → PreScore maxima → yoda Score + xGMI gang search → NormalizeScore →
// weighted sum → selectHost.
//
// CDNA4 mapping
//  * a 64-lane wave scores 8 nodes at once: lane group g (8 lanes) owns node base+g and
//    lane s of the group owns GPU slot s, so eligibility is one 64-bit __ballot split in
//    8-bit fields and every per-node reduction is 3 DPP lane moves inside the group;
//  * the k-GPU gang search walks a constant table of the C(8,k) subsets with k set bits
//    (≤ 70), 8 lanes per node, skipping subsets with ineligible GPUs; the objective uses
//    per-lane register tables (effective free HBM, total, occupancy, NUMA, the 28
//    card-pair xGMI qualities resolved by the host) — integer math mirrors the CPU;
//  * 64-bit divisions (the scoring is full of them) go through an exact double-estimate
//    + integer-correction path instead of the ~100-instruction software divide;
//  * blocks of 4 waves grid-stride over nodes; per-block LDS reductions, XCD-sharded
//    counters and check-before-atomic max/min keep cross-workgroup atomics to a handful;
//  * the dirty node rows of the last reservation ride in the filter kernel's arguments
//    (it reads them from there and block 0 writes them back to the table), and up to
//    kFuseSelectMax nodes the score kernel's last block (agent-scope ticket, release/
//    acquire per the CDNA visibility rules) runs the normalise+argmax itself: 2 launches
//    and no memcpy per pod in the steady state (3 above kFuseSelectMax);
//  * the winner is written straight into mapped pinned host memory, the `feasible` field
//    last with a system-scope release, and the host spins on it instead of a stream sync.
// No MFMA: the work is integer compare/reduce, not matmul-shaped.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "yoda_dev_abi.h"

namespace {

// engine FilterBit / Reason values (native/core/engine.hpp)
constexpr uint32_t F_NODE_UNSCHEDULABLE = 1u << 0;
constexpr uint32_t F_NODE_RESOURCES_FIT = 1u << 4;
constexpr uint32_t F_YODA = 1u << 5;
constexpr int RS_UNSCHEDULABLE = 1, RS_RESOURCES = 5, RS_NO_SCV = 6, RS_STALE = 7, RS_GPU_NUMBER = 8,
              RS_GPU_FIT = 11, RS_DEAD = 12, RS_EXT_RESOURCES = 13;

constexpr int kWaves = 4;
constexpr int kBlock = 64 * kWaves;
constexpr int kGroup = 8;                 // lanes per node
constexpr int kNodesPerWave = 64 / kGroup;
constexpr int kPatchRows = 4;             // dirty rows passed by value (4 × 512 B + the filter's args < 4 KiB)
constexpr int kFuseSelectMax = 2048;      // one block normalises + argmaxes up to this many nodes
constexpr int kSelBatch = 8;              // nodes per thread whose loads select_block issues together
constexpr int kBatchCap = 256;            // pods per batched launch sequence
constexpr int kShards = 8;

struct Globals {
  unsigned long long maxima[6];   // seeded 1 (collection.go:31-38)
  unsigned long long raw_lo;      // seeded ULLONG_MAX
  unsigned long long raw_hi;      // seeded 0 (scheduler.go:134 `highest := 0`)
  unsigned long long best_key;    // (final << 24) | perm(node)
  // counters sharded 8 ways (blockIdx % 8 ≈ one XCD under round-robin dispatch; speed
  // only) so 2k blocks do not serialise on one address; the select kernel sums shards
  int reasons[kShards][YODA_DEV_REASONS];
  int feasible[kShards];
  unsigned int ticket;
  int pad[3];
};

struct PatchArgs {
  int n;
  int32_t idx[kPatchRows];
  yoda_dev_node_t rows[kPatchRows];
};

// subsets of {0..7} grouped by popcount, ascending (lexicographic order is irrelevant:
// ties are broken explicitly by `better`)
struct SubsetTable {
  uint8_t masks[256];
  uint16_t start[10];
};

__constant__ SubsetTable c_subsets;

SubsetTable make_subsets() {
  SubsetTable t{};
  int p = 0;
  for (int k = 0; k <= 8; ++k) {
    t.start[k] = (uint16_t)p;
    for (int m = 0; m < 256; ++m)
      if (__builtin_popcount(m) == k) t.masks[p++] = (uint8_t)m;
  }
  t.start[9] = (uint16_t)p;
  return t;
}

__host__ __device__ inline void globals_reset(Globals* g) {
  for (int k = 0; k < 6; ++k) g->maxima[k] = 1;
  g->raw_lo = ULLONG_MAX;
  g->raw_hi = 0;
  g->best_key = 0;
  for (int s = 0; s < kShards; ++s) {
    for (int k = 0; k < YODA_DEV_REASONS; ++k) g->reasons[s][k] = 0;
    g->feasible[s] = 0;
  }
  g->ticket = 0;
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// relaxed agent-scope read of an accumulator (memory-side value, any XCD)
__device__ __forceinline__ unsigned long long peek(unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// atomics only when this block can still change the accumulator
// (`direct`: skip the check — one dependent memory round trip less per block, at the cost
// of every block's atomic reaching the accumulator. Measured on MI355X: direct wins by
// ≈1.5 µs up to ~256 blocks and loses by ≈2 µs from ~500 blocks on, so the host picks it
// per launch from the grid size; YODA_DEV_DIRECT_ATOMICS=0/1 forces either.)
__device__ __forceinline__ void max_if(unsigned long long* p, unsigned long long v, bool direct = false) {
  if (direct || v > peek(p)) atomicMax(p, v);
}
__device__ __forceinline__ void min_if(unsigned long long* p, unsigned long long v, bool direct = false) {
  if (direct || v < peek(p)) atomicMin(p, v);
}

// 1/d to full double precision: the hardware reciprocal refined by two Newton steps.
__device__ __forceinline__ double rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}
// Exact floor(n / d) for d > 0 given r ≈ 1/d (a few ulp): for n < 2^50 the estimate
// n·r is within 1 of the quotient and one integer multiply-subtract fixes it. Larger n (not
// produced by realistic clusters) take the software divide. Per-pod or per-node divisors
// pass a precomputed reciprocal; `udiv` computes it.
__device__ __forceinline__ uint64_t udiv_r(uint64_t n, uint64_t d, double r) {
  if (n < (1ull << 50)) {
    uint64_t q = (uint64_t)((double)n * r);
    const uint64_t qd = q * d;
    if (qd > n) --q;
    else if (n - qd >= d) ++q;
    return q;
  }
  return n / d;
}
__device__ __forceinline__ uint64_t udiv(uint64_t n, uint64_t d) {
  return d < (1ull << 50) ? udiv_r(n, d, rcp64((double)d)) : n / d;
}
// truncating int division by a small positive divisor (|n| < 2^30) from r ≈ 1/d: the
// estimate on |n| is within 1 of the quotient, one integer check fixes it
__device__ __forceinline__ int32_t sdiv_small_r(int32_t n, int32_t d, double r) {
  const int32_t a = n < 0 ? -n : n;
  int32_t q = (int32_t)((double)a * r);
  if ((q + 1) * d <= a) ++q;
  else if (q * d > a) --q;
  return n < 0 ? -q : q;
}

__device__ __forceinline__ uint64_t eff_free(uint32_t free, uint32_t pending, uint32_t total, uint32_t reserved) {
  const uint64_t sampled = free > pending ? (uint64_t)(free - pending) : 0;
  const uint64_t cap = total > reserved ? (uint64_t)(total - reserved) : 0;
  return sampled < cap ? sampled : cap;
}

// ---- cross-lane reductions on DPP lane moves (VALU, no LDS round trip like ds_bpermute).
// A node's 8 lanes are lanes 8g..8g+7: quad_perm xor 1, xor 2, then row_half_mirror (lane i ↔
// 7 − i of the same 8) reach every lane of the group; row_mirror (i ↔ 15 − i) pairs the two
// groups of a 16-lane row; readlane 0/16/32/48 combines the four rows. Every source lane of a
// move must be active: group reductions run where a whole group takes the same branch, wave
// reductions in wave-uniform control flow.
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppRowMirror = 0x140, kDppRowHalfMirror = 0x141;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL, typename T>
__device__ __forceinline__ T dpp(T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit lanes");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, dpp32<CTRL>(__builtin_bit_cast(uint32_t, v)));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint64_t r = (uint64_t)dpp32<CTRL>((uint32_t)u) | ((uint64_t)dpp32<CTRL>((uint32_t)(u >> 32)) << 32);
    return __builtin_bit_cast(T, r);
  }
}
template <typename T>
__device__ __forceinline__ T readlane(T v, int l) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint64_t r = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l) << 32);
    return __builtin_bit_cast(T, r);
  }
}
struct OpMax { template <typename T> __device__ T operator()(T a, T b) const { return a > b ? a : b; } };
struct OpMin { template <typename T> __device__ T operator()(T a, T b) const { return a < b ? a : b; } };
struct OpSum { template <typename T> __device__ T operator()(T a, T b) const { return a + b; } };
struct OpOr { template <typename T> __device__ T operator()(T a, T b) const { return a | b; } };

template <typename T, typename Op>
__device__ __forceinline__ T group_reduce(T v, Op op) {   // every lane of the 8 gets the result
  v = op(v, dpp<kDppXor1>(v));
  v = op(v, dpp<kDppXor2>(v));
  return op(v, dpp<kDppRowHalfMirror>(v));
}
template <typename T, typename Op>
__device__ __forceinline__ T across_groups(T v, Op op) {  // v group-uniform → wave-uniform
  v = op(v, dpp<kDppRowMirror>(v));
  return op(op(readlane(v, 0), readlane(v, 16)), op(readlane(v, 32), readlane(v, 48)));
}
template <typename T>
__device__ __forceinline__ T gmax(T v) { return group_reduce(v, OpMax{}); }
template <typename T>
__device__ __forceinline__ T gsum(T v) { return group_reduce(v, OpSum{}); }
template <typename T>
__device__ __forceinline__ T wmax_across_groups(T v) { return across_groups(v, OpMax{}); }
template <typename T>
__device__ __forceinline__ T wave_max(T v) { return across_groups(group_reduce(v, OpMax{}), OpMax{}); }
template <typename T>
__device__ __forceinline__ T wave_min(T v) { return across_groups(group_reduce(v, OpMin{}), OpMin{}); }
template <typename T>
__device__ __forceinline__ T wave_sum(T v) { return across_groups(group_reduce(v, OpSum{}), OpSum{}); }
template <typename T>
__device__ __forceinline__ T wave_or(T v) { return across_groups(group_reduce(v, OpOr{}), OpOr{}); }

// ------------------------------------------------------------------ dirty-row patch
__global__ void k_patch(PatchArgs a, yoda_dev_node_t* __restrict__ nodes) {
  const int rec = threadIdx.x >> 5, part = threadIdx.x & 31;
  if (rec >= a.n) return;
  const uint4* src = reinterpret_cast<const uint4*>(&a.rows[rec]);
  reinterpret_cast<uint4*>(nodes + a.idx[rec])[part] = src[part];
}

__global__ void k_scatter(const yoda_dev_node_t* __restrict__ stage, const int32_t* __restrict__ idx, int n,
                          yoda_dev_node_t* __restrict__ nodes) {
  const int rec = blockIdx.x * (blockDim.x / 32) + (threadIdx.x >> 5);
  if (rec >= n) return;
  const uint4* src = reinterpret_cast<const uint4*>(stage + rec);
  reinterpret_cast<uint4*>(nodes + idx[rec])[threadIdx.x & 31] = src[threadIdx.x & 31];
}

// stream-ordered after a k_scatter: the staging buffers it read may be reused
__global__ void k_upload_done(int32_t* flag, int32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------ K1: filter + maxima
// One lane group = one node (lane `sub` = GPU slot). Returns the node's filter reason (0 =
// feasible) and its eligible-GPU mask, and folds the card metrics of feasible nodes into the
// wave maxima `wmx` (wave-uniform afterwards). Shared by k_filter and k_batch. `MAXIMA`
// false: the verdict and mask only (wmx untouched; the PAIRS fix-up's scoring waves).
template <bool MAXIMA = true>
__device__ __forceinline__ int filter_eval(const yoda_dev_node_t* nd, bool valid, const yoda_dev_req_t& r,
                                           uint8_t cnd, uint32_t* wmx, uint32_t& emask_out, int grp, int sub) {
  const bool yoda = (r.filters & F_YODA) != 0;
  // every load of the node issued up front: one memory round trip per node
  const uint8_t flags = valid ? nd->flags : 0, ncards = nd->ncards;
  const uint32_t card_number = nd->card_number;
  const int64_t pod_count = nd->pod_count, alloc_pods = nd->alloc_pods, alloc_cpu = nd->alloc_cpu,
                req_cpu = nd->req_cpu, alloc_mem = nd->alloc_mem, req_mem = nd->req_mem;
  const int64_t ext_alloc = nd->ext_alloc, ext_used = nd->ext_used;
  const yoda_dev_card_t cd = nd->cards[sub];
  const uint8_t healthy = nd->healthy[sub];
  int reason = 0;
  if (!(flags & YODA_DEV_ALIVE)) {
    reason = RS_DEAD;
  } else if ((r.filters & F_NODE_UNSCHEDULABLE) && (flags & YODA_DEV_UNSCHEDULABLE) && !r.tolerates_unschedulable) {
    reason = RS_UNSCHEDULABLE;
  } else if (r.filters & F_NODE_RESOURCES_FIT) {
    if (pod_count + 1 > alloc_pods) reason = RS_RESOURCES;
    else if (r.cpu_m > 0 && alloc_cpu < r.cpu_m + req_cpu) reason = RS_RESOURCES;
    else if (r.mem > 0 && alloc_mem < r.mem + req_mem) reason = RS_RESOURCES;
    // the one extended resource the device rows carry (engine.cpp: the device's ext dimension)
    else if (r.ext > 0 && ext_used + r.ext > ext_alloc) reason = RS_EXT_RESOURCES;
  }
  if (!reason && cnd) reason = cnd;
  bool yoda_stage = false;
  if (!reason && yoda) {
    if (!(flags & YODA_DEV_HAS_SCV)) reason = RS_NO_SCV;
    else if (r.has_number ? !(r.number <= (uint64_t)card_number) : !(card_number > 0)) reason = RS_GPU_NUMBER;
    else if (flags & YODA_DEV_STALE) reason = RS_STALE;
    else yoda_stage = true;
  }
  const uint64_t ef = eff_free(cd.free, cd.pending, cd.total, cd.reserved);
  const bool e = yoda_stage && sub < ncards && healthy && ef >= r.memory &&
                 (!r.has_clock || (uint64_t)cd.clock == r.clock) && (!r.clock_min || (uint64_t)cd.clock >= r.clock_min);
  const uint32_t emask = (uint32_t)((__ballot(e) >> (grp * kGroup)) & 0xFFu);
  if (yoda_stage && (uint64_t)__popc(emask) < r.number) reason = RS_GPU_FIT;
  const bool ok = valid && reason == 0;
  emask_out = emask;
  if (MAXIMA && yoda) {
    const bool take = ok && ((emask >> sub) & 1u);
    // card metrics are u32 (ef ≤ free): 32-bit shuffles
    uint32_t v[6];
    v[0] = take ? cd.bandwidth : 0; v[1] = take ? cd.clock : 0; v[2] = take ? cd.core : 0;
    v[3] = take ? (uint32_t)ef : 0; v[4] = take ? cd.power : 0; v[5] = take ? cd.total : 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const uint32_t m = wmax_across_groups(gmax(v[k]));
      wmx[k] = m > wmx[k] ? m : wmx[k];
    }
  }
  return valid ? reason : 0;
}

__device__ __forceinline__ void filter_group(const yoda_dev_node_t* nd, int i, bool valid, const yoda_dev_req_t& r,
                                             const uint8_t* __restrict__ cand, uint8_t* __restrict__ feas,
                                             uint8_t* __restrict__ elig, int* s_reason, uint32_t* wmx,
                                             int& nfeas, int grp, int sub) {
  const uint8_t cnd = (r.use_candidates && valid) ? cand[i] : 0;
  uint32_t emask = 0;
  const int reason = filter_eval(nd, valid, r, cnd, wmx, emask, grp, sub);
  const bool ok = valid && reason == 0;
  if (valid && sub == 0) {
    feas[i] = ok;
    elig[i] = (uint8_t)emask;
    if (reason) atomicAdd(&s_reason[reason], 1);
  }
  if (sub == 0 && ok) ++nfeas;
}

__global__ __launch_bounds__(kBlock) void k_filter(const PatchArgs pa, yoda_dev_node_t* __restrict__ nodes, int n,
                                                   const yoda_dev_req_t r, const uint8_t* __restrict__ cand,
                                                   uint8_t* __restrict__ feas, uint8_t* __restrict__ elig,
                                                   Globals* __restrict__ g) {
  __shared__ unsigned long long s_max[kWaves][6];
  __shared__ int s_reason[YODA_DEV_REASONS];
  __shared__ int s_feas;
  const int lane = threadIdx.x & 63, wave = uniform(threadIdx.x >> 6);
  const int grp = lane >> 3, sub = lane & 7;
  if (threadIdx.x < YODA_DEV_REASONS) s_reason[threadIdx.x] = 0;
  if (threadIdx.x == 0) s_feas = 0;
  __syncthreads();
  uint32_t wmx[6] = {1, 1, 1, 1, 1, 1};
  int nfeas = 0;
  // with dirty rows the host launches one extra block: it writes them back to the table
  // for the score kernel and evaluates them from the arguments, in parallel with the rest
  const int workers = pa.n > 0 ? (int)gridDim.x - 1 : (int)gridDim.x;
  if ((int)blockIdx.x == workers) {
    if ((int)(threadIdx.x >> 5) < pa.n) {
      const int rec = threadIdx.x >> 5;
      reinterpret_cast<uint4*>(nodes + pa.idx[rec])[threadIdx.x & 31] =
          reinterpret_cast<const uint4*>(&pa.rows[rec])[threadIdx.x & 31];
    }
    if (wave == 0) {
      const int j = grp < pa.n ? grp : 0;
      filter_group(&pa.rows[j], pa.idx[j], grp < pa.n && pa.idx[j] < n, r, cand, feas, elig, s_reason, wmx, nfeas,
                   grp, sub);
    }
  } else {
    const int stride = workers * kWaves * kNodesPerWave;
    for (int base = uniform((blockIdx.x * kWaves + wave) * kNodesPerWave); base < n; base += stride) {
      const int i = base + grp;
      bool valid = i < n;
      // patched nodes are evaluated by the patch block, not from the (stale) table
#pragma unroll
      for (int j = 0; j < kPatchRows; ++j) valid = valid && !(j < pa.n && pa.idx[j] == i);
      filter_group(nodes + (i < n ? i : n - 1), i, valid, r, cand, feas, elig, s_reason, wmx, nfeas, grp, sub);
    }
  }
  nfeas = wave_sum(nfeas);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) s_max[wave][k] = wmx[k];
    if (nfeas) atomicAdd(&s_feas, nfeas);
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    unsigned long long m = 1;
    for (int w = 0; w < kWaves; ++w) m = s_max[w][threadIdx.x] > m ? s_max[w][threadIdx.x] : m;
    if (m > 1) max_if(&g->maxima[threadIdx.x], m, r.dev_flags & 1u);
  }
  const int sh = blockIdx.x % kShards;
  if (threadIdx.x < YODA_DEV_REASONS && s_reason[threadIdx.x]) atomicAdd(&g->reasons[sh][threadIdx.x], s_reason[threadIdx.x]);
  if (threadIdx.x == 0 && s_feas) atomicAdd(&g->feasible[sh], s_feas);
}

// ------------------------------------------------------------------ normalise + argmax helpers
// Block-wide best key over nodes blk*kBlock+tid, stride nblk*kBlock (returned by thread 0).
// scheduler.go:132-157: highest seeded 0, lowest = min; equal → lowest − 1.
__device__ unsigned long long select_block(int n, const yoda_dev_req_t& r, const uint8_t* __restrict__ feas,
                                           const int64_t* __restrict__ raw, const int64_t* __restrict__ total,
                                           Globals* __restrict__ g, int blk, int nblk) {
  __shared__ unsigned long long s_key[kWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool yoda_s = (r.filters & F_YODA) && r.w_yoda != 0;
  const int64_t hi = (int64_t)g->raw_hi;
  int64_t lo = (int64_t)g->raw_lo;
  if (hi == lo) --lo;
  const uint64_t den = (uint64_t)hi - (uint64_t)lo;
  unsigned long long best = 0;
  // kSelBatch strided nodes per thread per pass: every load of a pass is issued before the
  // first use, so the single-block (fused) walk pays ~n/(kBlock*kSelBatch) memory round
  // trips instead of one per node stride. (k_select's grid covers n with one node per
  // thread, so there slots 1..kSelBatch-1 are always out of range: the batching only pays
  // in the fused walk.)
  const int stride = nblk * kBlock;
  for (int i0 = blk * kBlock + threadIdx.x; i0 < n; i0 += stride * kSelBatch) {
    uint8_t fe[kSelBatch];
    int64_t tv[kSelBatch], rv[kSelBatch];
#pragma unroll
    for (int k = 0; k < kSelBatch; ++k) {
      const int i = i0 + k * stride;
      const bool in = i < n;
      fe[k] = in ? feas[i] : (uint8_t)0;
      tv[k] = in ? total[i] : 0;
      rv[k] = in ? raw[i] : 0;
    }
#pragma unroll
    for (int k = 0; k < kSelBatch; ++k) {
      if (!fe[k]) continue;
      const int i = i0 + k * stride;
      int64_t f = tv[k];
      if (yoda_s) f += (int64_t)udiv(((uint64_t)rv[k] - (uint64_t)lo) * 100ull, den) * r.w_yoda;
      const uint32_t p = ((uint32_t)i * r.perm_mul + r.perm_add) & 0xFFFFFFu;
      const unsigned long long key = ((unsigned long long)f << 24) | p;
      best = key > best ? key : best;
    }
  }
  best = wave_max(best);
  if (lane == 0) s_key[wave] = best;
  __syncthreads();
  unsigned long long b = 0;
  for (int w = 0; w < kWaves; ++w) b = s_key[w] > b ? s_key[w] : b;
  return b;
}

// Decode the winning key into the mapped result (single thread, after an acquire fence or
// a kernel boundary, so plain loads see every block's accumulators). The record goes out
// with `feasible` = -1 first, then `feasible` alone with a system-scope release, so the
// spinning host never sees a half-written result. Then re-arm the accumulators for the
// next pod (the kernel boundary publishes them on the device).
__device__ void publish(int n, const yoda_dev_req_t& r, unsigned long long key, const uint32_t* __restrict__ mask,
                        const int32_t* __restrict__ quality, Globals* __restrict__ g,
                        yoda_dev_result_t* __restrict__ out, yoda_dev_node_t* __restrict__ nodes) {
  int nf = 0;
  for (int s = 0; s < kShards; ++s) nf += g->feasible[s];
  yoda_dev_result_t res;
  res.feasible = -1;
  if (nf == 0) {
    res.node = -1;
    res.score = 0;
    res.mask = 0;
    res.quality = 0;
  } else {
    const uint32_t p = (uint32_t)(key & 0xFFFFFFull);
    const int32_t node = (int32_t)(((p - r.perm_add) * r.perm_inv) & 0xFFFFFFu);
    res.node = node;
    res.score = nf == 1 ? 0 : (int64_t)(key >> 24);
    res.mask = mask[node];
    res.quality = quality[node];
  }
  for (int k = 0; k < YODA_DEV_REASONS; ++k) {
    int s = 0;
    for (int h = 0; h < kShards; ++h) s += g->reasons[h][k];
    res.reasons[k] = s;
  }
  for (int k = 0; k < 6; ++k) res.maxima[k] = g->maxima[k];
  res.raw_lo = (int64_t)g->raw_lo;
  res.raw_hi = (int64_t)g->raw_hi;
  // batched cycles (dev_flags bit 1): assume the pod on the device too — the next pod's
  // filter launch reads the updated row (engine.cpp Engine::reserve, non-compat, with the
  // host having checked that every reservation counts as pending)
  if ((r.dev_flags & 2u) && nf > 0) {
    yoda_dev_node_t* nd = nodes + res.node;
    const uint32_t mb = (uint32_t)r.memory;
    for (int c = 0; c < YODA_DEV_CARDS; ++c)
      if ((res.mask >> c) & 1u) {
        nd->cards[c].reserved += mb;
        nd->cards[c].pending += mb;
      }
    nd->pod_count += 1;
    nd->req_cpu += r.cpu_m;
    nd->req_mem += r.mem;
    nd->ext_used += r.ext;
    nd->nz_cpu += r.nz_cpu_m;
    nd->nz_mem += r.nz_mem;
  }
  *out = res;
  __hip_atomic_store(&out->feasible, nf, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  globals_reset(g);
}

// (obj, mask) a better than b: smaller objective, then lexicographically smaller subset
__device__ __forceinline__ bool better(int64_t oa, uint32_t ma, int64_t ob, uint32_t mb) {
  if (oa != ob) return oa < ob;
  const uint32_t d = ma ^ mb;
  return d && ((d & (0u - d)) & ma);
}

// ------------------------------------------------------------------ K2: scores + gang search
// Per-pod constants of the score phase (maxima from the filter phase, gang-search bounds,
// reciprocals of the per-pod divisors).
struct ScoreConsts {
  uint64_t mx[6];
  double rmx[6];            // 1 / mx[k]
  int k, s_begin, s_end;
  int32_t P;
  double rP, rk, rk1;       // 1/P, 1/k, 1/(k-1) (0 where unused)
  bool search, yoda_s;
};

__device__ __forceinline__ void score_consts_maxima(ScoreConsts& s, const uint64_t* maxima) {
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    s.mx[j] = maxima[j];
    s.rmx[j] = rcp64((double)maxima[j]);
  }
}

__device__ __forceinline__ ScoreConsts score_consts(const yoda_dev_req_t& r, const uint64_t* maxima) {
  ScoreConsts s;
  if (maxima) score_consts_maxima(s, maxima);
  const bool yoda_f = (r.filters & F_YODA) != 0;
  s.yoda_s = yoda_f && r.w_yoda != 0;
  s.k = (int)(r.has_number ? (r.number > 64 ? 64 : r.number) : 1);
  s.search = yoda_f && s.k >= 1 && s.k <= YODA_DEV_CARDS;
  s.P = s.k * (s.k - 1) / 2;
  s.s_begin = s.search ? c_subsets.start[s.k] : 0;
  s.s_end = s.search ? c_subsets.start[s.k + 1] : 0;
  s.rP = s.P ? rcp64((double)s.P) : 0.0;
  s.rk = rcp64((double)(s.k > 0 ? s.k : 1));
  s.rk1 = s.k > 1 ? rcp64((double)(s.k - 1)) : 0.0;
  return s;
}

// Part A of scoring one node (lane `sub` = card `sub`), everything that does not depend on
// the filter phase's maxima: the gang / GPU-set choice (the Reserve choice if this node
// wins), the yoda score's allocate + actual + gang terms (`rbase_o`) and the upstream default
// scores (`total_o`). Outputs valid on the group's `sub == 0` lane when `act`. Every shuffle
// is executed by every lane (callers iterate wave-uniformly).
struct GangBest {
  int64_t o;
  int32_t lb;
  uint8_t m, found;
};

// `rep` / `nrep`: this group searches subsets s_begin + 8·rep + sub, step 8·nrep (the batch
// kernel splits a node's subset table over nrep lane groups; replicas ≥ 1 only search and
// hand their best back through `gang_o`, valid on sub == 0); replica 0 also scores.
__device__ __forceinline__ void score_node_a(const yoda_dev_node_t* nd, bool act, uint32_t emask,
                                             const yoda_dev_req_t& r, const ScoreConsts& sc,
                                             const uint8_t* s_masks, int sub, uint64_t& rbase_o, int64_t& total_o,
                                             uint32_t& mask_o, int32_t& quality_o, int rep = 0, int nrep = 1,
                                             GangBest* gang_o = nullptr, unsigned long long* stamp = nullptr,
                                             int part = 0) {
  const int k = sc.k;
  const bool search = sc.search, yoda_s = sc.yoda_s;
  const int32_t P = sc.P;
  const int s_begin = sc.s_begin, s_end = sc.s_end;
  const uint8_t ncards = nd->ncards;
  // ---- per-node register tables (every lane of the group holds the whole node). A 1-GPU
  // search needs only the lane's own card: it skips the tables and forms the tail's card
  // sums with a group reduction instead (`fast1`, wave-uniform)
  // `part` (the PAIRS fix-up splits the two halves over waves): 0 both, 1 the GPU-set choice
  // only (into gang_o), 2 the scores only (no set: the caller adds the chosen set's gang bonus)
  const bool fast1 = search && k == 1 && rep == 0 && part != 2;
  uint64_t ef[YODA_DEV_CARDS];
  uint32_t tot[YODA_DEV_CARDS], occ[YODA_DEV_CARDS];
  // the allocate/actual terms' card sums, formed from the same registers (every lane holds
  // the node): no cross-lane reduction
  uint64_t t64 = 0, a64 = 0, fsum = 0;
#pragma unroll
  for (int a = 0; a < YODA_DEV_CARDS && !fast1; ++a) {
    const uint4 lo4 = reinterpret_cast<const uint4*>(&nd->cards[a])[0];   // total, free, reserved, pending
    ef[a] = eff_free(lo4.y, lo4.w, lo4.x, lo4.z);
    tot[a] = lo4.x;
    occ[a] = nd->occ[a];
    if (a < ncards) {
      t64 += lo4.x;
      a64 += lo4.z;
      fsum += ef[a];
    }
  }
  if (stamp) stamp[0] = __builtin_amdgcn_s_memrealtime();   // (trace) tables loaded
  // ---- gang / GPU-set selection (the Reserve choice if this node wins); the 8 lanes'
  // candidates meet through DPP moves inside the group (the whole group is in the branch)
#define GANG_STEP1(CTRL)                                              \
  do {                                                                \
    const int64_t oo = dpp<CTRL>(best_o);                             \
    const uint32_t om = dpp<CTRL>(best_m);                            \
    const uint32_t of = dpp<CTRL>((uint32_t)found);                   \
    if (of && (!found || better(oo, om, best_o, best_m))) {           \
      best_o = oo; best_m = om; found = true;                         \
    }                                                                 \
  } while (0)
#define GANG_STEP(CTRL)                                               \
  do {                                                                \
    const int64_t oo = dpp<CTRL>(best_o);                             \
    const uint32_t om = dpp<CTRL>(best_m);                            \
    const int32_t ol = dpp<CTRL>(best_lb);                            \
    const uint32_t of = dpp<CTRL>((uint32_t)found);                   \
    if (of && (!found || better(oo, om, best_o, best_m))) {           \
      best_o = oo; best_m = om; best_lb = ol; found = true;           \
    }                                                                 \
  } while (0)
  uint32_t best_m = 0;
  int64_t best_o = LLONG_MAX;
  int32_t best_lb = 0;
  bool found = false;
  if (part == 2) {
    // scores only: the tables above hold the node's card sums
  } else if (fast1 && act) {
    // single-GPU pods (the bulk of a mixed burst): the k = 1 table is {1<<0 … 1<<7} in
    // order, so lane `sub` owns subset {sub}; no pairs (P = 0) and one NUMA domain leave
    // only the fit and occupancy terms — the generic loop's 28 predicated pair adds and
    // 8-card sums are skipped. Same integer arithmetic, so the result is bit-identical.
    // Each lane reads only its own card; the tail's card sums meet in one group reduction.
    const uint4 lo4 = reinterpret_cast<const uint4*>(&nd->cards[sub])[0];   // total, free, reserved, pending
    const uint64_t efs = eff_free(lo4.y, lo4.w, lo4.x, lo4.z);
    const bool in = sub < ncards;
    t64 = gsum(in ? (uint64_t)lo4.x : 0ull);
    a64 = gsum(in ? (uint64_t)lo4.z : 0ull);
    fsum = gsum(in ? efs : 0ull);
    if ((emask >> sub) & 1u) {
      const uint32_t tos = lo4.x, ocs = nd->occ[sub];
      const uint64_t fa = efs - r.memory;
      const int32_t leftover = tos ? (int32_t)udiv(fa * 1000000ull, (uint64_t)tos) : 0;   // ≤ 10^6
      const int32_t fit = r.binpack ? leftover : 1000000 - leftover;
      const int32_t occ_bad = (int32_t)(ocs * 100u);   // sdiv by k = 1
      best_o = (int64_t)(int32_t)r.w_fit * fit + (int64_t)(int32_t)r.w_occ * occ_bad;
      best_m = 1u << sub;
      best_lb = 0;
      found = true;
    }
    GANG_STEP1(kDppXor1);
    GANG_STEP1(kDppXor2);
    GANG_STEP1(kDppRowHalfMirror);
  } else if (search && act && k > 1) {
    // numa + card-pair qualities: only the multi-GPU search reads them
    uint32_t numa[YODA_DEV_CARDS];
#pragma unroll
    for (int a = 0; a < YODA_DEV_CARDS; ++a) numa[a] = nd->numa[a] & 63u;
    uint32_t lq[32];   // 64 u16 card-pair qualities, packed 2 per dword
    {
      const uint4* q4 = reinterpret_cast<const uint4*>(&nd->linkq[0][0]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint4 v = q4[t];
        lq[4 * t] = v.x; lq[4 * t + 1] = v.y; lq[4 * t + 2] = v.z; lq[4 * t + 3] = v.w;
      }
    }
    // every card pair equally good (idle or evenly loaded xGMI, the usual SPX node): a
    // subset of k cards sums to P·q, no per-pair adds
    const uint32_t q01 = lq[0] >> 16;   // linkq[0][1]
    bool uni = true;
#pragma unroll
    for (int a = 0; a < YODA_DEV_CARDS; ++a)
#pragma unroll
      for (int b = a + 1; b < YODA_DEV_CARDS; ++b) {
        const int idx = a * YODA_DEV_CARDS + b;
        uni = uni && ((lq[idx >> 1] >> ((idx & 1) * 16)) & 0xFFFFu) == q01;
      }
    // one subset per lane per step (evaluating two subsets per step as independent chains
    // measured slower on MI355X: 4-GPU pods 12.5 vs 11.7 µs of score_a at 4096 nodes, the
    // register footprint grows; profiles/device/r4/gang_ilp2_rejected_r4/)
    for (int t = s_begin + kGroup * rep + sub; t < s_end; t += kGroup * nrep) {
      const uint32_t m = s_masks[t];
      if (m & ~emask) continue;
      int32_t qsum = 0;
      int32_t qmin = 10000;
      uint64_t nmask = 0;
      uint64_t fa = 0, tt = 0;
      uint32_t oc = 0;
#pragma unroll
      for (int a = 0; a < YODA_DEV_CARDS; ++a) {
        const bool ia = (m >> a) & 1u;
        nmask |= ia ? (1ull << numa[a]) : 0ull;   // numa < 64
        fa += ia ? ef[a] - r.memory : 0;
        tt += ia ? tot[a] : 0;
        oc += ia ? occ[a] : 0u;
      }
      if (uni) {
        qsum = P * (int32_t)q01;
        qmin = (int32_t)q01 < qmin ? (int32_t)q01 : qmin;
      } else {
#pragma unroll
        for (int a = 0; a < YODA_DEV_CARDS; ++a) {
          const bool ia = (m >> a) & 1u;
#pragma unroll
          for (int b = a + 1; b < YODA_DEV_CARDS; ++b) {
            const int idx = a * YODA_DEV_CARDS + b;
            const int32_t q = (int32_t)((lq[idx >> 1] >> ((idx & 1) * 16)) & 0xFFFFu);
            const bool both = ia && ((m >> b) & 1u);
            qsum += both ? q : 0;
            qmin = (both && q < qmin) ? q : qmin;
          }
        }
      }
      const int32_t lb = P ? sdiv_small_r((P * 10000 - qsum) * 100, P, sc.rP) : 0;
      const int32_t d = __popcll(nmask);
      const int32_t numa_bad = k > 1 ? sdiv_small_r((d - 1) * 1000000, k - 1, sc.rk1) : 0;
      const int32_t leftover = tt ? (int32_t)udiv(fa * 1000000ull, tt) : 0;   // fa ≤ tt: ≤ 10^6
      const int32_t fit = r.binpack ? leftover : 1000000 - leftover;
      const int32_t occ_bad = sdiv_small_r((int32_t)(oc * 100u), k, sc.rk);
      // every term fits 32 bits and the host bounds |w| ≤ 10^6 (Engine::device_eligible):
      // 32×32→64-bit multiply-adds instead of 64×64
      const int32_t mb = P ? (10000 - qmin) * 100 : 0;   // bottleneck pair (≤ 10^6)
      const int64_t o = (int64_t)(int32_t)r.w_link * lb + (int64_t)(int32_t)r.w_minlink * mb +
                        (int64_t)(int32_t)r.w_numa * numa_bad + (int64_t)(int32_t)r.w_fit * fit +
                        (int64_t)(int32_t)r.w_occ * occ_bad;
      if (!found || better(o, m, best_o, best_m)) {
        best_o = o; best_m = m; best_lb = lb; found = true;
      }
    }
    GANG_STEP(kDppXor1);
    GANG_STEP(kDppXor2);
    GANG_STEP(kDppRowHalfMirror);
  }
#undef GANG_STEP1
#undef GANG_STEP
  if (stamp) stamp[1] = __builtin_amdgcn_s_memrealtime();   // (trace) GPU set chosen
  if (gang_o && act && sub == 0) *gang_o = GangBest{best_o, best_lb, (uint8_t)best_m, (uint8_t)found};
  if (part == 1) return;
  const int32_t quality = found ? 10000 - sdiv_small_r(best_lb, 100, 0.01) : 10000;
  // ---- yoda score terms that need no maxima (algorithm.go:28-87 with the Q1/Q2/Q3/Q4
  // fixes): allocate + actual over the node's cards (sums above), plus the gang bonus, and
  // the upstream default scores (engine.cpp Engine::score_nodes). The divisions are
  // independent, so the group's 8 lanes take one each instead of lane 0 chaining them:
  //   lane 0 actual·2, 1 allocate·3, 2/3 least cpu/mem, 4/5 most cpu/mem, 6 balanced;
  // every term is ≤ 500 (percentages of a node's own capacity), so one 32-bit DPP group sum
  // carries them packed: bits 0-8 yoda (≤ 500), 9-16 least (≤ 200), 17-24 most (≤ 200),
  // 25-31 balanced (≤ 100).
  if (act && rep == 0) {
    const int64_t rc = nd->nz_cpu + r.nz_cpu_m, rm = nd->nz_mem + r.nz_mem;
    const int64_t ac = nd->alloc_cpu, am = nd->alloc_mem;
    const bool lm = r.w_least || r.w_most;
    uint64_t num = 0, den = 0;
    uint32_t mul = 1, shift = 0;
    switch (sub) {
      case 0: if (yoda_s && t64) { num = fsum * 100; den = t64; mul = 2; } break;
      case 1: if (yoda_s && t64 && t64 >= a64) { num = (t64 - a64) * 100; den = t64; mul = 3; } break;
      case 2: if (lm && ac > 0 && rc <= ac) { num = (uint64_t)(ac - rc) * 100; den = (uint64_t)ac; } shift = 9; break;
      case 3: if (lm && am > 0 && rm <= am) { num = (uint64_t)(am - rm) * 100; den = (uint64_t)am; } shift = 9; break;
      case 4: if (lm && ac > 0) { num = (uint64_t)(rc < ac ? rc : ac) * 100; den = (uint64_t)ac; } shift = 17; break;
      case 5: if (lm && am > 0) { num = (uint64_t)(rm < am ? rm : am) * 100; den = (uint64_t)am; } shift = 17; break;
      default: break;
    }
    uint32_t part = den ? (uint32_t)udiv_r(num, den, rcp64((double)den)) * mul << shift : 0u;
    if (sub == 6 && r.w_balanced) {
      const double cf = ac > 0 ? (double)rc / (double)ac : 1.0;
      const double mf = am > 0 ? (double)rm / (double)am : 1.0;
      const uint32_t b = (cf >= 1 || mf >= 1) ? 0u : (uint32_t)(int64_t)((1.0 - fabs(cf - mf)) * 100);
      part = b << 25;
    }
    const uint32_t packed = gsum(part);
    if (sub == 0) {
      uint64_t rb = packed & 0x1FFu;
      if (yoda_s && r.has_number && r.number > 1 && r.number <= ncards && found)
        rb += (uint64_t)(quality / 100) * (uint64_t)r.w_gang_score;
      int64_t extra = r.w_const;
      if (lm) extra += r.w_least * (int64_t)(((packed >> 9) & 0xFFu) / 2) + r.w_most * (int64_t)(((packed >> 17) & 0xFFu) / 2);
      if (r.w_balanced) extra += r.w_balanced * (int64_t)(packed >> 25);
      rbase_o = rb;
      total_o = extra;
      mask_o = best_m;
      quality_o = quality;
    }
  }
}

// Part B: the yoda raw score = Σ over eligible cards of the maxima-normalised card metrics
// (basic) + part A's `rbase`; folds it into `lo`/`hi`. Valid on `sub == 0` when `act`.
__device__ __forceinline__ int64_t score_node_b(const yoda_dev_node_t* nd, bool act, uint32_t emask,
                                                const ScoreConsts& sc, int sub, uint64_t rbase,
                                                unsigned long long& lo, unsigned long long& hi) {
  uint64_t basic = 0;
  if (act && sc.yoda_s && ((emask >> sub) & 1u)) {
    const yoda_dev_card_t cd = nd->cards[sub];
    const uint64_t ef = eff_free(cd.free, cd.pending, cd.total, cd.reserved);
    basic = udiv_r((uint64_t)cd.bandwidth * 100, sc.mx[0], sc.rmx[0]) +
            udiv_r((uint64_t)cd.clock * 100, sc.mx[1], sc.rmx[1]) +
            udiv_r((uint64_t)cd.core * 100, sc.mx[2], sc.rmx[2]) +
            udiv_r((uint64_t)cd.power * 100, sc.mx[4], sc.rmx[4]) +
            udiv_r(ef * 100, sc.mx[3], sc.rmx[3]) * 2 + udiv_r((uint64_t)cd.total * 100, sc.mx[5], sc.rmx[5]);
  }
  basic = gsum((uint32_t)basic);   // ≤ 8 cards × 700: 32-bit lanes
  int64_t s_out = 0;
  if (act && sub == 0 && sc.yoda_s) {
    const uint64_t s = basic + rbase;
    s_out = s > (uint64_t)LLONG_MAX ? 0 : (int64_t)s;
    const unsigned long long us = (unsigned long long)s_out;
    lo = us < lo ? us : lo;
    hi = us > hi ? us : hi;
  }
  return s_out;
}

// score_node_b for k_batch: returns the raw score before the int64 clamp (the clamp is applied
// where it is read, so `s − basic` gives part A back exactly) and the maxima-normalised part
// (`basic_o`, ≤ 8 cards × 700); lo / hi fold the clamped value. Valid on `sub == 0` when `act`.
__device__ __forceinline__ uint64_t score_node_b_k(const yoda_dev_node_t* nd, bool act, uint32_t emask,
                                                   const ScoreConsts& sc, int sub, uint64_t rbase,
                                                   unsigned long long& lo, unsigned long long& hi, uint32_t& basic_o) {
  uint64_t basic = 0;
  if (act && sc.yoda_s && ((emask >> sub) & 1u)) {
    const yoda_dev_card_t cd = nd->cards[sub];
    const uint64_t ef = eff_free(cd.free, cd.pending, cd.total, cd.reserved);
    basic = udiv_r((uint64_t)cd.bandwidth * 100, sc.mx[0], sc.rmx[0]) +
            udiv_r((uint64_t)cd.clock * 100, sc.mx[1], sc.rmx[1]) +
            udiv_r((uint64_t)cd.core * 100, sc.mx[2], sc.rmx[2]) +
            udiv_r((uint64_t)cd.power * 100, sc.mx[4], sc.rmx[4]) +
            udiv_r(ef * 100, sc.mx[3], sc.rmx[3]) * 2 + udiv_r((uint64_t)cd.total * 100, sc.mx[5], sc.rmx[5]);
  }
  basic_o = gsum((uint32_t)basic);
  uint64_t s = 0;
  if (act && sub == 0 && sc.yoda_s) {
    s = basic_o + rbase;
    const unsigned long long us = s > (uint64_t)LLONG_MAX ? 0ull : s;
    lo = us < lo ? us : lo;
    hi = us > hi ? us : hi;
  }
  return s;
}

// SPEC: what makes two pods' maxima differ on the same cards — the clock requirement (a pod held
// to one clock only sees those cards); the speculation table's key and slot
__device__ __forceinline__ uint64_t spec_key(const yoda_dev_req_t& r) {
  return ((uint64_t)r.has_clock << 63) ^ (r.clock << 24) ^ r.clock_min;
}
__device__ __forceinline__ int spec_slot(uint64_t key) { return (int)((key * 0x9E3779B97F4A7C15ull) >> 62); }

// Both parts (the per-pod launch chain's k_score).
__device__ __forceinline__ void score_node(const yoda_dev_node_t* nd, bool act, uint32_t emask,
                                           const yoda_dev_req_t& r, const ScoreConsts& sc,
                                           const uint8_t* s_masks, int sub, int64_t& raw_o, int64_t& total_o,
                                           uint32_t& mask_o, int32_t& quality_o, unsigned long long& lo,
                                           unsigned long long& hi) {
  uint64_t rbase = 0;
  score_node_a(nd, act, emask, r, sc, s_masks, sub, rbase, total_o, mask_o, quality_o);
  const int64_t raw = score_node_b(nd, act, emask, sc, sub, rbase, lo, hi);
  if (act && sub == 0) raw_o = raw;
}

__global__ __launch_bounds__(kBlock) void k_score(yoda_dev_node_t* __restrict__ nodes, int n,
                                                  const yoda_dev_req_t r, const uint8_t* __restrict__ feas,
                                                  const uint8_t* __restrict__ elig, int64_t* __restrict__ raw,
                                                  int64_t* __restrict__ total_out, uint32_t* __restrict__ mask_out,
                                                  int32_t* __restrict__ quality_out, Globals* __restrict__ g,
                                                  yoda_dev_result_t* __restrict__ out, int fuse_select) {
  __shared__ unsigned long long s_lo[kWaves], s_hi[kWaves];
  __shared__ bool s_last;
  __shared__ uint8_t s_masks[256];   // subset table in LDS: the search loop reads it every step
  static_assert(kBlock == 256, "one table byte per thread");
  s_masks[threadIdx.x] = c_subsets.masks[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = uniform(threadIdx.x >> 6);
  const int grp = lane >> 3, sub = lane & 7;
  const uint64_t gmx[6] = {g->maxima[0], g->maxima[1], g->maxima[2], g->maxima[3], g->maxima[4], g->maxima[5]};
  const ScoreConsts sc = score_consts(r, gmx);
  unsigned long long lo = ULLONG_MAX, hi = 0;
  const int stride = gridDim.x * kWaves * kNodesPerWave;
  for (int base = uniform((blockIdx.x * kWaves + wave) * kNodesPerWave); base < n; base += stride) {
    const int i = base + grp;
    // no early exit on an all-infeasible wave: the node loads below then issue together
    // with feas/elig instead of one round trip later
    const bool act = i < n && feas[i];
    const yoda_dev_node_t* nd = nodes + (i < n ? i : n - 1);
    const uint32_t emask = act ? elig[i] : 0u;
    int64_t raw_v = 0, total_v = 0;
    uint32_t mask_v = 0;
    int32_t quality_v = 0;
    score_node(nd, act, emask, r, sc, s_masks, sub, raw_v, total_v, mask_v, quality_v, lo, hi);
    if (act && sub == 0) {
      raw[i] = raw_v;
      total_out[i] = total_v;
      mask_out[i] = mask_v;
      quality_out[i] = quality_v;
    }
  }
  // wave-level min/max of the raw score (lanes that scored nothing hold the identities)
  lo = wave_min(lo);
  hi = wave_max(hi);
  if (lane == 0) {
    s_lo[wave] = lo;
    s_hi[wave] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0 && sc.yoda_s) {
    unsigned long long blo = ULLONG_MAX, bhi = 0;
    for (int w = 0; w < kWaves; ++w) {
      blo = s_lo[w] < blo ? s_lo[w] : blo;
      bhi = s_hi[w] > bhi ? s_hi[w] : bhi;
    }
    if (blo != ULLONG_MAX) min_if(&g->raw_lo, blo, r.dev_flags & 1u);
    if (bhi) max_if(&g->raw_hi, bhi, r.dev_flags & 1u);
  }
  if (!fuse_select) return;
  // last block in: every block's raw/total/mask/quality stores and lo/hi atomics are visible
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(&g->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const unsigned long long best = select_block(n, r, feas, raw, total_out, g, 0, 1);
  if (threadIdx.x == 0) publish(n, r, best, mask_out, quality_out, g, out, nodes);
}

// ------------------------------------------------------------------ K3: normalize + argmax + result
__global__ __launch_bounds__(kBlock) void k_select(int n, const yoda_dev_req_t r, const uint8_t* __restrict__ feas,
                                                   const int64_t* __restrict__ raw, const int64_t* __restrict__ total,
                                                   const uint32_t* __restrict__ mask, const int32_t* __restrict__ quality,
                                                   Globals* __restrict__ g, yoda_dev_result_t* __restrict__ out,
                                                   yoda_dev_node_t* __restrict__ nodes) {
  __shared__ bool s_last;
  const unsigned long long b = select_block(n, r, feas, raw, total, g, blockIdx.x, gridDim.x);
  if (threadIdx.x == 0) {
    if (b) max_if(&g->best_key, b, r.dev_flags & 1u);
    // release this block's contribution, then take a ticket (agent scope: other XCDs)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(&g->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last || threadIdx.x != 0) return;
  // last block: every other block's atomicMax has landed
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const unsigned long long key = __hip_atomic_load(&g->best_key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  publish(n, r, key, mask, quality, g, out, nodes);
}

// ------------------------------------------------------------------ persistent batch kernel
// k_batch: ONE dispatch schedules a whole batch of pods (filter → maxima → score/gang →
// normalise/argmax → assume, pod after pod) with the node table resident in LDS.
//
//  * block g owns nodes [g*npb, g*npb + npb) for the whole launch; their 512-B rows are read
//    into LDS once (plus the host's pending dirty rows) and every phase of every pod reads them
//    from there — no HBM round trip inside the batch. The winner's owner applies the assume to
//    its LDS row (the same update as `publish`, dev_flags bit 1), so pod b+1 sees pod b's
//    reservation; dirty rows go back to the table at the end.
//  * the three cross-workgroup reductions of a pod (maxima + feasible/reason counts, raw
//    lo/hi, best key) are all-gathers of 8-byte {tag, value} granules: every block stores its
//    partial record write-through (agent-scope relaxed atomic store = sc1), then one thread
//    per producer block polls that record until every tag equals the phase's epoch and the
//    block reduces the G records itself. The data is the flag: no fence, no counter, no
//    reset (tags grow monotonically across launches). Each record kind has its own slot
//    (tag mod 3: tags are epoch + 3·pod + kind, epochs ≡ 1 mod 3): a block overwrites its
//    record of one kind only after an exchange of another kind that every block joined after
//    reading the first — also when a pod skips record 2 (speculated maxima, below).
//  * the batch's requests are read from mapped host memory, req b+1 prefetched during pod b;
//    results collect in a device buffer and the last block (agent release/acquire ticket)
//    copies them to mapped host memory and raises `done` with a system-scope release.
//  * every spin is bounded (abort word + s_memrealtime deadline): a block that never arrives
//    makes every waiter give up, the host sees `done` missing and falls back.
constexpr int kMaxNodesPerBlock = 256;    // 256 × 542 B of LDS per block (+ the batch's score columns)
constexpr int kRecStride = 16;            // granules per record slot
// record 1: maxima[6], feasible, 8 reason counts packed 2 × u16; with score columns (COLS) the
// feasible granule carries PodTopologySpread's feasible non-ignored nodes in its high half, and
// the domain mask of those follows (lo, hi)
// (a batch without score columns — COLS false — keeps the shorter records: 11 / 4 / 2-3)
constexpr int kRec1 = 13;
// SPEC kernels (PAIRS without columns): record 1 also carries the block's raw lo / hi under the
// speculated maxima (granules 11..14)
constexpr int kRec1S = 7 + (8 + 1) / 2 + 4;
constexpr int kRec2 = 6;                  // raw lo, hi (2 granules each), spread lo, hi (1 each: int32 ≥ 0)
constexpr int kRec3 = 3;                  // best key (2 granules), the block best's mask / flags / domains
constexpr int kMaxGrid = 256;
constexpr int kSP = YODA_DEV_SPREAD_SLOTS, kIMG = YODA_DEV_IMAGE_SLOTS, kDOM = YODA_DEV_DOMAINS;
// LDS bytes per node: row + raw + total + quality + basic + 2 × feas + 2 × elig + mask + dirty; a batch
// with score columns adds batch_col_bytes (spread raw + per slot count and domain, per image
// slot its score)
constexpr size_t kBatchRowBytes = sizeof(yoda_dev_node_t) + 8 + 8 + 4 + 4 + 6;
__host__ __device__ constexpr size_t batch_col_bytes(int n_sp, int n_img) {
  return (n_sp > 0 ? 4 + 5 * (size_t)n_sp : 0) + 4 * (size_t)n_img;
}
constexpr int kMaxGroups = kMaxNodesPerBlock / kNodesPerWave;   // 8-node filter groups per block
// reason codes the batch path can produce (no candidate reasons: the engine sends no
// candidates to batches), packed into granules 7..10 of record 1
constexpr int kNR = 8;                    // reason codes a batch can produce (record 1 packs 2 per granule)
constexpr int kRsPairs = (kNR + 1) / 2;   // their granules
// per-group aggregates (s_grp): 0..5 maxima (max), 6 feasible (sum), 7.. reasons (sum), then
// spread's feasible non-ignored nodes (sum) and domain mask (or, two halves)
constexpr int kFNfi = 7 + kNR, kFDlo = 8 + kNR, kFDhi = 9 + kNR, kNF1 = 10 + kNR;
// record 1 transposed for the reduction (s_rec / s_glob fields). Without columns the reason
// pairs are unpacked: 0..5 maxima, 6 feasible, 7..14 reasons (15 fields). With columns the
// granules are reduced as they are — feasible | non-ignored << 16 and the reason pairs summed as
// u16 halves (the host keeps such batches below 65536 nodes), the domain halves or-ed — so the
// 13 fields fit one 16-lane pass of a 4-wave block (18 unpacked fields took a second pass:
// ~1.1 µs per pod on the PAIRS fix-up owner's critical path, profiles/device/r6/)
constexpr int kGDlo = 7 + kRsPairs, kGDhi = 8 + kRsPairs;   // record-1 granules of the domain mask
constexpr int kNF1T = 7 + kNR;                              // the most transposed fields (no columns)
__constant__ int c_batch_reasons[kNR] = {RS_UNSCHEDULABLE, RS_RESOURCES, RS_NO_SCV, RS_STALE, RS_GPU_NUMBER,
                                         RS_GPU_FIT, RS_DEAD, RS_EXT_RESOURCES};

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

struct BatchArgs {
  PatchArgs pa;                       // host reservations since the last launch (dirty rows)
  yoda_dev_node_t* nodes;
  int n, npb, B, seq;
  uint32_t tag0;                      // epoch of record 1 of pod 0 (tags: tag0 + 3b + phase)
  long long deadline_ticks;           // per spin, s_memrealtime ticks (100 MHz)
  const yoda_dev_req_t* reqs;         // device view of mapped host memory
  unsigned long long* slots;          // [3][kMaxGrid][kRecStride]: records 3, 1, 2 (tag mod 3)
  yoda_dev_result_t* res;             // device scratch, one per pod
  yoda_dev_result_t* out;             // device view of mapped host memory
  int32_t* done;                      // mapped host word: seq when `out` is complete
  unsigned int* ticket;
  unsigned int* abort_word;
  unsigned long long* trace;          // optional: block 0's phase stamps, kTracePts per pod
  // score columns of this batch (yoda_dev_batch_extras; device views of mapped host memory,
  // read once in the prologue); n_sp / n_img = 0: none
  const int32_t* sp_cnt;              // [n_sp][n] the slot selector's matching pods per node
  const uint8_t* sp_dom;              // [n_sp][n] the node's domain, YODA_DEV_DOM_NONE: ignored
  const int32_t* sp_zc;               // [n_sp][kDOM] matching pods per domain
  const int32_t* img;                 // [n_img][n] weighted ImageLocality scores
  const double* logtab;               // log(i + 2) (the host's libm): PodTopologySpread weights
  int n_sp, n_img;
};
constexpr int kResWords = (int)(sizeof(yoda_dev_result_t) / 8);
static_assert(kResWords == 19 && YODA_DEV_REASONS == 16 && offsetof(yoda_dev_result_t, feasible) == 4 &&
                  offsetof(yoda_dev_result_t, score) == 8 && offsetof(yoda_dev_result_t, mask) == 16 &&
                  offsetof(yoda_dev_result_t, quality) == 20 && offsetof(yoda_dev_result_t, reasons) == 24 &&
                  offsetof(yoda_dev_result_t, maxima) == 88 && offsetof(yoda_dev_result_t, raw_lo) == 136 &&
                  offsetof(yoda_dev_result_t, raw_hi) == 144,
              "the publish step's word layout");
// the reason codes of c_batch_reasons, for compile-time indexing
constexpr int kBatchReasonCodes[kNR] = {RS_UNSCHEDULABLE, RS_RESOURCES, RS_NO_SCV, RS_STALE, RS_GPU_NUMBER,
                                        RS_GPU_FIT, RS_DEAD, RS_EXT_RESOURCES};
static_assert(kRec1S == 7 + kRsPairs + 4 && kRec1S <= kRecStride, "SPEC record 1: the plain record + raw lo / hi");
static_assert(7 + kRsPairs + 2 == kRec1 && kRec1 <= kNF1T && kRec1 <= 16,
              "record 1: 7 fields + the reason counts as u16 pairs + 2 domain-mask granules, one reduction pass");
constexpr int kTracePts = 24;   // 9 phase stamps per pod (block 0), 9 of the PAIRS fix-up's owner, padded
constexpr int kReqWords = sizeof(yoda_dev_req_t) / 4;
static_assert(sizeof(yoda_dev_req_t) % 4 == 0 && kReqWords <= 64, "req fits one wave");

__device__ __forceinline__ gu64* slot_ptr(const BatchArgs& a, uint32_t tag, int blk) {
  return (gu64*)(a.slots + ((size_t)(tag % 3u) * kMaxGrid + blk) * kRecStride);
}

__device__ __forceinline__ void store_granule(gu64* p, uint32_t tag, uint32_t v) {
  __hip_atomic_store(p, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// true = keep spinning; false = give up (another block aborted, or the deadline passed)
__device__ __forceinline__ bool spin_ok(const BatchArgs& a, unsigned& spins, long long t0) {
  __builtin_amdgcn_s_sleep(1);
  // the abort word and the clock every 64 spins; every spin under a sub-millisecond deadline
  // (the failure-path test forces aborts with one)
  const unsigned every = a.deadline_ticks < 100000 ? 0u : 63u;
  if ((++spins & every) != 0) return true;
  const unsigned ab = __hip_atomic_load((gu32*)a.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (uniform((int)ab)) return false;
  if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.deadline_ticks) {
    __hip_atomic_store((gu32*)a.abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  return true;
}

// Records are read two granules (16 B) per request: buffer_load_dwordx4 with sc1, the
// coherence bits of __hip_atomic_load's agent-scope dwordx2. Every granule is still written by
// one 8-byte atomic store and carries its own tag, so a pair caught between two stores only
// fails its tag check. A gather is request-bound — each of the G blocks reads G records, and
// every granule of a record costs G² requests chip-wide (MI355X, 4096 nodes, G = 256 blocks:
// 3 more granules per record 1 cost ~1 µs per pod) — so halving the requests is what counts.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// (+ one slot per block set for SPEC's fix-up record: the PAIRS owner's re-scored group lo / hi)
constexpr uint32_t kSlotBytes = (3u * kMaxGrid + 2u) * kRecStride * 8u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slot_rsrc(const BatchArgs& a) {
  return __builtin_amdgcn_make_buffer_rsrc(a.slots, 0, (int)kSlotBytes, 0x00020000);
}
__device__ __forceinline__ uint32_t slot_off(uint32_t tag, int blk) {
  return (((tag % 3u) * kMaxGrid + (uint32_t)blk) * kRecStride) * 8u;
}
__device__ __forceinline__ uint32_t fix_slot_off(int set) { return ((3u * kMaxGrid + (uint32_t)set) * kRecStride) * 8u; }
// granules k, k + 1 of the slot at byte offset `off`; a lane outside the grid reads nothing and
// sees (0, tag) twice
__device__ __forceinline__ u32x4 load_pair(__amdgpu_buffer_rsrc_t rs, uint32_t off, int k, bool in, uint32_t tag) {
  if (!in) return u32x4{0u, tag, 0u, tag};
  return __builtin_amdgcn_raw_buffer_load_b128(rs, off + 8u * (uint32_t)k, 0, 16 /* sc1 */);
}
// granules 2.. of a record (granules 0, 1 were the poll); false if one is not yet from `tag`
template <int K>
__device__ __forceinline__ bool read_rest(__amdgpu_buffer_rsrc_t rs, uint32_t off, bool in, uint32_t tag,
                                          uint32_t (&v)[K]) {
  bool ok = true;
#pragma unroll
  for (int k = 2; k < K; k += 2) {   // (K odd: the pair's second granule lies inside the 16-granule slot)
    const u32x4 y = load_pair(rs, off, k, in, tag);
    v[k] = y.x;
    ok &= y.y == tag;
    if (k + 1 < K) {
      v[k + 1] = y.z;
      ok &= y.w == tag;
    }
  }
  return ok;
}
// the poll: granules 0 (and 1) of a record
template <int K>
__device__ __forceinline__ bool read_head(const u32x4& x, uint32_t tag, uint32_t (&v)[K]) {
  v[0] = x.x;
  if constexpr (K > 1) v[1] = x.z;
  return x.y == tag && (K < 2 || x.w == tag);
}

// Thread t < G polls the record of block p_off + t for epoch `tag` (K granules) until every
// tag matches; returns false (block-uniform) when the wait was abandoned.
template <int K>
__device__ __forceinline__ bool gather(const BatchArgs& a, uint32_t tag, int G, int p_off, uint32_t (&v)[K],
                                       int* s_fail) {
  const int t = threadIdx.x;
  bool failed = false;
  if (uniform(t & ~63) < G) {   // waves holding at least one producer
    const __amdgpu_buffer_rsrc_t rs = slot_rsrc(a);
    const bool in = t < G;
    const uint32_t off = slot_off(tag, p_off + (in ? t : 0));
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned spins = 0;;) {
      __asm__ volatile("" ::: "memory");   // every round reads the slots again
      // poll the first pair of every record until each has landed, then read the rest
      // (written in the same instant by the producer's other threads): a waiting block
      // loads G requests per round instead of G·K/2 — with G blocks all polling each other
      // that is the fabric traffic of the wait
      bool ok = read_head<K>(load_pair(rs, off, 0, in, tag), tag, v);
      if (__all(ok)) {
        ok = read_rest<K>(rs, off, in, tag, v);
        if (__all(ok)) break;
      }
      if (!spin_ok(a, spins, t0)) {
        failed = true;
        break;
      }
    }
  }
  if (failed && (threadIdx.x & 63) == 0) *s_fail = 1;
  __syncthreads();
  return *s_fail == 0;
}

// gather() for one wave alone, no barrier (G ≤ 128: lane t polls producers t and t + 64;
// producer `skip` is not polled — its values are left 0): wave 0 for records 2 / 3, and the
// PAIRS fix-up owner's gathering wave for record 1 while the block's other waves still score
// the winner's group. Returns false when the wait was abandoned (the caller raises s_fail).
template <int K>
__device__ __forceinline__ bool gather_wave0_2(const BatchArgs& a, uint32_t tag, int G, int p_off, uint32_t (&v)[K],
                                               uint32_t (&v2)[K], int skip) {
  const int t = threadIdx.x & 63, t2 = t + 64;
  const bool in = t < G && t != skip, in2 = t2 < G && t2 != skip;
  const __amdgpu_buffer_rsrc_t rs = slot_rsrc(a);
  const uint32_t off = slot_off(tag, p_off + (t < G ? t : 0)), off2 = slot_off(tag, p_off + (t2 < G ? t2 : 0));
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned spins = 0;;) {
    __asm__ volatile("" ::: "memory");
    bool ok = read_head<K>(load_pair(rs, off, 0, in, tag), tag, v);
    ok &= read_head<K>(load_pair(rs, off2, 0, in2, tag), tag, v2);
    if (__all(ok)) {
      ok = read_rest<K>(rs, off, in, tag, v);
      ok &= read_rest<K>(rs, off2, in2, tag, v2);
      if (__all(ok)) return true;   // (a skipped producer's values are 0)
    }
    if (!spin_ok(a, spins, t0)) return false;
  }
}
// one wave's gather; G ≤ 64: one producer per lane (v2 zeroed, unused), else two (gather_wave0_2)
template <int K>
__device__ __forceinline__ bool gather_wave0(const BatchArgs& a, uint32_t tag, int G, int p_off, uint32_t (&v)[K],
                                             uint32_t (&v2)[K], int skip = -1) {
  if (G > 64) return gather_wave0_2<K>(a, tag, G, p_off, v, v2, skip);
#pragma unroll
  for (int k = 0; k < K; ++k) v2[k] = 0;
  const int t = threadIdx.x & 63;
  const bool in = t < G && t != skip;
  const __amdgpu_buffer_rsrc_t rs = slot_rsrc(a);
  const uint32_t off = slot_off(tag, p_off + (t < G ? t : 0));
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  for (unsigned spins = 0;;) {
    __asm__ volatile("" ::: "memory");
    bool ok = read_head<K>(load_pair(rs, off, 0, in, tag), tag, v);
    if (__all(ok)) {
      ok = read_rest<K>(rs, off, in, tag, v);
      if (__all(ok)) return true;
    }
    if (!spin_ok(a, spins, t0)) return false;
  }
}

#define TRACE(pt)                                                                      \
  do {                                                                                 \
    if (a.trace && gi == 0 && tid == 0) a.trace[(size_t)b * kTracePts + (pt)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// BW waves per block (4 or 8): 8 puts two waves on every SIMD (latency hiding) and 64 nodes
// per block, halving the all-gather producers at a given cluster size.
//
// PAIRS: two pods in flight. The grid is two sets of blocks holding the same node ranges
// (replicated rows); set s runs pods s, s+2, s+4, …. While one set runs pod b's exchanges,
// score B and select, the other set has already filtered and scored pod b+1 against its rows
// (every assume up to pod b−1 applied). When pod b's winner is known (its record 3 carries the
// winner's GPU mask), the other set applies that assume to its replica and only the owner of the
// winner's node redoes that one 8-node group: its wave 0 re-filters it, sends record 1 and
// gathers the set's records 1, while waves 1.. choose the group's GPU sets and compute its
// scores (two halves on different waves, joined after the barrier): an assume changes one row,
// so every other node's filter and score A for pod b+1 stand. The per-pod critical path loses
// the filter and score A of every block but one group's; results are bit-identical to the
// serial order (reference: the per-pod cycle of scheduler.go:132-157 / algorithm.go:28-87,
// run for consecutive pods against the same node table).
template <int BW, bool PAIRS, bool COLS>
__global__ __launch_bounds__(64 * BW) void k_batch(const BatchArgs a) {
  constexpr int kBB = 64 * BW;
  // record sizes of this instantiation: score columns add spread fields to records 1 and 2 and
  // the winner's domains to record 3
  // SPEC (PAIRS without columns): every block runs phase B on its set's previous maxima before
  // record 1 (while the other set's exchanges run), record 1 carries the block's raw lo / hi,
  // and record 2 is exchanged only when the gathered maxima differ from the speculated ones —
  // one dependent exchange per pod instead of two before the best key (profiles/device/r6/:
  // the maxima repeat for 100 % of the bench mix's pods at normal load)
  constexpr bool SPEC = PAIRS && !COLS;
  constexpr int REC1 = SPEC ? kRec1S : COLS ? kRec1 : kRec1 - 2, REC2 = COLS ? kRec2 : kRec2 - 2;
  constexpr int REC3 = (COLS || PAIRS) ? kRec3 : kRec3 - 1, NF1 = COLS ? kRec1 : kNF1T;
  extern __shared__ __align__(16) unsigned char s_dyn[];
  __shared__ uint8_t s_masks[256];
  // request ring: pods b (and b−1 in PAIRS mode, for its assume) plus the prefetched next ones
  __shared__ __align__(16) uint32_t s_req[4][sizeof(yoda_dev_req_t) / 4];
  __shared__ int s_fix;   // PAIRS: the other set's last winner's row here, or −1
  __shared__ int s_fixg;  // PAIRS: the block (of this set) holding that row, or −1 (no winner)
  __shared__ unsigned long long s_fixlh[2];   // SPEC: the fix-up owner's re-scored group lo / hi
  __shared__ unsigned long long s_part[BW][16];
  __shared__ unsigned long long s_glob[kNF1T];
  // G ≤ 64: wave 0 holds every record of a gather and reduces it alone; the result reaches the
  // block through these words and one barrier (no per-wave partials, no second barrier)
  __shared__ unsigned long long s_red[4];
  __shared__ uint32_t s_rec[kNF1T][kMaxGrid + 4];   // gather-1 records transposed (+4: bank skew)
  // filter aggregates per 8-node group: 6 maxima, feasible count, the reason counts, spread's
  // feasible non-ignored count and domain mask halves
  __shared__ uint32_t s_grp[kMaxGroups][kNF1];
  // PodTopologySpread: matching pods per domain of each slot (every block keeps the whole table
  // and applies each winner), the last winner's record-3 granule 2 (its domains)
  __shared__ int32_t s_zc[kSP][kDOM];
  __shared__ uint32_t s_wdom;
  __shared__ GangBest s_gang[8 * BW];
  __shared__ int s_fail;
  __shared__ uint32_t s_bfeas;   // this block's feasible nodes for the current pod (record 1)
  // SPEC: the maxima this set's last pod gathered (the speculation; 1s before its first pod) and
  // each 8-node group's raw lo / hi under them
  __shared__ uint64_t s_spec[6];
  // … per clock requirement too (a pod limited to one clock sees other cards' maxima): 4 entries
  // {key, maxima}; the speculation is the entry of the pod's key, else the last pod's
  __shared__ uint64_t s_ptab[4][7];
  __shared__ uint64_t s_cur[6];   // this pod's speculated maxima
  __shared__ unsigned long long s_glh[kMaxGroups][2];
  __shared__ bool s_last;
  static_assert(sizeof(yoda_dev_result_t) % 8 == 0, "result copied as u64 words");

  const int npb = a.npb, g = blockIdx.x;
  // G: the blocks that produce one pod's records (one set in PAIRS mode); gi: this block's node
  // range; p0 / q0: the first block of this set / of the other set
  const int G = PAIRS ? (int)gridDim.x / 2 : (int)gridDim.x;
  const int set = PAIRS ? g / G : 0;
  const int gi = g - set * G;
  const int p0 = set * G, q0 = (1 - set) * G;
  const int base = gi * npb;
  const int cnt = a.n - base < npb ? a.n - base : npb;   // ≥ 1: the host sizes G = ceil(n / npb)
  yoda_dev_node_t* s_rows = reinterpret_cast<yoda_dev_node_t*>(s_dyn);
  int64_t* s_raw = reinterpret_cast<int64_t*>(s_dyn + (size_t)npb * sizeof(yoda_dev_node_t));
  int64_t* s_total = s_raw + npb;
  int32_t* s_quality = reinterpret_cast<int32_t*>(s_total + npb);
  // the batch's score columns (sized by a.n_sp / a.n_img: absent without slots)
  int32_t* s_sp = s_quality + npb;                                    // spread raw score, −1: ignored
  int32_t* s_cnt = s_sp + (a.n_sp > 0 ? npb : 0);                     // [n_sp][npb] matching pods
  int32_t* s_img = s_cnt + a.n_sp * npb;                              // [n_img][npb] ImageLocality
  // phase B's maxima part of s_raw (32-bit: a wrong speculation, e.g. the 1s before a set's
  // first pod, can make it exceed 16 bits)
  uint32_t* s_basic = reinterpret_cast<uint32_t*>(s_img + a.n_img * npb);
  uint8_t* s_feas2 = reinterpret_cast<uint8_t*>(s_basic + npb);           // [2][npb] by pod parity
  uint8_t* s_elig2 = s_feas2 + 2 * npb;                               // [2][npb]
  uint8_t* s_mask = s_elig2 + 2 * npb;
  uint8_t* s_dirty = s_mask + npb;
  uint8_t* s_dom = s_dirty + npb;                                     // [n_sp][npb] domains
  const int tid = threadIdx.x, lane = tid & 63, wave = uniform(tid >> 6);
  const int grp = lane >> 3, sub = lane & 7;

  // ---- prologue: rows → LDS (a pending host row replaces the table's), subsets, request 0
  for (int t = tid; t < cnt * 32; t += kBB) {
    const int row = t >> 5, part = t & 31, i = base + row;
    int pj = -1;
    for (int j = 0; j < a.pa.n; ++j) pj = a.pa.idx[j] == i ? j : pj;
    const uint4 v = pj >= 0 ? reinterpret_cast<const uint4*>(&a.pa.rows[pj])[part]
                            : reinterpret_cast<const uint4*>(a.nodes + i)[part];
    reinterpret_cast<uint4*>(s_rows + row)[part] = v;
    if (part == 0) s_dirty[row] = pj >= 0;
  }
  // pending rows outside [0, n) belong to no block: block 0 writes them through
  if (g == 0 && (tid >> 5) < a.pa.n && a.pa.idx[tid >> 5] >= a.n) {
    const int rec = tid >> 5;
    reinterpret_cast<uint4*>(a.nodes + a.pa.idx[rec])[tid & 31] = reinterpret_cast<const uint4*>(&a.pa.rows[rec])[tid & 31];
  }
  if (tid < 256) s_masks[tid] = c_subsets.masks[tid];
  // score columns of the batch (one burst per block from mapped host memory)
  if constexpr (COLS)
  for (int t = tid; t < a.n_sp * cnt; t += kBB) {
    const int sl = t / cnt, row = t - sl * cnt;
    s_cnt[sl * npb + row] = a.sp_cnt[(size_t)sl * a.n + base + row];
    s_dom[sl * npb + row] = a.sp_dom[(size_t)sl * a.n + base + row];
  }
  if constexpr (COLS)
  for (int t = tid; t < a.n_img * cnt; t += kBB) {
    const int sl = t / cnt, row = t - sl * cnt;
    s_img[sl * npb + row] = a.img[(size_t)sl * a.n + base + row];
  }
  if constexpr (COLS)
    for (int t = tid; t < a.n_sp * kDOM; t += kBB) s_zc[t / kDOM][t % kDOM] = a.sp_zc[t];
  if (tid < kReqWords) {
    s_req[0][tid] = reinterpret_cast<const uint32_t*>(a.reqs)[tid];
    if (PAIRS && a.B > 1) s_req[1][tid] = reinterpret_cast<const uint32_t*>(a.reqs + 1)[tid];
  }
  if (tid == 0) s_fail = 0;
  if (tid < 6) s_spec[tid] = 1;
  if (tid < 4) s_ptab[tid][0] = ~0ull;
  __syncthreads();

  // Filter every 8-node group of this block for request `rq` (or only group `only`) into the
  // parity-`par` feasibility arrays (pod parity: phase A of a pod never reads what the next
  // pod's filter writes) and the per-group aggregates s_grp. Wave-uniform.
  auto filter_one = [&](const yoda_dev_req_t& rq, int par, int gq) {
      uint8_t* fe = s_feas2 + par * npb;
      uint8_t* el = s_elig2 + par * npb;
      const int j = gq * kNodesPerWave + grp;
      const bool valid = j < cnt;
      uint32_t wmx[6] = {1, 1, 1, 1, 1, 1};
      uint32_t emask = 0;
      const int reason = filter_eval(s_rows + (valid ? j : 0), valid, rq, 0, wmx, emask, grp, sub);
      const bool fok = valid && reason == 0;
      if (valid && sub == 0) {
        fe[j] = fok;
        el[j] = (uint8_t)emask;
      }
      const bool head = sub == 0;
      const uint32_t nf = (uint32_t)__popcll(__ballot(head && fok));
      uint32_t rc[kNR];
#pragma unroll
      for (int q = 0; q < kNR; ++q) rc[q] = (uint32_t)__popcll(__ballot(head && reason == c_batch_reasons[q]));
      // PodTopologySpread (soft): the feasible nodes carrying every key of the pod's slot, and
      // the domains among them (upstream initPreScoreState's topology sizes)
      uint32_t nfi = 0, dlo = 0, dhi = 0;
      if constexpr (COLS) {
        const int sl = rq.spread_slot;
        if (sl >= 0) {   // wave-uniform
          const uint32_t d = valid ? s_dom[sl * npb + j] : (uint32_t)YODA_DEV_DOM_NONE;
          const bool counted = head && fok && d != YODA_DEV_DOM_NONE;
          nfi = (uint32_t)__popcll(__ballot(counted));
          dlo = wave_or(counted && d < 32 ? 1u << d : 0u);
          dhi = wave_or(counted && d >= 32 ? 1u << (d - 32) : 0u);
        }
      }
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) s_grp[gq][k] = wmx[k];
        s_grp[gq][6] = nf;
#pragma unroll
        for (int q = 0; q < kNR; ++q) s_grp[gq][7 + q] = rc[q];
        if constexpr (COLS) {
          s_grp[gq][kFNfi] = nfi;
          s_grp[gq][kFDlo] = dlo;
          s_grp[gq][kFDhi] = dhi;
        }
      }
  };
  // a gathered record 1 into column t of the transposed fields (without columns the reason
  // pairs are unpacked; with columns every granule is a field as it is)
  auto transpose1 = [&](const uint32_t (&v)[REC1], int t) {
    if constexpr (COLS) {
#pragma unroll
      for (int k = 0; k < REC1; ++k) s_rec[k][t] = v[k];
    } else {
#pragma unroll
      for (int k = 0; k < 7; ++k) s_rec[k][t] = v[k];
#pragma unroll
      for (int q = 0; q < kNR; ++q) s_rec[7 + q][t] = (q & 1) ? (v[7 + q / 2] >> 16) : (v[7 + q / 2] & 0xFFFFu);
    }
  };
  auto filter_groups = [&](const yoda_dev_req_t& rq, int par) {
    for (int gq = wave; gq * kNodesPerWave < cnt; gq += BW) filter_one(rq, par, gq);
  };
  // record 1 from the group aggregates: threads 0..REC1-1 (wave 0), after every group's
  // s_grp row is visible to them
  // (SPEC: the raw lo / hi leave out group `skipq` — the PAIRS owner's group, whose lo / hi follow
  // in the fix-up record once re-scored)
  auto record1 = [&](uint32_t tag1, int skipq = -1, bool own_lh = false) -> uint32_t {
    uint32_t v = 0;
    unsigned long long blo = ULLONG_MAX, bhi = 0;   // SPEC: over the groups but skipq, wave 0
    if constexpr (SPEC) {
      if (wave == 0) {   // (wave-uniform) one group per lane, one LDS round trip
        const int ngr = (cnt + kNodesPerWave - 1) / kNodesPerWave;
        if (lane < ngr && lane != skipq) {
          blo = s_glh[lane][0];
          bhi = s_glh[lane][1];
        }
        blo = wave_min(blo);
        bhi = wave_max(bhi);
        if (own_lh && tid == 0) {   // the PAIRS owner's own lo / hi beside the others' (gather_early)
          s_red[2] = blo;
          s_red[3] = bhi;
        }
      }
    }
    if (tid < REC1) {   // block totals over the groups → the record's 11 granules
      const int ngr = (cnt + kNodesPerWave - 1) / kNodesPerWave;
      if (tid < 7) {
        v = tid < 6 ? 1u : 0u;
        for (int q = 0; q < ngr; ++q) v = tid < 6 ? (s_grp[q][tid] > v ? s_grp[q][tid] : v) : v + s_grp[q][tid];
        if (tid == 6) {
          s_bfeas = v;
          if constexpr (COLS) {   // + the feasible non-ignored nodes (≤ npb ≤ 256 each)
            uint32_t nfi = 0;
            for (int q = 0; q < ngr; ++q) nfi += s_grp[q][kFNfi];
            v |= nfi << 16;
          }
        }
      } else if (tid < 7 + kRsPairs) {   // reason counts packed as u16 pairs (≤ npb ≤ 256 per block)
        const int r0 = 7 + 2 * (tid - 7);
        uint32_t lo = 0, hi = 0;
        for (int q = 0; q < ngr; ++q) {
          lo += s_grp[q][r0];
          hi += r0 + 1 < 7 + kNR ? s_grp[q][r0 + 1] : 0u;
        }
        v = lo | (hi << 16);
      } else if constexpr (COLS) {   // spread: the domain mask halves (or)
        const int f = tid == kGDlo ? kFDlo : kFDhi;
        for (int q = 0; q < ngr; ++q) v |= s_grp[q][f];
      } else if constexpr (SPEC) {   // raw lo (11, 12) / hi (13, 14) over the groups, as u32 halves
        const unsigned long long x = tid < 7 + kRsPairs + 2 ? blo : bhi;
        v = ((tid - 7 - kRsPairs) & 1) ? (uint32_t)(x >> 32) : (uint32_t)x;
      }
      store_granule(slot_ptr(a, tag1, g) + tid, tag1, v);
    }
    return v;   // (thread tid's granule; 0 beyond the record)
  };

  // Replica 0 of each node in [j_lo, j_lo + span) scored with its own subset best: where
  // another of the `nrep` replicas (s_gang[q·span + node]) found a better set, take it and move
  // the gang bonus (the only score term that depends on the set). After a barrier.
  auto merge_gang = [&](const yoda_dev_req_t& r, const ScoreConsts& sc, const uint8_t* s_feas, int j_lo, int span,
                        int nrep) {
    for (int j = j_lo + tid; j < cnt && j < j_lo + span; j += kBB) {
      if (!s_feas[j]) continue;
      const GangBest b0 = s_gang[j - j_lo];
      GangBest bb = b0;
      for (int q = 1; q < nrep; ++q) {
        const GangBest o = s_gang[q * span + (j - j_lo)];
        if (o.found && (!bb.found || better(o.o, o.m, bb.o, bb.m))) bb = o;
      }
      if (bb.found == b0.found && bb.m == b0.m) continue;
      const int32_t q_old = s_quality[j];
      const int32_t q_new = bb.found ? 10000 - sdiv_small_r(bb.lb, 100, 0.01) : 10000;
      s_mask[j] = bb.m;
      s_quality[j] = q_new;
      if (sc.yoda_s && r.has_number && r.number > 1 && r.number <= s_rows[j].ncards) {
        uint64_t rb = (uint64_t)s_raw[j];
        if (b0.found) rb -= (uint64_t)(q_old / 100) * (uint64_t)r.w_gang_score;
        if (bb.found) rb += (uint64_t)(q_new / 100) * (uint64_t)r.w_gang_score;
        s_raw[j] = (int64_t)rb;
      }
    }
  };

  // Score A (gang search, the yoda terms that need no maxima — kept in s_raw until phase B —,
  // default scores) for the 8-node groups [gfirst, gfirst + gcount) of this block. A
  // multi-GPU pod's subset search is split over `nrep` lane groups per node when the block has
  // more waves than those groups (8 waves over 32 nodes: two groups per node); the replicas'
  // bests meet through LDS. Wave-uniform.
  const int ngroups = (npb + kNodesPerWave - 1) / kNodesPerWave;
  auto score_a_groups = [&](const yoda_dev_req_t& r, const ScoreConsts& sc, const uint8_t* s_feas,
                            const uint8_t* s_elig, int gfirst, int gcount) {
    const int nrep = (sc.search && sc.k > 1 && gcount <= BW) ? BW / gcount : 1;
    const int span = gcount * kNodesPerWave, j_lo = gfirst * kNodesPerWave;
    for (int it = wave; it < gcount * nrep; it += BW) {
      const int rep = it / gcount;
      const int j = j_lo + (it - rep * gcount) * kNodesPerWave + grp;
      const bool act = j < cnt && s_feas[j];
      const uint32_t emask = act ? s_elig[j] : 0u;
      uint64_t rbase = 0;
      int64_t total_v = 0;
      uint32_t mask_v = 0;
      int32_t quality_v = 0;
      // a replica's best goes straight to its LDS slot (< nrep·span ≤ 8·BW; a pointer to a
      // local would put the struct in scratch memory)
      score_node_a(s_rows + (j < cnt ? j : 0), act, emask, r, sc, s_masks, sub, rbase, total_v, mask_v, quality_v,
                   rep, nrep, nrep > 1 ? &s_gang[rep * span + (j - j_lo)] : nullptr);
      if (act && sub == 0 && rep == 0) {
        s_raw[j] = (int64_t)rbase;
        s_total[j] = total_v;
        s_mask[j] = (uint8_t)mask_v;
        s_quality[j] = quality_v;
      }
    }
    if (nrep > 1) {
      __syncthreads();
      merge_gang(r, sc, s_feas, j_lo, span, nrep);
    }
  };

  // PAIRS fix-up, score A of group `gq` on waves 1..BW−1 while wave 0 re-filters it for record 1:
  // each scoring wave evaluates the group's filter verdict and eligible mask itself (no LDS
  // hand-off from wave 0). The two independent halves of score A run on different waves: waves
  // 1..nrep choose the GPU set (a multi-GPU subset search split over them, replica wave−1, into
  // s_gang), wave nrep+1 computes the scores without the set's gang bonus (into s_raw /
  // s_total); `combine_fix` joins them after the barrier that also joins wave 0.
  auto score_a_fix = [&](const yoda_dev_req_t& r, const ScoreConsts& sc, int gq, int nrep, int tb) {
    const bool gang = wave >= 1 && wave <= nrep, scores = wave == nrep + 1;
    if (!gang && !scores) return;   // wave-uniform
    const int j = gq * kNodesPerWave + grp;
    const bool valid = j < cnt;
    const yoda_dev_node_t* nd = s_rows + (valid ? j : 0);
    uint32_t wmx_unused[6], emask = 0;
    const int reason = filter_eval<false>(nd, valid, r, 0, wmx_unused, emask, grp, sub);
    const bool act = valid && reason == 0;
    if (a.trace && tid == 64) a.trace[(size_t)tb * kTracePts + 14] = __builtin_amdgcn_s_memrealtime();
    uint64_t rbase = 0;
    int64_t total_v = 0;
    uint32_t mask_v = 0;
    int32_t quality_v = 0;
    if (gang) {
      score_node_a(nd, act, act ? emask : 0u, r, sc, s_masks, sub, rbase, total_v, mask_v, quality_v, wave - 1, nrep,
                   &s_gang[(wave - 1) * kNodesPerWave + grp],
                   (a.trace && tid == 64) ? a.trace + (size_t)tb * kTracePts + 16 : nullptr, 1);
      if (a.trace && tid == 64) a.trace[(size_t)tb * kTracePts + 15] = __builtin_amdgcn_s_memrealtime();
    } else {
      score_node_a(nd, act, act ? emask : 0u, r, sc, s_masks, sub, rbase, total_v, mask_v, quality_v, 0, 1, nullptr,
                   nullptr, 2);
      if (act && sub == 0) {
        s_raw[j] = (int64_t)rbase;
        s_total[j] = total_v;
      }
    }
  };
  // after the barrier: the best of the nrep GPU-set replicas of each feasible node of the group,
  // its mask, gang quality and (multi-GPU yoda pods) the gang bonus the scores wave left out —
  // the same terms score_node_a adds when it does both halves
  auto combine_fix = [&](const yoda_dev_req_t& r, const ScoreConsts& sc, const uint8_t* s_feas, int j_lo, int nrep) {
    if (tid < kNodesPerWave) {
      const int j = j_lo + tid;
      if (j < cnt && s_feas[j]) {
        GangBest bb = s_gang[tid];
        for (int q = 1; q < nrep; ++q) {
          const GangBest o = s_gang[q * kNodesPerWave + tid];
          if (o.found && (!bb.found || better(o.o, o.m, bb.o, bb.m))) bb = o;
        }
        const int32_t quality = bb.found ? 10000 - sdiv_small_r(bb.lb, 100, 0.01) : 10000;
        s_mask[j] = bb.found ? bb.m : 0u;
        s_quality[j] = quality;
        if (sc.yoda_s && r.has_number && r.number > 1 && r.number <= s_rows[j].ncards && bb.found)
          s_raw[j] = (int64_t)((uint64_t)s_raw[j] + (uint64_t)(quality / 100) * (uint64_t)r.w_gang_score);
      }
    }
  };

  // SPEC phase B on the speculated maxima (in `sc`) for 8-node groups gfirst + wstart, + wstep,
  // … < gend: each group's raw scores (s_raw: part A → the full raw score, s_basic: the maxima
  // part, so a wrong speculation is undone exactly) and its lo / hi (s_glh). Wave-uniform.
  auto phase_b_groups = [&](const ScoreConsts& sc, const uint8_t* s_feas, const uint8_t* s_elig, int gfirst, int gend,
                            int wstart, int wstep) {
    for (int gq = gfirst + wstart; gq < gend; gq += wstep) {
      const int j = gq * kNodesPerWave + grp;
      const bool act = j < cnt && s_feas[j];
      const uint32_t emask = act ? s_elig[j] : 0u;
      const uint64_t rbase = (act && sub == 0) ? (uint64_t)s_raw[j] : 0;
      unsigned long long lo = ULLONG_MAX, hi = 0;
      uint32_t basic = 0;
      const uint64_t sv = score_node_b_k(s_rows + (j < cnt ? j : 0), act, emask, sc, sub, rbase, lo, hi, basic);
      if (act && sub == 0) {
        s_raw[j] = (int64_t)sv;
        s_basic[j] = basic;
      }
      lo = wave_min(lo);
      hi = wave_max(hi);
      if (lane == 0) {
        s_glh[gq][0] = lo;
        s_glh[gq][1] = hi;
      }
    }
  };

  // assume (engine.cpp Engine::reserve, non-compat, reservation pending) of pod `rq` on row j
  // with GPU set `mask`: one thread
  auto assume_row = [&](const yoda_dev_req_t& rq, int j, uint32_t mask) {
    yoda_dev_node_t* nd = s_rows + j;
    const uint32_t mb = (uint32_t)rq.memory;
    // branch-free: every card's two words are loaded together instead of a dependent LDS
    // round trip per taken card
#pragma unroll
    for (int c = 0; c < YODA_DEV_CARDS; ++c) {
      const uint32_t add = ((mask >> c) & 1u) ? mb : 0u;
      nd->cards[c].reserved += add;
      nd->cards[c].pending += add;
    }
    nd->pod_count += 1;
    nd->req_cpu += rq.cpu_m;
    nd->req_mem += rq.mem;
    nd->ext_used += rq.ext;
    nd->nz_cpu += rq.nz_cpu_m;
    nd->nz_mem += rq.nz_mem;
    s_dirty[j] = 1;
    if constexpr (COLS)
      for (int sl = 0; sl < a.n_sp; ++sl) s_cnt[sl * npb + j] += (int32_t)((rq.match_mask >> sl) & 1u);
  };

  bool ok = true;
  for (int b = set; b < a.B && ok; b += PAIRS ? 2 : 1) {
    // the request is read from LDS where it is used (uniform address: a broadcast read).
    // Copying all 49 words into scalar registers for the whole pod measured slower — the
    // copy spilled other scalars (167 vs 131 SGPR spills): 13.7 vs 13.2 µs/pod at 256 nodes,
    // 16.05 vs 15.9 at 4096 (profiles/device/r4/kernel_ab_r4/)
    const yoda_dev_req_t& r = *reinterpret_cast<const yoda_dev_req_t*>(s_req[b & 3]);
    const uint32_t tag1 = a.tag0 + 3u * (uint32_t)b, tag2 = tag1 + 1u, tag3 = tag1 + 2u;
    // prefetch request b+1 (PAIRS: and b+2, this set's next pod; b+1 is the other set's, whose
    // assume this set applies) — they land while this pod's phases run, stored after gather 1
    uint32_t pre = 0, pre2 = 0;
    if (tid < kReqWords) {
      if (b + 1 < a.B) pre = reinterpret_cast<const uint32_t*>(a.reqs + b + 1)[tid];
      if (PAIRS && b + 2 < a.B) pre2 = reinterpret_cast<const uint32_t*>(a.reqs + b + 2)[tid];
    }
    TRACE(0);

    // ================= phase F: filter → per-group aggregates → record 1. (Filtering pod
    // b+1 speculatively while pod b's record 3 travels, re-filtering only the winner's group,
    // measured slower on MI355X: 15.9 vs 15.1 µs/pod at 4096 nodes — the filter lands in the
    // gather wait instead of under it.)
    const int par = PAIRS ? ((b >> 1) & 1) : (b & 1);   // this set's consecutive pods alternate
    uint8_t* s_feas = s_feas2 + par * npb;
    uint8_t* s_elig = s_elig2 + par * npb;
    filter_groups(r, par);
    __syncthreads();
    ScoreConsts sc = score_consts(r, nullptr);
    int fix = -1;   // PAIRS: the other set's last winner's row, in its owner block only
    int fixg = -1;  // PAIRS: that owner block (every block of the set knows it), −1: none
    bool early1 = false;   // PAIRS owner: wave 0 already gathered record 1 (into s_rec)
    if constexpr (PAIRS) {
      // score A of every group now, against the rows as of this set's last pod; then the other
      // set's pod b−1: its winner, from its record 3 (best key; the GPU mask, whether the record's
      // block had a feasible node, whether the pod fit anywhere)
      score_a_groups(r, sc, s_feas, s_elig, 0, ngroups);
      if constexpr (SPEC) {   // phase B on the speculated maxima, before the other set's winner
        if (tid < 6) {
          const uint64_t key = spec_key(r);
          const int slot = spec_slot(key);
          s_cur[tid] = s_ptab[slot][0] == key ? s_ptab[slot][1 + tid] : s_spec[tid];
        }
        __syncthreads();   // (also: a multi-GPU pod's gang merge rewrote part A across waves)
        score_consts_maxima(sc, s_cur);
        phase_b_groups(sc, s_feas, s_elig, 0, ngroups, wave, BW);
        __syncthreads();
      }
      if (b >= 1) {
        if (tid == 0) {   // before the holder's write: same wave, or the gather's barrier
          s_fix = -1;
          s_fixg = -1;
        }
        // (each record kind has its own slot: the other set overwrites this record 3 only with
        // its pod b+1's, which needs pod b's winner from this set — and every block of this set
        // publishes its part of that after this read)
        // the one record that holds the winner: its key, from a block with a feasible node
        // (keys of feasible nodes are unique; a block without one reports key 0), and the pod
        // fit somewhere. Its thread applies the assume if this block holds the node.
        auto take_winner = [&](unsigned long long key, const uint32_t (&v)[3], unsigned long long t_g3, int prod) {
          const yoda_dev_req_t& rp = *reinterpret_cast<const yoda_dev_req_t*>(s_req[(b - 1) & 3]);
          s_fixg = prod;   // the record's producer holds the winner's node
          const uint32_t pp = (uint32_t)(key & 0xFFFFFFull);
          const int w = (int)(((pp - rp.perm_add) * rp.perm_inv) & 0xFFFFFFu);
          if (w >= base && w < base + cnt) {
            assume_row(rp, w - base, v[2] & 0xFFu);
            s_fix = w - base;
            if (a.trace) a.trace[(size_t)b * kTracePts + 13] = t_g3;
          }
        };
        auto holds = [&](bool have, unsigned long long mk, unsigned long long key, const uint32_t (&v)[3]) {
          return have && mk == key && ((v[2] >> 9) & 1u) && ((v[2] >> 8) & 1u);
        };
        // every block of this set counts pod b−1's winner in its spread domain tables (granule 2
        // of the holder's record: the winner's domains); one thread
        auto count_winner = [&](uint32_t g2) {
          const yoda_dev_req_t& rp = *reinterpret_cast<const yoda_dev_req_t*>(s_req[(b - 1) & 3]);
          for (int sl = 0; sl < a.n_sp; ++sl) {
            const uint32_t d = (g2 >> (16 + 8 * sl)) & 0xFFu;
            if (((rp.match_mask >> sl) & 1u) && d != YODA_DEV_DOM_NONE) s_zc[sl][d] += 1;
          }
        };
        if (G <= 128) {
          // wave 0 alone (lane t: producers t and t + 64) gathers, reduces and assumes
          if (wave == 0) {
            uint32_t v[3], v2[3];
            if (gather_wave0<3>(a, tag3 - 3u, G, q0, v, v2)) {
              const unsigned long long t_g3 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
              const bool have = tid < G, have2 = tid + 64 < G;
              const unsigned long long mk = have ? ((unsigned long long)v[1] << 32 | v[0]) : 0ull;
              const unsigned long long mk2 = have2 ? ((unsigned long long)v2[1] << 32 | v2[0]) : 0ull;
              const unsigned long long key = wave_max(mk > mk2 ? mk : mk2);
              const bool h1 = holds(have, mk, key, v), h2 = !h1 && holds(have2, mk2, key, v2);
              if (h1) take_winner(key, v, t_g3, lane);
              else if (h2) take_winner(key, v2, t_g3, lane + 64);
              if (COLS && a.n_sp > 0) {
                const unsigned long long bal = __ballot(h1 || h2);
                if (bal) {
                  const int src = __ffsll((long long)bal) - 1;
                  const uint32_t g2 = (uint32_t)__builtin_amdgcn_readlane((int)(h1 ? v[2] : v2[2]), src);
                  if (lane == 0) count_winner(g2);
                }
              }
            } else if (lane == 0) {
              s_fail = 1;
            }
          }
          __syncthreads();
          if (s_fail) {
            ok = false;
            break;
          }
        } else {
          uint32_t v[3];
          if (!gather<3>(a, tag3 - 3u, G, q0, v, &s_fail)) {
            ok = false;
            break;
          }
          const unsigned long long t_g3 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0ull;
          const bool have = tid < G;
          const unsigned long long mk = have ? ((unsigned long long)v[1] << 32 | v[0]) : 0ull;
          const unsigned long long wk = wave_max(mk);
          if (lane == 0) s_part[wave][0] = wk;
          __syncthreads();
          unsigned long long key = 0;
          for (int w = 0; w < BW; ++w) key = s_part[w][0] > key ? s_part[w][0] : key;
          if (holds(have, mk, key, v)) {
            take_winner(key, v, t_g3, tid);
            if (COLS && a.n_sp > 0) count_winner(v[2]);   // (every block has one thread reading the holder's record)
          }
          __syncthreads();
        }
        fix = s_fix;
        fixg = s_fixg;
      }
      if (fix >= 0) {
        // owner: wave 0 re-filters the winner's group and sends record 1 (its s_grp row is
        // written and read by wave 0 alone: LDS operations of one wave complete in order)
        // while the other waves score it
        const int fg = fix / kNodesPerWave;
        // one replica per 8 subsets of the pod's size, at most BW−1: a replica without subsets
        // would still redo the node's tables and default scores beside the searching waves
        const int nsub = sc.s_end - sc.s_begin;
        const int nrep = (sc.search && sc.k > 1) ? min(BW - 2, max(1, (nsub + kGroup - 1) / kGroup)) : 1;
        if (a.trace && tid == 0) a.trace[(size_t)b * kTracePts + 9] = __builtin_amdgcn_s_memrealtime();
        early1 = G <= 128;
        // the wave that gathers every other block's record 1 meanwhile: a spare one (beyond the
        // GPU-set replicas and the scores wave) from the start, else wave 0 after record 1.
        // Its own record goes into the transposed records from wave 0's registers.
        const int gw = nrep + 1 < BW - 1 ? BW - 1 : 0;
        auto gather_early = [&]() {
          uint32_t v[REC1], v2[REC1];
          if (gather_wave0<REC1>(a, tag1, G, p0, v, v2, gi)) {
            if (a.trace && lane == 0) a.trace[(size_t)b * kTracePts + 18] = __builtin_amdgcn_s_memrealtime();
            const int t2 = lane + 64;
            const bool h1 = lane < G && lane != gi, h2 = t2 < G && t2 != gi;
            if (h1) transpose1(v, lane);
            if (h2) transpose1(v2, t2);
            if constexpr (SPEC) {   // the other blocks' raw lo / hi under the speculated maxima
              const unsigned long long l1 = h1 ? ((unsigned long long)v[12] << 32 | v[11]) : ULLONG_MAX;
              const unsigned long long l2 = h2 ? ((unsigned long long)v2[12] << 32 | v2[11]) : ULLONG_MAX;
              const unsigned long long g1 = h1 ? ((unsigned long long)v[14] << 32 | v[13]) : 0ull;
              const unsigned long long g2 = h2 ? ((unsigned long long)v2[14] << 32 | v2[13]) : 0ull;
              const unsigned long long wl = wave_min(l1 < l2 ? l1 : l2), wh = wave_max(g1 > g2 ? g1 : g2);
              if (lane == 0) {
                s_red[0] = wl;
                s_red[1] = wh;
              }
            }
          } else if (lane == 0) {
            s_fail = 1;
          }
        };
        // this block's column of the transposed records (wave 0, after record 1)
        auto own_column = [&](uint32_t own) {
          if (early1 && tid < REC1) {
            if (COLS || tid < 7) {
              s_rec[tid][gi] = own;
            } else if (tid < 7 + kRsPairs) {
              const int q0 = 2 * (tid - 7);
              s_rec[7 + q0][gi] = own & 0xFFFFu;
              if (q0 + 1 < kNR) s_rec[8 + q0][gi] = own >> 16;
            }
          }
        };
        if (wave == 0) {
          filter_one(r, par, fg);
          __builtin_amdgcn_wave_barrier();
          own_column(record1(tag1, fg, early1));
          if (a.trace && tid == 0) a.trace[(size_t)b * kTracePts + 10] = __builtin_amdgcn_s_memrealtime();
          if constexpr (SPEC) {   // the maxima part of the group's phase B (speculated maxima in sc),
                                  // while the other waves score it: finished right after the barrier
            const int j = fg * kNodesPerWave + grp;
            const bool act = j < cnt && s_feas[j];
            unsigned long long lo_u = ULLONG_MAX, hi_u = 0;
            uint32_t basic = 0;
            (void)score_node_b_k(s_rows + (j < cnt ? j : 0), act, act ? s_elig[j] : 0u, sc, sub, 0, lo_u, hi_u, basic);
            if (act && sub == 0) s_basic[j] = basic;
          }
          if (early1 && gw == 0) gather_early();
        } else if (early1 && wave == gw) {
          gather_early();
        } else {
          score_a_fix(r, sc, fg, nrep, b);
        }
        __syncthreads();
        if (a.trace && tid == 0) a.trace[(size_t)b * kTracePts + 23] = __builtin_amdgcn_s_memrealtime();
        combine_fix(r, sc, s_feas, fg * kNodesPerWave, nrep);
        if constexpr (SPEC) {
          // the group's raw scores finished on the speculated maxima (the scores wave left the
          // maxima part in s_basic) and its lo / hi sent as the fix-up record, which every block of
          // the set folds into record 1's (combine_fix's lanes: same wave, in order)
          if (tid < kNodesPerWave) {   // one node each (a whole 8-lane group)
            const int j = fg * kNodesPerWave + tid;
            const bool act = j < cnt && s_feas[j];
            unsigned long long lo = ULLONG_MAX, hi = 0;
            if (act) {
              const uint64_t sv = sc.yoda_s ? (uint64_t)s_raw[j] + s_basic[j] : 0ull;
              s_raw[j] = (int64_t)sv;
              if (sc.yoda_s) lo = hi = sv > (uint64_t)LLONG_MAX ? 0ull : sv;
            }
            lo = group_reduce(lo, OpMin{});
            hi = group_reduce(hi, OpMax{});
            if (tid < 4) {
              const unsigned long long x = tid < 2 ? lo : hi;
              store_granule((gu64*)(a.slots + fix_slot_off(set) / 8u) + tid, tag1,
                            (tid & 1) ? (uint32_t)(x >> 32) : (uint32_t)x);
            }
          }
        }
        if (a.trace && tid == 0) a.trace[(size_t)b * kTracePts + 11] = __builtin_amdgcn_s_memrealtime();
      } else {
        record1(tag1);
      }
      TRACE(1);
      TRACE(2);
    } else {
      record1(tag1);
      TRACE(1);
      // ================= phase A (while record 1 travels)
      score_a_groups(r, sc, s_feas, s_elig, 0, ngroups);
      TRACE(2);
    }

    // ================= gather 1: global maxima, feasible and reason counts
    {
      if (!early1) {
        uint32_t v[REC1];
        if (!gather<REC1>(a, tag1, G, p0, v, &s_fail)) {
          ok = false;
          break;
        }
        if (PAIRS && fix >= 0 && a.trace && tid == 0) a.trace[(size_t)b * kTracePts + 19] = __builtin_amdgcn_s_memrealtime();
        // transpose through LDS (7 + kNR fields × G), then 16 threads per field reduce it
        if (tid < G) transpose1(v, tid);
        if constexpr (SPEC) {   // raw lo / hi under the speculated maxima: per wave, then s_red
          const bool have = tid < G;
          const unsigned long long l = have ? ((unsigned long long)v[12] << 32 | v[11]) : ULLONG_MAX;
          const unsigned long long h = have ? ((unsigned long long)v[14] << 32 | v[13]) : 0ull;
          const unsigned long long wl = wave_min(l), wh = wave_max(h);
          if (lane == 0) {
            s_part[wave][2] = wl;
            s_part[wave][3] = wh;
          }
        }
        __syncthreads();
        if (PAIRS && fix >= 0 && a.trace && tid == 0) a.trace[(size_t)b * kTracePts + 20] = __builtin_amdgcn_s_memrealtime();
      } else if (s_fail) {   // (PAIRS owner: wave 0 gathered before the fix-up barrier)
        ok = false;
        break;
      }
      const int seg = tid & 15;
      for (int f = tid >> 4; f < NF1; f += kBB >> 4) {   // 16 lanes per field; f is uniform per 16 lanes
        const bool is_max = f < 6, is_or = COLS && f >= kGDlo;
        // a lane's ≤ kMaxGrid / 16 records of the field in one LDS round trip (a loop carried
        // through acc waited out every load: ~1 µs per pass at G = 256), past G masked (every
        // field's identity is 0: the maxima start at 1)
        uint32_t x[kMaxGrid / 16];
#pragma unroll
        for (int i = 0; i < kMaxGrid / 16; ++i) x[i] = s_rec[f][seg + 16 * i];
        uint32_t acc = is_max ? 1u : 0u;
#pragma unroll
        for (int i = 0; i < kMaxGrid / 16; ++i) {
          const uint32_t y = seg + 16 * i < G ? x[i] : 0u;
          acc = is_max ? (y > acc ? y : acc) : is_or ? (acc | y) : acc + y;
        }
        // the 16 lanes of a field are one DPP row (f is row-uniform)
        if (is_max) {
          acc = group_reduce(acc, OpMax{});
          acc = OpMax{}(acc, dpp<kDppRowMirror>(acc));
        } else if (is_or) {
          acc = group_reduce(acc, OpOr{});
          acc |= dpp<kDppRowMirror>(acc);
        } else {
          acc = group_reduce(acc, OpSum{});
          acc += dpp<kDppRowMirror>(acc);
        }
        if (seg == 0) s_glob[f] = acc;
      }
      if (PAIRS && fix >= 0 && a.trace && tid == 0) a.trace[(size_t)b * kTracePts + 21] = __builtin_amdgcn_s_memrealtime();
      // (also orders a PAIRS owner's gang merge before phase B)
      __syncthreads();
    }
    if (PAIRS && fix >= 0 && a.trace && tid == 0) a.trace[(size_t)b * kTracePts + 12] = __builtin_amdgcn_s_memrealtime();
    // SPEC: the gathered maxima against the speculated ones (every block of the set compares the
    // same values: a block-set-uniform choice), and the raw lo / hi that hold if they match
    bool hit = false;
    unsigned long long slo1 = ULLONG_MAX, shi1 = 0;
    if constexpr (SPEC) {
      hit = true;
#pragma unroll
      for (int k = 0; k < 6; ++k) hit = hit && s_glob[k] == s_cur[k];
      if (a.trace && gi == 0 && tid == 0) a.trace[(size_t)b * kTracePts + 22] = hit ? 1ull : 2ull;
      if (early1) {
        slo1 = s_red[0] < s_red[2] ? s_red[0] : s_red[2];
        shi1 = s_red[1] > s_red[3] ? s_red[1] : s_red[3];
      } else {
        for (int w = 0; w < BW; ++w) {
          slo1 = s_part[w][2] < slo1 ? s_part[w][2] : slo1;
          shi1 = s_part[w][3] > shi1 ? s_part[w][3] : shi1;
        }
      }
      if (hit && fixg >= 0) {   // (set-uniform) the owner's re-scored group: one record, polled by one lane
        if (wave == 0) {
          const __amdgpu_buffer_rsrc_t rs = slot_rsrc(a);
          const uint32_t off = fix_slot_off(set);
          const long long t0 = __builtin_amdgcn_s_memrealtime();
          bool got = false;
          for (unsigned spins = 0;;) {
            __asm__ volatile("" ::: "memory");
            const u32x4 x = load_pair(rs, off, 0, lane == 0, tag1), y = load_pair(rs, off, 2, lane == 0, tag1);
            if (__all(x.y == tag1 && x.w == tag1 && y.y == tag1 && y.w == tag1)) {
              if (lane == 0) {
                s_fixlh[0] = (unsigned long long)x.z << 32 | x.x;
                s_fixlh[1] = (unsigned long long)y.z << 32 | y.x;
              }
              got = true;
              break;
            }
            if (!spin_ok(a, spins, t0)) break;
          }
          if (!got && lane == 0) s_fail = 1;
        }
        __syncthreads();
        if (s_fail) {
          ok = false;
          break;
        }
        slo1 = s_fixlh[0] < slo1 ? s_fixlh[0] : slo1;
        shi1 = s_fixlh[1] > shi1 ? s_fixlh[1] : shi1;
      }
    }
    int reasons7[kNR];
#pragma unroll
    for (int q = 0; q < kNR; ++q)
      reasons7[q] = COLS ? (int)((s_glob[7 + q / 2] >> (16 * (q & 1))) & 0xFFFFu) : (int)s_glob[7 + q];
    const int nf = COLS ? (int)(s_glob[6] & 0xFFFFu) : (int)s_glob[6];
    const uint64_t gmx[6] = {s_glob[0], s_glob[1], s_glob[2], s_glob[3], s_glob[4], s_glob[5]};
    score_consts_maxima(sc, gmx);
    // PodTopologySpread weights log(size + 2) (engine.cpp spread_scores): the hostname
    // constraint's size is the feasible non-ignored nodes, the domain constraint's the domains
    // among them; the logarithms come from the host's libm (a table), as the CPU engine's
    const int spl = r.spread_slot;
    // request b+1 (prefetched at the start of this pod) to LDS; the barriers of the
    // remaining phases order it before the next pod reads it
    if (tid < kReqWords) {
      if (b + 1 < a.B) s_req[(b + 1) & 3][tid] = pre;
      if (PAIRS && b + 2 < a.B) s_req[(b + 2) & 3][tid] = pre2;
    }
    TRACE(3);

    // ================= phase B: maxima-normalised card metrics → raw scores, lo/hi → record 2
    // (SPEC: only when the speculated maxima were wrong — part A is recovered as s_raw − s_basic)
    unsigned long long glo = ULLONG_MAX, ghi = 0;
    if (hit) {
      glo = slo1;
      ghi = shi1;
      TRACE(4);
    } else {
      unsigned long long lo = ULLONG_MAX, hi = 0, slo = ULLONG_MAX, shi = 0;
      double w0 = 0.0, w1 = 0.0;   // the constraints' weights (pod-uniform)
      if (COLS && spl >= 0) {
        const uint32_t ndom = (uint32_t)__popc((uint32_t)s_glob[kGDlo]) + (uint32_t)__popc((uint32_t)s_glob[kGDhi]);
        const uint32_t nfi = (uint32_t)(s_glob[6] >> 16);
        w0 = a.logtab[r.ckind[0] ? ndom : nfi];
        if (r.spread_nc > 1) w1 = a.logtab[r.ckind[1] ? ndom : nfi];
      }
      for (int j0 = wave * kNodesPerWave; j0 < cnt; j0 += BW * kNodesPerWave) {
        const int j = j0 + grp;
        const bool act = j < cnt && s_feas[j];
        const uint32_t emask = act ? s_elig[j] : 0u;
        const uint64_t rbase = (act && sub == 0) ? (uint64_t)s_raw[j] - (SPEC ? (uint64_t)s_basic[j] : 0ull) : 0;
        uint32_t basic = 0;
        const uint64_t raw_v = score_node_b_k(s_rows + (j < cnt ? j : 0), act, emask, sc, sub, rbase, lo, hi, basic);
        if (act && sub == 0) s_raw[j] = (int64_t)raw_v;   // (unclamped: Sel clamps)
        if (COLS && act && sub == 0 && spl >= 0) {
          // Σ over the constraints, in order, of count × weight + (maxSkew − 1) in float64 with
          // the CPU's rounding (no contraction), truncated; −1: the node lacks a key (ignored)
          const uint32_t d = s_dom[spl * npb + j];
          int32_t sp = -1;
          if (d != YODA_DEV_DOM_NONE) {
            double total = 0.0;
            for (int c = 0; c < (int)r.spread_nc; ++c) {
              const int32_t cv = r.ckind[c] ? s_zc[spl][d] : s_cnt[spl * npb + j];
              total = __dadd_rn(total, __dadd_rn(__dmul_rn((double)cv, c ? w1 : w0), (double)(r.cskew[c] - 1)));
            }
            sp = (int32_t)(int64_t)total;   // the host bounds the columns so that this fits
            const unsigned long long us = (unsigned long long)sp;
            slo = us < slo ? us : slo;
            shi = us > shi ? us : shi;
          }
          s_sp[j] = sp;
        }
      }
      lo = wave_min(lo);
      hi = wave_max(hi);
      if (COLS && spl >= 0) {
        slo = wave_min(slo);
        shi = wave_max(shi);
      }
      if (lane == 0) {
        s_part[wave][0] = lo;
        s_part[wave][1] = hi;
        s_part[wave][2] = slo;
        s_part[wave][3] = shi;
      }
      __syncthreads();
      if (tid < REC2) {
        unsigned long long blo = ULLONG_MAX, bhi = 0;
        const int q = tid < 4 ? 0 : 2;   // raw lo/hi, then spread lo/hi
        for (int w = 0; w < BW; ++w) {
          blo = s_part[w][q] < blo ? s_part[w][q] : blo;
          bhi = s_part[w][q + 1] > bhi ? s_part[w][q + 1] : bhi;
        }
        const unsigned long long x = (tid < 4 ? (tid & 3) < 2 : tid == 4) ? blo : bhi;
        // (spread lo / hi: one granule each, no spread node → lo 0xFFFFFFFF)
        const uint32_t g32 = tid < 4 ? ((tid & 1) ? (uint32_t)(x >> 32) : (uint32_t)x)
                                     : (uint32_t)(x < 0xFFFFFFFFull ? x : 0xFFFFFFFFull);
        store_granule(slot_ptr(a, tag2, g) + tid, tag2, g32);
      }
      TRACE(4);
      if (G <= 128) {
        // wave 0 alone gathers and reduces; one barrier hands lo/hi to the block
        if (wave == 0) {
          uint32_t v[REC2], v2[REC2];
          if (gather_wave0<REC2>(a, tag2, G, p0, v, v2)) {
            const bool have = tid < G, have2 = tid + 64 < G;
            {   // raw lo/hi
              const unsigned long long l1 = have ? ((unsigned long long)v[1] << 32 | v[0]) : ULLONG_MAX;
              const unsigned long long l2 = have2 ? ((unsigned long long)v2[1] << 32 | v2[0]) : ULLONG_MAX;
              const unsigned long long h1 = have ? ((unsigned long long)v[3] << 32 | v[2]) : 0ull;
              const unsigned long long h2 = have2 ? ((unsigned long long)v2[3] << 32 | v2[2]) : 0ull;
              const unsigned long long wlo = wave_min(l1 < l2 ? l1 : l2), whi = wave_max(h1 > h2 ? h1 : h2);
              if (lane == 0) {
                s_red[0] = wlo;
                s_red[1] = whi;
              }
            }
            if constexpr (COLS) {   // spread lo/hi (32-bit)
              const uint32_t l1 = have ? v[4] : 0xFFFFFFFFu, l2 = have2 ? v2[4] : 0xFFFFFFFFu;
              const uint32_t h1 = have ? v[5] : 0u, h2 = have2 ? v2[5] : 0u;
              const uint32_t wlo = wave_min(l1 < l2 ? l1 : l2), whi = wave_max(h1 > h2 ? h1 : h2);
              if (lane == 0) {
                s_red[2] = wlo == 0xFFFFFFFFu ? ULLONG_MAX : wlo;
                s_red[3] = whi;
              }
            }
          } else if (lane == 0) {
            s_fail = 1;
          }
        }
        __syncthreads();
        if (s_fail) {
          ok = false;
          break;
        }
        glo = s_red[0];
        ghi = s_red[1];
      } else {
        uint32_t v[REC2];
        if (!gather<REC2>(a, tag2, G, p0, v, &s_fail)) {
          ok = false;
          break;
        }
        // (the gather's barrier ordered every read of the record-2 partials before these writes)
        const bool have = tid < G;
        {
          const unsigned long long mlo = have ? ((unsigned long long)v[1] << 32 | v[0]) : ULLONG_MAX;
          const unsigned long long mhi = have ? ((unsigned long long)v[3] << 32 | v[2]) : 0ull;
          const unsigned long long wlo = wave_min(mlo), whi = wave_max(mhi);
          if (lane == 0) {
            s_part[wave][0] = wlo;
            s_part[wave][1] = whi;
          }
        }
        if constexpr (COLS) {   // spread lo/hi (32-bit)
          const uint32_t wlo = wave_min(have ? v[4] : 0xFFFFFFFFu), whi = wave_max(have ? v[5] : 0u);
          if (lane == 0) {
            s_part[wave][2] = wlo == 0xFFFFFFFFu ? ULLONG_MAX : wlo;
            s_part[wave][3] = whi;
          }
        }
        __syncthreads();
        for (int w = 0; w < BW; ++w) {
          glo = s_part[w][0] < glo ? s_part[w][0] : glo;
          ghi = s_part[w][1] > ghi ? s_part[w][1] : ghi;
        }
        if (COLS && tid == 0) {   // spread lo / hi: read from LDS where used (fewer live registers)
          unsigned long long sl = ULLONG_MAX, sh = 0;
          for (int w = 0; w < BW; ++w) {
            sl = s_part[w][2] < sl ? s_part[w][2] : sl;
            sh = s_part[w][3] > sh ? s_part[w][3] : sh;
          }
          s_red[2] = sl;
          s_red[3] = sh;
        }
        __syncthreads();
      }
    }
    TRACE(5);

    // ================= phase Sel: normalise + block argmax → record 3 → global best key
    unsigned long long key = 0;
    {
      const int64_t hi = (int64_t)ghi;
      int64_t lo = (int64_t)glo;
      if (hi == lo) --lo;
      const uint64_t den = (uint64_t)hi - (uint64_t)lo;
      const double rden = rcp64((double)den);
      unsigned long long best = 0;
      // PodTopologySpread NormalizeScore: ignored nodes 0; MaxNodeScore when the highest is 0;
      // else 100·(hi + lo − s) / hi (all terms ≥ 0)
      const int64_t shi = (int64_t)s_red[3], slo = (int64_t)s_red[2];
      const int img_sl = r.img_slot;
      for (int j = tid; j < cnt; j += kBB) {
        if (!s_feas[j]) continue;
        int64_t f = s_total[j];
        if (sc.yoda_s) {
          const uint64_t rs = (uint64_t)s_raw[j], rv = rs > (uint64_t)LLONG_MAX ? 0ull : rs;
          f += (int64_t)udiv_r((rv - (uint64_t)lo) * 100ull, den, rden) * r.w_yoda;
        }
        if (COLS && spl >= 0) {
          const int64_t sp = s_sp[j];
          const int64_t norm = sp < 0 ? 0 : shi == 0 ? 100 : (100 * (shi + slo - sp)) / shi;   // (sp: int32)
          f += norm * (int64_t)r.spread_w;
        }
        if (COLS && img_sl >= 0) f += s_img[img_sl * npb + j];
        const uint32_t p = ((uint32_t)(base + j) * r.perm_mul + r.perm_add) & 0xFFFFFFu;
        const unsigned long long k = ((unsigned long long)f << 24) | p;
        best = k > best ? k : best;
      }
      best = wave_max(best);
      if (lane == 0) s_part[wave][0] = best;
      __syncthreads();
      if (SPEC && tid < 7) {   // this set's next pods speculate on them
        const uint64_t key = spec_key(r);
        const int slot = spec_slot(key);
        if (tid < 6) {
          if (nf > 0) s_spec[tid] = gmx[tid];   // (no feasible node: the maxima stay at 1, no guide)
          s_ptab[slot][1 + tid] = gmx[tid];
        } else {
          s_ptab[slot][0] = key;
        }
      }
      if (tid < REC3) {
        unsigned long long bb = 0;
        for (int w = 0; w < BW; ++w) bb = s_part[w][0] > bb ? s_part[w][0] : bb;
        uint32_t x = tid == 0 ? (uint32_t)bb : (uint32_t)(bb >> 32);
        if (tid == 2) {   // the block best's GPU mask (PAIRS), whether the pod fits anywhere and here,
                          // and the node's domain in each spread slot (every block counts the winner)
          uint32_t m = 0, dd = 0xFFFF0000u;
          const bool here = s_bfeas > 0;   // (a best key of 0 is a feasible node's when here)
          if (here) {
            const uint32_t pb = (uint32_t)(bb & 0xFFFFFFull);
            const int nb = (int)(((pb - r.perm_add) * r.perm_inv) & 0xFFFFFFu);
            if (nb >= base && nb < base + cnt) {
              m = s_mask[nb - base];
              for (int sl = 0; sl < a.n_sp; ++sl)
                dd = (dd & ~(0xFFu << (16 + 8 * sl))) | ((uint32_t)s_dom[sl * npb + nb - base] << (16 + 8 * sl));
            }
          }
          x = m | ((nf > 0 ? 1u : 0u) << 8) | ((here ? 1u : 0u) << 9) | dd;
        }
        store_granule(slot_ptr(a, tag3, g) + tid, tag3, x);
      }
      TRACE(6);
      if (G <= 128) {
        if (wave == 0) {
          uint32_t v[REC3], v2[REC3];
          if (gather_wave0<REC3>(a, tag3, G, p0, v, v2)) {
            const unsigned long long k1 = tid < G ? ((unsigned long long)v[1] << 32 | v[0]) : 0ull;
            const unsigned long long k2 = tid + 64 < G ? ((unsigned long long)v2[1] << 32 | v2[0]) : 0ull;
            const unsigned long long wk = wave_max(k1 > k2 ? k1 : k2);
            if (lane == 0) s_red[0] = wk;
            if constexpr (COLS) {   // the winning record's granule 2 (its domains)
              const bool h1 = tid < G && k1 == wk && ((v[2] >> 9) & 1u);
              const bool h2 = tid + 64 < G && k2 == wk && ((v2[2] >> 9) & 1u);
              const unsigned long long bal = __ballot(h1 || h2);
              if (bal) {
                const int src = __ffsll((long long)bal) - 1;
                const uint32_t g2 = (uint32_t)__builtin_amdgcn_readlane((int)(h1 ? v[2] : v2[2]), src);
                if (lane == 0) s_wdom = g2;
              }
            }
          } else if (lane == 0) {
            s_fail = 1;
          }
        }
        __syncthreads();
        if (s_fail) {
          ok = false;
          break;
        }
        key = s_red[0];
      } else {
        uint32_t v[REC3];
        if (!gather<REC3>(a, tag3, G, p0, v, &s_fail)) {
          ok = false;
          break;
        }
        const unsigned long long mk = tid < G ? ((unsigned long long)v[1] << 32 | v[0]) : 0ull;
        const unsigned long long wk = wave_max(mk);
        if (lane == 0) s_part[wave][0] = wk;
        __syncthreads();
        for (int w = 0; w < BW; ++w) key = s_part[w][0] > key ? s_part[w][0] : key;
        if constexpr (COLS) {
          if (tid < G && mk == key && ((v[2] >> 9) & 1u)) s_wdom = v[2];
          __syncthreads();
        }
      }
    }
    TRACE(7);

    // ================= winner: its owner publishes the result and assumes the pod
    int node = -1;
    if (nf > 0) {
      const uint32_t p = (uint32_t)(key & 0xFFFFFFull);
      node = (int)(((p - r.perm_add) * r.perm_inv) & 0xFFFFFFu);
    }
    // every block counts the winner in its domain tables (the owner its node count: assume_row)
    if (COLS && nf > 0 && tid == 0)
      for (int sl = 0; sl < a.n_sp; ++sl) {
        const uint32_t d = (s_wdom >> (16 + 8 * sl)) & 0xFFu;
        if (((r.match_mask >> sl) & 1u) && d != YODA_DEV_DOM_NONE) s_zc[sl][d] += 1;
      }
    const bool owner = nf > 0 ? (node >= base && node < base + cnt) : gi == 0;
    if (owner) {
      const int j = nf > 0 ? node - base : 0;
      const uint32_t mask = nf > 0 ? (uint32_t)s_mask[j] : 0u;
      const int32_t quality = nf > 0 ? s_quality[j] : 0;
      if (tid == 0 && nf > 0) assume_row(r, j, mask);
      // the result: lane k of wave 0 writes its 64-bit word k, every value selected with
      // constant indices (a local struct with the reasons array indexed by reason code lived in
      // scratch memory: ~30 scratch accesses and vmcnt waits on the owner's path each pod)
      if (tid < kResWords) {
        uint64_t w = 0;
        if (tid == 0) w = (uint64_t)(uint32_t)node | ((uint64_t)(uint32_t)nf << 32);
        if (tid == 1) w = (uint64_t)(nf > 1 ? (int64_t)(key >> 24) : 0);   // a lone feasible node scores 0
        if (tid == 2) w = (uint64_t)mask | ((uint64_t)(uint32_t)quality << 32);
#pragma unroll
        for (int q = 0; q < kNR; ++q) {   // reasons[code] as u32 pairs in words 3..10
          const int code = kBatchReasonCodes[q];
          if (tid == 3 + code / 2) w |= (uint64_t)(uint32_t)reasons7[q] << (32 * (code & 1));
        }
#pragma unroll
        for (int k = 0; k < 6; ++k)
          if (tid == 11 + k) w = gmx[k];
        if (tid == 17) w = glo;
        if (tid == 18) w = ghi;
        reinterpret_cast<unsigned long long*>(a.res + b)[tid] = w;
      }
    }
    __syncthreads();
    TRACE(8);
  }

  // ---- epilogue: dirty rows back to the table; the last block hands the results to the host.
  // PAIRS: only the set that ran the batch's last pod holds every assume (the other set never
  // learns that pod's winner), so only its replica is written back
  if (!PAIRS || set == ((a.B - 1) & 1))
  for (int t = tid; t < cnt * 32; t += kBB) {
    const int row = t >> 5;
    if (s_dirty[row]) reinterpret_cast<uint4*>(a.nodes + base + row)[t & 31] = reinterpret_cast<const uint4*>(s_rows + row)[t & 31];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = t == gridDim.x - 1;
    if (s_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!s_last) return;
  const bool aborted = __hip_atomic_load(a.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  if (!aborted) {
    const int words = a.B * (int)(sizeof(yoda_dev_result_t) / 8);
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(a.res);
    unsigned long long* dst = reinterpret_cast<unsigned long long*>(a.out);
    for (int w = tid; w < words; w += kBB) dst[w] = src[w];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(a.done, aborted ? -a.seq : a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

struct Ctx {
  int device = 0, cap = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  // bulk row uploads: host rows in mapped pinned memory that k_scatter reads directly (no
  // DMA copy, no completion signal for the runtime's threads to service); `h_upflag` is
  // raised by k_upload_done after the scatter, and the host waits on it only before it
  // rewrites the staging buffers
  yoda_dev_node_t *d_nodes = nullptr, *d_stage = nullptr, *h_stage = nullptr;
  int32_t *d_idx = nullptr, *h_idx = nullptr;
  int32_t *h_upflag = nullptr, *d_upflag = nullptr;
  int32_t up_seq = 0;
  uint8_t *d_feas = nullptr, *d_elig = nullptr, *d_cand = nullptr, *h_cand = nullptr;
  int64_t *d_raw = nullptr, *d_total = nullptr;
  uint32_t* d_mask = nullptr;
  int32_t* d_quality = nullptr;
  yoda_dev_result_t *h_res = nullptr, *d_res_map = nullptr;
  yoda_dev_result_t *h_resb = nullptr, *d_resb = nullptr;   // batched cycles: one slot per pod
  Globals* d_g = nullptr;
  float last_us = 0;
  int grid = 1024;
  bool timing = false;        // event timing of each cycle (benchmarks); off in the scheduler
  int direct_atomics = -1;    // -1: by grid size; 0/1 forced (YODA_DEV_DIRECT_ATOMICS)
  int fuse_max = kFuseSelectMax;   // YODA_DEV_FUSE_MAX overrides (A/B of the fused select)
  PatchArgs pend{};           // dirty rows waiting to ride in the next filter launch
  // persistent batch kernel (k_batch)
  bool persist = true;        // YODA_DEV_PERSIST=0: batches run as per-pod launch chains
  int cus = 256;
  int cus_total = 256;        // compute units of the device (occupancy check)
  int npb_min = 0;            // YODA_DEV_NPB: minimum nodes per block (0: 8 per wave)
  int batch_waves = 0;        // YODA_DEV_BWAVES: k_batch waves per block (4 or 8; 0 = by cluster size)
  // two pods in flight (k_batch PAIRS: two block sets alternate pods, each filtering and
  // scoring its next pod during the other's exchanges) when twice the grid is resident
  // (≤ 4096 nodes on MI355X). MI355X, bench mix: 13.5 vs 15.6–16.2 µs/pod at 4096 nodes, 11.9
  // vs 12.8–13.5 at 256 (profiles/device/r4/pairs/). YODA_DEV_PAIRS=0 turns it off
  bool pairs = true;
  int occ_blocks_pairs = -1;
  // per spin wait inside k_batch, 100 MHz ticks (YODA_DEV_SPIN_DEADLINE_US): a gather normally
  // completes in microseconds; 20 ms only elapses when a block is not resident (a tenant
  // kernel holds the CUs) — then every block gives up and the batch aborts
  long long deadline_ticks = 2000000ll;
  // host-side bound on one device call: base + per pod (YODA_DEV_HOST_DEADLINE_US = base).
  // Past it the host abandons the call (the engine places the pods on the CPU) and the
  // context refuses work until its stream drains (busy_check)
  double host_deadline_us = 20000.0, host_deadline_per_pod_us = 50.0;
  bool abandoned = false;
  std::chrono::steady_clock::time_point next_probe{};   // busy_check: next stream query
  // counters (yoda_dev_counters): every kernel dispatch, k_batch dispatches and the pods they
  // placed, abandoned calls, calls refused while draining, k_batch GPU time (timing on)
  long long n_dispatch = 0, n_kbatch = 0, n_kbatch_pods = 0, n_abandon = 0, n_busy = 0;
  double kbatch_us = 0;
  long long n_query = 0;   // stream queries made by busy_check, and their time
  double query_us = 0;
  double abandon_wait_us = 0;   // how long the host waited on the last call it abandoned
  double wait_us_per_pod = 0;   // k_batch wall µs per pod, smoothed (the host's pre-sleep)
  long long n_presleep = 0;
  int occ_waves = 0, occ_lds = -1, occ_blocks = 0;   // cached k_batch occupancy query
  bool occ_cols = false;
  bool force_cols = false;   // YODA_DEV_FORCE_COLS=1: batches without columns on the COLS kernel (A/B)
  yoda_dev_req_t *h_reqs = nullptr, *d_reqs_map = nullptr;
  yoda_dev_result_t* d_bres = nullptr;
  unsigned long long* d_slots = nullptr;
  unsigned int* d_words = nullptr;     // [0] ticket, [1] abort
  int32_t *h_done = nullptr, *d_done_map = nullptr;
  uint32_t epoch = 1;
  int seq = 0;
  int last_grid = 0, last_npb = 0;
  bool last_pairs = false;
  unsigned long long* d_trace = nullptr;   // yoda_dev_batch_trace: block 0's phase stamps
  int trace_pods = 0;
  // score columns staged by yoda_dev_batch_extras for the next batch (mapped pinned memory the
  // kernel reads in its prologue) and the log table of PodTopologySpread's weights
  int32_t *h_sp_cnt = nullptr, *d_sp_cnt = nullptr, *h_sp_zc = nullptr, *d_sp_zc = nullptr;
  uint8_t *h_sp_dom = nullptr, *d_sp_dom = nullptr;
  int32_t *h_img = nullptr, *d_img = nullptr;
  double* d_logtab = nullptr;
  int x_n = 0, x_sp = 0, x_img = 0;   // staged columns (consumed by the next batch)
  int lds_static = 0;                 // k_batch's static LDS (the dynamic part gets the rest)
};

#define CK(x)                               \
  do {                                      \
    hipError_t e__ = (x);                   \
    if (e__ != hipSuccess) return (int)e__; \
  } while (0)

// A call the host abandoned at its deadline may still be queued or running on the stream:
// until it drains, the context takes no new work (-9: the engine stays on the CPU path and
// keeps its rows dirty). Once drained, the batch words are re-armed.
int busy_check(Ctx* c) {
  if (!c->abandoned) return 0;
  // a stream query costs far more than a refusal while the GPU is held (≈ 0.3 ms measured
  // under a tenant kernel): probe at most every 2 ms, refuse in between
  const auto now = std::chrono::steady_clock::now();
  if (now < c->next_probe) {
    ++c->n_busy;
    return -9;
  }
  const hipError_t q = hipStreamQuery(c->stream);
  const auto after = std::chrono::steady_clock::now();
  ++c->n_query;
  c->query_us += std::chrono::duration<double, std::micro>(after - now).count();
  c->next_probe = after + std::chrono::milliseconds(2);
  if (q == hipErrorNotReady) {
    ++c->n_busy;
    return -9;
  }
  c->abandoned = false;
  CK(hipMemsetAsync(c->d_words, 0, 64, c->stream));
  CK(hipStreamSynchronize(c->stream));
  return 0;
}

double host_deadline_s(const Ctx* c, int pods) {
  return (c->host_deadline_us + c->host_deadline_per_pod_us * (pods > 0 ? pods : 1)) * 1e-6;
}

// launch the pending rows on their own (before a bulk scatter or a debug read)
int flush_pending(Ctx* c) {
  if (c->pend.n == 0) return 0;
  hipLaunchKernelGGL(k_patch, dim3(1), dim3(32 * kPatchRows), 0, c->stream, c->pend, c->d_nodes);
  ++c->n_dispatch;
  c->pend.n = 0;
  CK(hipGetLastError());
  return 0;
}

// The last bulk upload's scatter has finished reading the staging buffers (its flag is up):
// usually long ago; otherwise spin, asking the stream now and then (a failed launch).
int wait_upload(Ctx* c) {
  if (c->up_seq == 0) return 0;
  volatile int32_t* flag = c->h_upflag;
  for (unsigned spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == c->up_seq) return 0;
    if ((spin & 1023) == 0) {
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) == c->up_seq ? 0 : -4;
      if (q != hipErrorNotReady) return (int)q;
    }
    __builtin_ia32_pause();
  }
}

// Wait for the device to publish the result: spin on the mapped `feasible` field (written
// last, system-scope release), polling the stream now and then so a failed launch or a
// result that never comes cannot hang the scheduler.
int wait_result(Ctx* c) {
  volatile int32_t* flag = &c->h_res->feasible;
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = host_deadline_s(c, 1);
  for (unsigned spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) >= 0) return 0;
    if ((spin & 1023) == 0) {
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) >= 0 ? 0 : -4;
      if (q != hipErrorNotReady) return (int)q;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
        c->abandoned = true;   // the GPU is held by other work: the engine uses the CPU meanwhile
        c->abandon_wait_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        ++c->n_abandon;
        return -8;
      }
    }
    __builtin_ia32_pause();
  }
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
  c->cus = cus < kMaxGrid ? cus : kMaxGrid;
  c->cus_total = cus;
  if (const char* v = getenv("YODA_DEV_PERSIST")) c->persist = v[0] != '0';
  if (const char* v = getenv("YODA_DEV_NPB")) c->npb_min = atoi(v) > 0 ? atoi(v) : 0;
  if (const char* v = getenv("YODA_DEV_SPIN_DEADLINE_US")) c->deadline_ticks = atoll(v) > 0 ? atoll(v) * 100 : 1;
  if (const char* v = getenv("YODA_DEV_HOST_DEADLINE_US")) c->host_deadline_us = atof(v) > 0 ? atof(v) : 1.0;
  if (const char* v = getenv("YODA_DEV_BWAVES")) c->batch_waves = atoi(v) == 4 ? 4 : atoi(v) == 8 ? 8 : 0;
  if (const char* v = getenv("YODA_DEV_PAIRS")) c->pairs = v[0] != '0';
  if (const char* v = getenv("YODA_DEV_FORCE_COLS")) c->force_cols = v[0] == '1';
  if (const char* v = getenv("YODA_DEV_DIRECT_ATOMICS")) c->direct_atomics = v[0] == '1' ? 1 : 0;
  if (const char* v = getenv("YODA_DEV_FUSE_MAX")) c->fuse_max = atoi(v);
  const SubsetTable st = make_subsets();
  if ((e = hipMemcpyToSymbol(HIP_SYMBOL(c_subsets), &st, sizeof st)) != hipSuccess) return fail("subsets", e);
  if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) return fail("stream", e);
  if ((e = hipEventCreate(&c->e0)) != hipSuccess) return fail("event", e);
  if ((e = hipEventCreate(&c->e1)) != hipSuccess) return fail("event", e);
  const size_t N = (size_t)capacity;
  if ((e = hipMalloc(&c->d_nodes, N * sizeof(yoda_dev_node_t))) != hipSuccess) return fail("nodes", e);
  if ((e = hipMemset(c->d_nodes, 0, N * sizeof(yoda_dev_node_t))) != hipSuccess) return fail("memset", e);
  if ((e = hipHostMalloc(&c->h_stage, N * sizeof(yoda_dev_node_t), hipHostMallocMapped)) != hipSuccess)
    return fail("pinned stage", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_stage, c->h_stage, 0)) != hipSuccess) return fail("stage map", e);
  if ((e = hipHostMalloc(&c->h_idx, N * sizeof(int32_t), hipHostMallocMapped)) != hipSuccess) return fail("idx", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_idx, c->h_idx, 0)) != hipSuccess) return fail("idx map", e);
  if ((e = hipHostMalloc(&c->h_upflag, 64, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return fail("upload flag", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_upflag, c->h_upflag, 0)) != hipSuccess) return fail("upload flag map", e);
  *c->h_upflag = 0;
  if ((e = hipMalloc(&c->d_feas, N)) != hipSuccess) return fail("feas", e);
  if ((e = hipMalloc(&c->d_elig, N)) != hipSuccess) return fail("elig", e);
  if ((e = hipMalloc(&c->d_cand, N)) != hipSuccess) return fail("cand", e);
  if ((e = hipHostMalloc(&c->h_cand, N, hipHostMallocDefault)) != hipSuccess) return fail("cand", e);
  if ((e = hipMalloc(&c->d_raw, N * sizeof(int64_t))) != hipSuccess) return fail("raw", e);
  if ((e = hipMalloc(&c->d_total, N * sizeof(int64_t))) != hipSuccess) return fail("total", e);
  if ((e = hipMalloc(&c->d_mask, N * sizeof(uint32_t))) != hipSuccess) return fail("mask", e);
  if ((e = hipMalloc(&c->d_quality, N * sizeof(int32_t))) != hipSuccess) return fail("quality", e);
  // result: mapped, coherent pinned host memory written by the select kernel's last block
  if ((e = hipHostMalloc(&c->h_res, sizeof(yoda_dev_result_t), hipHostMallocMapped | hipHostMallocCoherent)) !=
      hipSuccess)
    return fail("result", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_res_map, c->h_res, 0)) != hipSuccess) return fail("result map", e);
  if ((e = hipHostMalloc(&c->h_resb, kBatchCap * sizeof(yoda_dev_result_t),
                         hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return fail("batch results", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_resb, c->h_resb, 0)) != hipSuccess) return fail("batch map", e);
  if ((e = hipMalloc(&c->d_g, sizeof(Globals))) != hipSuccess) return fail("globals", e);
  // persistent batch kernel state
  if ((e = hipHostMalloc(&c->h_reqs, kBatchCap * sizeof(yoda_dev_req_t), hipHostMallocMapped | hipHostMallocCoherent)) !=
      hipSuccess)
    return fail("batch requests", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_reqs_map, c->h_reqs, 0)) != hipSuccess) return fail("requests map", e);
  if ((e = hipHostMalloc(&c->h_done, 64, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return fail("batch done", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_done_map, c->h_done, 0)) != hipSuccess) return fail("done map", e);
  if ((e = hipMalloc(&c->d_bres, kBatchCap * sizeof(yoda_dev_result_t))) != hipSuccess) return fail("batch scratch", e);
  const size_t slot_bytes = kSlotBytes;
  if ((e = hipMalloc(&c->d_slots, slot_bytes)) != hipSuccess) return fail("slots", e);
  if ((e = hipMemset(c->d_slots, 0, slot_bytes)) != hipSuccess) return fail("slots", e);
  if ((e = hipMalloc(&c->d_words, 64)) != hipSuccess) return fail("words", e);
  if ((e = hipMemset(c->d_words, 0, 64)) != hipSuccess) return fail("words", e);
  // score columns (2 slots each) and log(i + 2) for i ≤ capacity from the host's libm (the CPU
  // engine's std::log), so device and CPU weights are the same doubles
  if ((e = hipHostMalloc(&c->h_sp_cnt, kSP * N * sizeof(int32_t), hipHostMallocMapped)) != hipSuccess)
    return fail("spread counts", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_sp_cnt, c->h_sp_cnt, 0)) != hipSuccess) return fail("spread map", e);
  if ((e = hipHostMalloc(&c->h_sp_dom, kSP * N, hipHostMallocMapped)) != hipSuccess) return fail("spread domains", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_sp_dom, c->h_sp_dom, 0)) != hipSuccess) return fail("spread map", e);
  if ((e = hipHostMalloc(&c->h_sp_zc, kSP * kDOM * sizeof(int32_t), hipHostMallocMapped)) != hipSuccess)
    return fail("spread zones", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_sp_zc, c->h_sp_zc, 0)) != hipSuccess) return fail("spread map", e);
  if ((e = hipHostMalloc(&c->h_img, kIMG * N * sizeof(int32_t), hipHostMallocMapped)) != hipSuccess)
    return fail("image scores", e);
  if ((e = hipHostGetDevicePointer((void**)&c->d_img, c->h_img, 0)) != hipSuccess) return fail("image map", e);
  {
    double* lt = new double[N + 3];
    for (size_t i = 0; i < N + 3; ++i) lt[i] = std::log((double)(i + 2));
    e = hipMalloc(&c->d_logtab, (N + 3) * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(c->d_logtab, lt, (N + 3) * sizeof(double), hipMemcpyHostToDevice);
    delete[] lt;
    if (e != hipSuccess) return fail("log table", e);
  }
  // every byte of LDS the static part leaves goes to the dynamic part (rows + columns)
  int lds_max = 65536;
  hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, device);
  static const void* const kBatchKernels[] = {
      (const void*)k_batch<4, false, false>, (const void*)k_batch<8, false, false>, (const void*)k_batch<4, true, false>,
      (const void*)k_batch<8, true, false>,  (const void*)k_batch<4, false, true>,  (const void*)k_batch<8, false, true>,
      (const void*)k_batch<4, true, true>,   (const void*)k_batch<8, true, true>};
  for (const void* kf : kBatchKernels) {
    hipFuncAttributes fa{};
    if ((e = hipFuncGetAttributes(&fa, kf)) != hipSuccess) return fail("k_batch attributes", e);
    c->lds_static = (int)fa.sharedSizeBytes > c->lds_static ? (int)fa.sharedSizeBytes : c->lds_static;
  }
  const int dyn_max = lds_max - c->lds_static;
  if (dyn_max < (int)(kMaxNodesPerBlock * kBatchRowBytes)) {
    snprintf(err, err_len, "k_batch LDS: %d B static + %zu B rows > %d B", c->lds_static,
             kMaxNodesPerBlock * kBatchRowBytes, lds_max);
    delete c;
    return nullptr;
  }
  for (const void* kf : kBatchKernels)
    if ((e = hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, dyn_max)) != hipSuccess)
      return fail("k_batch LDS", e);
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
  hipFree(c->d_nodes); hipHostFree(c->h_stage); hipHostFree(c->h_idx); hipHostFree(c->h_upflag);
  hipFree(c->d_feas); hipFree(c->d_elig); hipFree(c->d_cand); hipHostFree(c->h_cand); hipFree(c->d_raw);
  hipFree(c->d_total); hipFree(c->d_mask); hipFree(c->d_quality); hipHostFree(c->h_res); hipHostFree(c->h_resb); hipFree(c->d_g);
  hipHostFree(c->h_reqs); hipHostFree(c->h_done); hipFree(c->d_bres); hipFree(c->d_slots); hipFree(c->d_words);
  hipHostFree(c->h_sp_cnt); hipHostFree(c->h_sp_dom); hipHostFree(c->h_sp_zc); hipHostFree(c->h_img); hipFree(c->d_logtab);
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
  if (const int b = busy_check(c)) return b;
  if (n <= kPatchRows) {
    // steady state (a reservation dirtied one node): the rows wait host-side and travel in
    // the next filter launch's arguments; a newer row for the same node replaces the old
    PatchArgs& a = c->pend;
    int fresh = 0;
    for (int i = 0; i < n; ++i) {
      bool seen = false;
      for (int j = 0; j < a.n; ++j) seen |= a.idx[j] == idx[i];
      fresh += !seen;
    }
    if (a.n + fresh > kPatchRows && flush_pending(c) != 0) return -6;
    for (int i = 0; i < n; ++i) {
      int j = 0;
      while (j < a.n && a.idx[j] != idx[i]) ++j;
      if (j == a.n) ++a.n;
      a.idx[j] = idx[i];
      a.rows[j] = rows[i];
    }
    return 0;
  }
  if (flush_pending(c) != 0) return -6;   // older rows first: the bulk upload may overwrite them
  // the previous upload's scatter must have read the staging buffers before they are rewritten
  if (const int w = wait_upload(c)) return w;
  memcpy(c->h_stage, rows, (size_t)n * sizeof(yoda_dev_node_t));
  memcpy(c->h_idx, idx, (size_t)n * sizeof(int32_t));
  std::atomic_thread_fence(std::memory_order_release);
  const int per_block = 8;   // 8 records × 32 lanes = 256 threads
  hipLaunchKernelGGL(k_scatter, dim3((n + per_block - 1) / per_block), dim3(256), 0, c->stream, c->d_stage, c->d_idx,
                     n, c->d_nodes);
  c->up_seq = c->up_seq >= (1 << 30) ? 1 : c->up_seq + 1;
  hipLaunchKernelGGL(k_upload_done, dim3(1), dim3(64), 0, c->stream, c->d_upflag, c->up_seq);
  c->n_dispatch += 2;
  CK(hipGetLastError());
  return 0;
}

}  // extern "C"

namespace {

// Enqueue one scheduling cycle (filter → score [→ select]) writing its result to `out`
// (device view of mapped host memory). `extra_flags` is OR'ed into dev_flags.
int launch_cycle(Ctx* c, int n, yoda_dev_req_t r, yoda_dev_result_t* out, uint32_t extra_flags) {
  const int per_block = kWaves * kNodesPerWave;
  int grid = (n + per_block - 1) / per_block;
  grid = grid < c->grid ? grid : c->grid;
  int grid_sel = (n + kBlock - 1) / kBlock;
  grid_sel = grid_sel < c->grid ? grid_sel : c->grid;
  r.dev_flags = ((c->direct_atomics < 0 ? grid <= 256 : c->direct_atomics == 1) ? 1u : 0u) | extra_flags;
  const int fuse = n <= c->fuse_max;
  hipLaunchKernelGGL(k_filter, dim3(grid + (c->pend.n > 0 ? 1 : 0)), dim3(kBlock), 0, c->stream, c->pend, c->d_nodes,
                     n, r, c->d_cand, c->d_feas, c->d_elig, c->d_g);
  ++c->n_dispatch;
  c->pend.n = 0;
  hipLaunchKernelGGL(k_score, dim3(grid), dim3(kBlock), 0, c->stream, c->d_nodes, n, r, c->d_feas, c->d_elig,
                     c->d_raw, c->d_total, c->d_mask, c->d_quality, c->d_g, out, fuse);
  ++c->n_dispatch;
  if (!fuse) {
    hipLaunchKernelGGL(k_select, dim3(grid_sel), dim3(kBlock), 0, c->stream, n, r, c->d_feas, c->d_raw, c->d_total,
                       c->d_mask, c->d_quality, c->d_g, out, c->d_nodes);
    ++c->n_dispatch;
  }
  CK(hipGetLastError());
  return 0;
}

// Spin until `slot->feasible` is published (see wait_result).
int wait_slot(Ctx* c, yoda_dev_result_t* slot, int pods) {
  volatile int32_t* flag = &slot->feasible;
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = host_deadline_s(c, pods);
  for (unsigned spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) >= 0) return 0;
    if ((spin & 1023) == 0) {
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) >= 0 ? 0 : -4;
      if (q != hipErrorNotReady) return (int)q;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
        c->abandoned = true;
        c->abandon_wait_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        ++c->n_abandon;
        return -8;
      }
    }
    __builtin_ia32_pause();
  }
}

}  // namespace

extern "C" {

int yoda_dev_schedule(void* p, int n, const yoda_dev_req_t* req, const uint8_t* cand, yoda_dev_result_t* out) {
  Ctx* c = (Ctx*)p;
  if (n <= 0 || n > c->cap) return -1;
  if (req->use_candidates && !cand) return -3;
  CK(hipSetDevice(c->device));
  if (const int b = busy_check(c)) return b;
  if (req->use_candidates) {
    memcpy(c->h_cand, cand, (size_t)n);
    CK(hipMemcpyAsync(c->d_cand, c->h_cand, (size_t)n, hipMemcpyHostToDevice, c->stream));
  }
  __atomic_store_n(&c->h_res->feasible, -1, __ATOMIC_RELEASE);   // sentinel: overwritten by the device
  if (c->timing) CK(hipEventRecord(c->e0, c->stream));
  const int rc = launch_cycle(c, n, *req, c->d_res_map, 0u);
  if (rc != 0) return rc;
  if (c->timing) {
    CK(hipEventRecord(c->e1, c->stream));
    CK(hipEventSynchronize(c->e1));
    float ms = 0;
    if (hipEventElapsedTime(&ms, c->e0, c->e1) == hipSuccess) c->last_us = ms * 1000.0f;
  }
  const int w = wait_result(c);
  if (w != 0) return w;
  memcpy(out, c->h_res, sizeof(*out));
  return 0;
}

// Persistent path: one k_batch dispatch per chunk of ≤ kBatchCap pods. Returns 1 when the
// cluster does not fit the LDS-resident layout (the caller then uses the launch chain).
static int batch_persistent(Ctx* c, int n, int B, const yoda_dev_req_t* reqs, yoda_dev_result_t* out) {
  // staged score columns belong to this call's nodes and first chunk only (in-batch counts are
  // the kernel's own; a second chunk would restart from the staged ones)
  const bool cols = c->x_sp > 0 || c->x_img > 0 || (c->force_cols && n <= 65535);
  // (a COLS batch sums record-1 counts as u16 halves: below 65536 nodes)
  if ((c->x_sp > 0 || c->x_img > 0) && (c->x_n != n || B > kBatchCap || n > 65535)) return -3;
  int npb = (n + c->cus - 1) / c->cus;
  // 4 waves while one pass of 8 nodes per wave covers a block's share (a wave per SIMD is
  // fastest then); beyond, 8 waves: two per SIMD hide each other's latency and halve the
  // passes (MI355X, 4096 nodes: 15.7 vs 17.7 µs/pod; 16 384: 25.8 vs 23.0; 65 536: 59 vs 43)
  const int waves = c->batch_waves ? c->batch_waves : (npb > 4 * kNodesPerWave ? 8 : 4);
  // up to 1024 nodes one 8-node group per block (≤ 128 blocks): the block's other waves split
  // a multi-GPU pod's subset search, and the exchanges stay cheap at that grid (MI355X,
  // BASELINE mix: 256 nodes 13.4 vs 14.7 µs/pod, 1024 nodes 14.3 vs 14.8; at 2048 nodes 256
  // blocks lose, profiles/device/r3/geometry/)
  const int npb_min = c->npb_min > 0 ? c->npb_min : (n <= 1024 ? kNodesPerWave : waves * kNodesPerWave);
  npb = npb < npb_min ? npb_min : npb;
  if (npb > kMaxNodesPerBlock) return cols ? -3 : 1;
  const int G = (n + npb - 1) / npb;
  if (G > kMaxGrid) return cols ? -3 : 1;
  const size_t lds = (size_t)npb * (kBatchRowBytes + batch_col_bytes(c->x_sp, c->x_img));
  // every block spins on the others' records: all G must be resident at once. The device's
  // capacity for this geometry (blocks per CU × CUs) must cover G, or the batch takes the
  // launch chain (no cross-block waits). A tenant kernel holding CUs at run time is the
  // host deadline's job (abandon + CPU path), not this check's.
  if (c->occ_waves != waves || c->occ_lds != (int)lds || c->occ_cols != cols) {
    int nb = 0, np = 0;
    const void* k1 = cols ? (waves == 8 ? (const void*)k_batch<8, false, true> : (const void*)k_batch<4, false, true>)
                          : (waves == 8 ? (const void*)k_batch<8, false, false> : (const void*)k_batch<4, false, false>);
    const void* k2 = cols ? (waves == 8 ? (const void*)k_batch<8, true, true> : (const void*)k_batch<4, true, true>)
                          : (waves == 8 ? (const void*)k_batch<8, true, false> : (const void*)k_batch<4, true, false>);
    const hipError_t oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k1, waves * 64, lds);
    const hipError_t op = hipOccupancyMaxActiveBlocksPerMultiprocessor(&np, k2, waves * 64, lds);
    c->occ_waves = waves;
    c->occ_lds = (int)lds;
    c->occ_cols = cols;
    c->occ_blocks = oe == hipSuccess ? nb : 0;
    c->occ_blocks_pairs = op == hipSuccess ? np : 0;
  }
  if ((long long)c->occ_blocks * c->cus_total < G) return cols ? -3 : 1;
  // two sets of G blocks: every one resident, and within the slot table
  const bool pairs = c->pairs && 2 * G <= kMaxGrid && (long long)c->occ_blocks_pairs * c->cus_total >= 2 * G;
  c->last_grid = G;
  c->last_npb = npb;
  for (int base = 0; base < B; base += kBatchCap) {
    const int m = B - base < kBatchCap ? B - base : kBatchCap;
    for (int j = 0; j < m; ++j)
      if (reqs[base + j].use_candidates) return -3;
    memcpy(c->h_reqs, reqs + base, (size_t)m * sizeof(yoda_dev_req_t));
    if (c->epoch > 0xF0000000u) {   // tag space exhausted: forget every old tag
      CK(hipMemsetAsync(c->d_slots, 0, kSlotBytes, c->stream));
      c->epoch = 1;
    }
    BatchArgs a;
    a.pa = c->pend;
    a.nodes = c->d_nodes;
    a.n = n;
    a.npb = npb;
    a.B = m;
    c->seq = c->seq >= (1 << 30) ? 1 : c->seq + 1;
    a.seq = c->seq;
    a.tag0 = c->epoch;
    c->epoch += 3u * (uint32_t)m + 3u;
    a.deadline_ticks = c->deadline_ticks;   // 20 ms per wait by default
    a.reqs = c->d_reqs_map;
    a.slots = c->d_slots;
    a.res = c->d_bres;
    a.out = c->d_resb;
    a.done = c->d_done_map;
    a.ticket = c->d_words;
    a.abort_word = c->d_words + 1;
    a.trace = c->d_trace;
    a.sp_cnt = c->d_sp_cnt;
    a.sp_dom = c->d_sp_dom;
    a.sp_zc = c->d_sp_zc;
    a.img = c->d_img;
    a.logtab = c->d_logtab;
    a.n_sp = c->x_sp;
    a.n_img = c->x_img;
    __atomic_store_n(c->h_done, 0, __ATOMIC_RELEASE);
    if (c->timing) CK(hipEventRecord(c->e0, c->stream));
    if (pairs && m >= 2) {
      if (cols) {
        if (waves == 8) hipLaunchKernelGGL((k_batch<8, true, true>), dim3(2 * G), dim3(512), lds, c->stream, a);
        else hipLaunchKernelGGL((k_batch<4, true, true>), dim3(2 * G), dim3(256), lds, c->stream, a);
      } else {
        if (waves == 8) hipLaunchKernelGGL((k_batch<8, true, false>), dim3(2 * G), dim3(512), lds, c->stream, a);
        else hipLaunchKernelGGL((k_batch<4, true, false>), dim3(2 * G), dim3(256), lds, c->stream, a);
      }
    } else {
      if (cols) {
        if (waves == 8) hipLaunchKernelGGL((k_batch<8, false, true>), dim3(G), dim3(512), lds, c->stream, a);
        else hipLaunchKernelGGL((k_batch<4, false, true>), dim3(G), dim3(256), lds, c->stream, a);
      } else {
        if (waves == 8) hipLaunchKernelGGL((k_batch<8, false, false>), dim3(G), dim3(512), lds, c->stream, a);
        else hipLaunchKernelGGL((k_batch<4, false, false>), dim3(G), dim3(256), lds, c->stream, a);
      }
    }
    c->last_pairs = pairs && m >= 2;
    c->pend.n = 0;
    CK(hipGetLastError());
    ++c->n_dispatch;
    ++c->n_kbatch;
    if (c->timing) CK(hipEventRecord(c->e1, c->stream));
    // wait for `done` (system-scope release by the last block), polling the stream now and
    // then so a failed launch cannot hang the scheduler. A batch runs for milliseconds: spin
    // for the first ~100 µs (short batches), then poll every ~20 µs instead of burning a core.
    // Past the host deadline (blocks not resident: a tenant kernel holds the CUs) the batch
    // is abandoned — the engine places it on the CPU — and the context refuses work until
    // the stream drains (the kernel's own spin deadline ends it once it gets the CUs).
    const auto t0 = std::chrono::steady_clock::now();
    const double limit = host_deadline_s(c, m);
    // most of a long batch's run is known in advance (µs per pod of the recent batches): sleep
    // through ~3/4 of it in one go instead of ~50 µs-spaced wake-ups (each one a few µs of
    // this thread's CPU, ≈ 2 µs/pod in config 6), then poll as below
    if (c->wait_us_per_pod > 0 && m >= 16) {
      const double ahead_us = 0.75 * c->wait_us_per_pod * m - 80.0;   // − the timer's slack
      const double cap_us = 0.5 * limit * 1e6;   // a slow past batch must not outsleep the deadline
      if (ahead_us > 100.0) {
        std::this_thread::sleep_for(std::chrono::microseconds((long long)(ahead_us < cap_us ? ahead_us : cap_us)));
        ++c->n_presleep;
      }
    }
    int d = 0;
    for (unsigned spin = 1;; ++spin) {
      d = __atomic_load_n(c->h_done, __ATOMIC_ACQUIRE);
      if (d != 0) break;
      if (spin > 2048) std::this_thread::sleep_for(std::chrono::microseconds(20));
      // the stream is asked only now and then (a launch failure or the host deadline): `done`
      // is the completion signal, and each query wakes the runtime's own threads
      if (spin <= 2048 ? (spin & 255) == 0 : (spin & 63) == 0) {
        const hipError_t q = hipStreamQuery(c->stream);
        if (q == hipSuccess) {
          d = __atomic_load_n(c->h_done, __ATOMIC_ACQUIRE);
          break;
        }
        if (q != hipErrorNotReady) return (int)q;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
          c->abandoned = true;
          c->abandon_wait_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
          ++c->n_abandon;
          return -8;
        }
      }
      __builtin_ia32_pause();
    }
    if (d != c->seq) {   // aborted (a spin gave up) or no result: re-arm and report
      CK(hipStreamSynchronize(c->stream));
      CK(hipMemsetAsync(c->d_words, 0, 64, c->stream));
      CK(hipStreamSynchronize(c->stream));
      return -7;
    }
    memcpy(out + base, c->h_resb, (size_t)m * sizeof(yoda_dev_result_t));
    c->trace_pods = m;
    c->n_kbatch_pods += m;
    if (m >= 16) {   // the batch's wall time per pod (launch → done seen), smoothed
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / m;
      c->wait_us_per_pod = c->wait_us_per_pod > 0 ? 0.75 * c->wait_us_per_pod + 0.25 * us : us;
    }
    if (c->timing) {
      CK(hipEventSynchronize(c->e1));
      float ms = 0;
      if (hipEventElapsedTime(&ms, c->e0, c->e1) == hipSuccess) {
        c->last_us = ms * 1000.0f;
        c->kbatch_us += ms * 1000.0;
      }
    }
  }
  return 0;
}

int yoda_dev_batch_extras(void* p, int n, int n_spread, const int32_t* cnt, const uint8_t* dom, const int32_t* zc,
                          int n_img, const int32_t* img) {
  Ctx* c = (Ctx*)p;
  if (!c || n <= 0 || n > c->cap || n_spread < 0 || n_spread > kSP || n_img < 0 || n_img > kIMG) return -1;
  // the previous batch is complete (calls are synchronous): the staging memory is free
  if (n_spread) {
    memcpy(c->h_sp_cnt, cnt, (size_t)n_spread * n * sizeof(int32_t));
    memcpy(c->h_sp_dom, dom, (size_t)n_spread * n);
    memcpy(c->h_sp_zc, zc, (size_t)n_spread * kDOM * sizeof(int32_t));
  }
  if (n_img) memcpy(c->h_img, img, (size_t)n_img * n * sizeof(int32_t));
  c->x_n = n;
  c->x_sp = n_spread;
  c->x_img = n_img;
  return 0;
}

// B consecutive cycles enqueued back to back: each cycle's winner is assumed on the
// device (its node row updated in place by the publishing block), so cycle b+1 sees cycle
// b's reservation exactly as sequential host cycles would — no host round trip between
// pods. Candidates are not supported here (callers use yoda_dev_schedule for those).
int yoda_dev_schedule_batch(void* p, int n, int B, const yoda_dev_req_t* reqs, yoda_dev_result_t* out) {
  Ctx* c = (Ctx*)p;
  if (n <= 0 || n > c->cap || B < 0) return -1;
  CK(hipSetDevice(c->device));
  const bool cols = c->x_sp > 0 || c->x_img > 0;
  if (const int b = busy_check(c)) {
    c->x_sp = c->x_img = 0;
    return b;
  }
  if (c->persist && B > 0) {
    const int rc = batch_persistent(c, n, B, reqs, out);
    c->x_sp = c->x_img = 0;   // the staged columns were this call's
    if (rc <= 0) return rc;
  }
  c->x_sp = c->x_img = 0;
  if (cols) return -3;        // the launch chain has no score columns
  for (int base = 0; base < B; base += kBatchCap) {
    const int m = B - base < kBatchCap ? B - base : kBatchCap;
    for (int j = 0; j < m; ++j) {
      if (reqs[base + j].use_candidates) return -3;
      __atomic_store_n(&c->h_resb[j].feasible, -1, __ATOMIC_RELEASE);
    }
    for (int j = 0; j < m; ++j) {
      const int rc = launch_cycle(c, n, reqs[base + j], c->d_resb + j, 2u);
      if (rc != 0) return rc;
    }
    const int w = wait_slot(c, &c->h_resb[m - 1], m);
    if (w != 0) return w;
    for (int j = 0; j < m; ++j)
      if (__atomic_load_n(&c->h_resb[j].feasible, __ATOMIC_ACQUIRE) < 0) return -4;
    memcpy(out + base, c->h_resb, (size_t)m * sizeof(yoda_dev_result_t));
    c->trace_pods = m;
  }
  return 0;
}

// Phase trace of the persistent kernel (benchmarks): on = 1 records, per pod of the last
// k_batch chunk, block 0's s_memrealtime stamps (100 MHz) at kTracePts phase boundaries:
// start, F published, A computed, F gathered, B published, B gathered, Sel published, Sel
// gathered, end.
// Returns the number of pods copied to `out` (kTracePts words each), or the grid/npb of the
// last launch when out is NULL (grid << 16 | npb).
int yoda_dev_batch_trace(void* p, int on, unsigned long long* out, int max_pods) {
  Ctx* c = (Ctx*)p;
  if (!c) return -1;
  CK(hipSetDevice(c->device));
  if (on && !c->d_trace) {
    CK(hipMalloc(&c->d_trace, (size_t)kBatchCap * kTracePts * 8));
    // the PAIRS owner stamps (9..13) are written only for pods with a fix-up: zero = none
    CK(hipMemset(c->d_trace, 0, (size_t)kBatchCap * kTracePts * 8));
  }
  if (!on && c->d_trace) {
    CK(hipFree(c->d_trace));
    c->d_trace = nullptr;
  }
  if (!out) return (c->last_grid << 16) | c->last_npb;
  if (!c->d_trace) return 0;
  const int m = c->trace_pods < max_pods ? c->trace_pods : max_pods;
  CK(hipStreamSynchronize(c->stream));
  if (m > 0) CK(hipMemcpy(out, c->d_trace, (size_t)m * kTracePts * 8, hipMemcpyDeviceToHost));
  return m;
}

// PAIRS mode on/off for the next batches (tests compare both; YODA_DEV_PAIRS sets the default)
void yoda_dev_set_pairs(void* p, int on) {
  if (p) ((Ctx*)p)->pairs = on != 0;
}

void yoda_dev_set_timing(void* p, int on) {
  if (p) ((Ctx*)p)->timing = on != 0;
}

int yoda_dev_debug(void* p, int n, uint8_t* feas, int64_t* raw, int64_t* total, uint32_t* mask, int32_t* quality) {
  Ctx* c = (Ctx*)p;
  if (n <= 0 || n > c->cap) return -1;
  CK(hipSetDevice(c->device));
  if (const int b = busy_check(c)) return b;
  if (flush_pending(c) != 0) return -6;
  CK(hipStreamSynchronize(c->stream));
  if (feas) CK(hipMemcpy(feas, c->d_feas, (size_t)n, hipMemcpyDeviceToHost));
  if (raw) CK(hipMemcpy(raw, c->d_raw, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (total) CK(hipMemcpy(total, c->d_total, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (mask) CK(hipMemcpy(mask, c->d_mask, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  if (quality) CK(hipMemcpy(quality, c->d_quality, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost));
  return 0;
}

float yoda_dev_last_us(void* p) { return p ? ((Ctx*)p)->last_us : 0.f; }

// 1 while the context refuses work (an abandoned call still drains; see busy_check), else 0.
// The engine asks before packing rows for an upload.
int yoda_dev_busy(void* p) {
  Ctx* c = (Ctx*)p;
  if (!c || !c->abandoned) return 0;
  if (hipSetDevice(c->device) != hipSuccess) return 1;
  return busy_check(c) != 0;
}

// out[0..8] (9 values; 11 with the batch wait's pre-sleep count and µs/pod, 12 with whether the last
// k_batch ran in PAIRS mode; n = the caller's buffer length, checked): kernel dispatches, k_batch
// dispatches, pods placed by k_batch, calls abandoned at the host deadline, calls refused while
// an abandoned one drained, k_batch GPU µs (timing on), stream queries made while draining and
// their µs, the host's wait on the last abandoned call
int yoda_dev_counters(void* p, double* out, int n) {
  const Ctx* c = (const Ctx*)p;
  if (!c || !out || n < 9) return -1;
  out[0] = (double)c->n_dispatch;
  out[1] = (double)c->n_kbatch;
  out[2] = (double)c->n_kbatch_pods;
  out[3] = (double)c->n_abandon;
  out[4] = (double)c->n_busy;
  out[5] = c->kbatch_us;
  out[6] = (double)c->n_query;
  out[7] = c->query_us;
  out[8] = c->abandon_wait_us;
  if (n >= 11) {   // the host's batch wait: pre-sleeps taken, smoothed µs per pod
    out[9] = (double)c->n_presleep;
    out[10] = c->wait_us_per_pod;
  }
  if (n >= 12) out[11] = c->last_pairs ? 1.0 : 0.0;   // the last k_batch ran two pods in flight
  return 0;
}

}  // extern "C"
