// gfx950 device placement scorer: one scheduling cycle of the yoda profile over every node
// of a large MI355X cluster, bit-exact with the CPU engine (native/core/engine.cpp, fixed
// mode) — Filter → PreScore maxima → yoda Score + xGMI gang search → NormalizeScore →
// weighted sum → selectHost.
//
// CDNA4 mapping
//  * a 64-lane wave scores 8 nodes at once: lane group g (8 lanes) owns node base+g and
//    lane s of the group owns GPU slot s, so eligibility is one 64-bit __ballot split in
//    8-bit fields and every per-node reduction is a 3-step __shfl_xor inside the group;
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
#include <cstdint>
#include <cstdio>
#include <cstdlib>
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

// Exact floor(n / d) for d > 0: a correctly rounded double quotient is within 1 of the
// truth while n < 2^53; one integer multiply-subtract fixes it. Larger n (not produced
// by realistic clusters) take the software divide.
__device__ __forceinline__ uint64_t udiv(uint64_t n, uint64_t d) {
  if (n < (1ull << 53) && d < (1ull << 53)) {
    uint64_t q = (uint64_t)((double)n / (double)d);
    const uint64_t qd = q * d;
    if (qd > n) --q;
    else if (n - qd >= d) ++q;
    return q;
  }
  return n / d;
}
// truncating int division by a tiny divisor (≤ 28): every non-integer quotient is at least
// 1/28 away from an integer, far beyond the double rounding error → exact
__device__ __forceinline__ int32_t sdiv_small(int32_t n, int32_t d) { return (int32_t)((double)n / (double)d); }

__device__ __forceinline__ uint64_t eff_free(uint32_t free, uint32_t pending, uint32_t total, uint32_t reserved) {
  const uint64_t sampled = free > pending ? (uint64_t)(free - pending) : 0;
  const uint64_t cap = total > reserved ? (uint64_t)(total - reserved) : 0;
  return sampled < cap ? sampled : cap;
}

template <typename T>
__device__ __forceinline__ T gmax(T v) {   // max over the 8 lanes of a group
#pragma unroll
  for (int off = 4; off > 0; off >>= 1) {
    const T o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}
template <typename T>
__device__ __forceinline__ T gsum(T v) {
#pragma unroll
  for (int off = 4; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wmax_across_groups(T v) {   // max over the 8 groups of a wave
#pragma unroll
  for (int off = 8; off < 64; off <<= 1) {
    const T o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

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

// ------------------------------------------------------------------ K1: filter + maxima
// One lane group = one node (lane `sub` = GPU slot). Writes feas/elig, counts the reason,
// folds the card metrics of feasible nodes into the wave maxima `wmx`.
__device__ __forceinline__ void filter_group(const yoda_dev_node_t* nd, int i, bool valid, const yoda_dev_req_t& r,
                                             const uint8_t* __restrict__ cand, uint8_t* __restrict__ feas,
                                             uint8_t* __restrict__ elig, int* s_reason, unsigned long long* wmx,
                                             int& nfeas, int grp, int sub) {
  const bool yoda = (r.filters & F_YODA) != 0;
  // every load of the node issued up front: one memory round trip per node
  const uint8_t flags = valid ? nd->flags : 0, ncards = nd->ncards;
  const uint32_t card_number = nd->card_number;
  const int64_t pod_count = nd->pod_count, alloc_pods = nd->alloc_pods, alloc_cpu = nd->alloc_cpu,
                req_cpu = nd->req_cpu, alloc_mem = nd->alloc_mem, req_mem = nd->req_mem;
  const yoda_dev_card_t cd = nd->cards[sub];
  const uint8_t healthy = nd->healthy[sub];
  const uint8_t cnd = (r.use_candidates && valid) ? cand[i] : 0;
  int reason = 0;
  if (!(flags & YODA_DEV_ALIVE)) {
    reason = RS_DEAD;
  } else if ((r.filters & F_NODE_UNSCHEDULABLE) && (flags & YODA_DEV_UNSCHEDULABLE) && !r.tolerates_unschedulable) {
    reason = RS_UNSCHEDULABLE;
  } else if (r.filters & F_NODE_RESOURCES_FIT) {
    if (pod_count + 1 > alloc_pods) reason = RS_RESOURCES;
    else if (r.cpu_m > 0 && alloc_cpu < r.cpu_m + req_cpu) reason = RS_RESOURCES;
    else if (r.mem > 0 && alloc_mem < r.mem + req_mem) reason = RS_RESOURCES;
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
  if (valid && sub == 0) {
    feas[i] = ok;
    elig[i] = (uint8_t)emask;
    if (reason) atomicAdd(&s_reason[reason], 1);
  }
  if (sub == 0 && ok) ++nfeas;
  if (yoda) {
    const bool take = ok && ((emask >> sub) & 1u);
    unsigned long long v[6];
    v[0] = take ? cd.bandwidth : 0; v[1] = take ? cd.clock : 0; v[2] = take ? cd.core : 0;
    v[3] = take ? ef : 0; v[4] = take ? cd.power : 0; v[5] = take ? cd.total : 0;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const unsigned long long m = wmax_across_groups(gmax(v[k]));
      wmx[k] = m > wmx[k] ? m : wmx[k];
    }
  }
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
  unsigned long long wmx[6] = {1, 1, 1, 1, 1, 1};
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
  nfeas = gsum(nfeas);
  nfeas += __shfl_xor(nfeas, 8, 64);
  nfeas += __shfl_xor(nfeas, 16, 64);
  nfeas += __shfl_xor(nfeas, 32, 64);
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
  // trips instead of one per node stride
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
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_xor(best, off, 64);
    best = o > best ? o : best;
  }
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
  const bool yoda_f = (r.filters & F_YODA) != 0;
  const bool yoda_s = yoda_f && r.w_yoda != 0;
  const uint64_t mx0 = g->maxima[0], mx1 = g->maxima[1], mx2 = g->maxima[2], mx3 = g->maxima[3], mx4 = g->maxima[4],
                 mx5 = g->maxima[5];
  const int k = (int)(r.has_number ? (r.number > 64 ? 64 : r.number) : 1);
  const bool search = yoda_f && k >= 1 && k <= YODA_DEV_CARDS;
  const int32_t P = k * (k - 1) / 2;
  const int s_begin = search ? c_subsets.start[k] : 0, s_end = search ? c_subsets.start[k + 1] : 0;
  const int64_t nz_cpu = r.nz_cpu_m, nz_mem = r.nz_mem;
  unsigned long long lo = ULLONG_MAX, hi = 0;
  const int stride = gridDim.x * kWaves * kNodesPerWave;
  for (int base = uniform((blockIdx.x * kWaves + wave) * kNodesPerWave); base < n; base += stride) {
    const int i = base + grp;
    // no early exit on an all-infeasible wave: the node loads below then issue together
    // with feas/elig instead of one round trip later
    const bool act = i < n && feas[i];
    const yoda_dev_node_t* nd = nodes + (i < n ? i : n - 1);
    const uint32_t emask = act ? elig[i] : 0u;
    const uint8_t ncards = nd->ncards;
    // ---- per-node register tables (every lane of the group holds the whole node)
    uint64_t ef[YODA_DEV_CARDS];
    uint32_t tot[YODA_DEV_CARDS], occ[YODA_DEV_CARDS], numa[YODA_DEV_CARDS];
#pragma unroll
    for (int a = 0; a < YODA_DEV_CARDS; ++a) {
      const uint4 lo4 = reinterpret_cast<const uint4*>(&nd->cards[a])[0];   // total, free, reserved, pending
      ef[a] = eff_free(lo4.y, lo4.w, lo4.x, lo4.z);
      tot[a] = lo4.x;
      occ[a] = nd->occ[a];
      numa[a] = nd->numa[a] & 63u;
    }
    uint32_t lq[32];   // 64 u16 card-pair qualities, packed 2 per dword
    {
      const uint4* q4 = reinterpret_cast<const uint4*>(&nd->linkq[0][0]);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        const uint4 v = q4[t];
        lq[4 * t] = v.x; lq[4 * t + 1] = v.y; lq[4 * t + 2] = v.z; lq[4 * t + 3] = v.w;
      }
    }
    // ---- gang / GPU-set selection (the Reserve choice if this node wins)
    uint32_t best_m = 0;
    int64_t best_o = LLONG_MAX;
    int32_t best_lb = 0;
    bool found = false;
    if (search && act && k == 1) {
      // single-GPU pods (the bulk of a mixed burst): the k = 1 table is {1<<0 … 1<<7} in
      // order, so lane `sub` owns subset {sub}; no pairs (P = 0) and one NUMA domain leave
      // only the fit and occupancy terms — the generic loop's 28 predicated pair adds and
      // 8-card sums are skipped. Same integer arithmetic, so the result is bit-identical.
      if ((emask >> sub) & 1u) {
        uint64_t efs = ef[0];
        uint32_t tos = tot[0], ocs = occ[0];
#pragma unroll
        for (int a = 1; a < YODA_DEV_CARDS; ++a) {
          efs = sub == a ? ef[a] : efs;
          tos = sub == a ? tot[a] : tos;
          ocs = sub == a ? occ[a] : ocs;
        }
        const uint64_t fa = efs - r.memory;
        const int64_t leftover = tos ? (int64_t)udiv(fa * 1000000ull, (uint64_t)tos) : 0;
        const int64_t fit = r.binpack ? leftover : 1000000 - leftover;
        const int64_t occ_bad = (int64_t)sdiv_small((int32_t)(ocs * 100u), 1);
        best_o = r.w_fit * fit + r.w_occ * occ_bad;
        best_m = 1u << sub;
        best_lb = 0;
        found = true;
      }
#pragma unroll
      for (int off = 4; off > 0; off >>= 1) {
        const int64_t oo = __shfl_xor(best_o, off, 64);
        const uint32_t om = __shfl_xor(best_m, off, 64);
        const int32_t ol = __shfl_xor(best_lb, off, 64);
        const int of = __shfl_xor((int)found, off, 64);
        if (of && (!found || better(oo, om, best_o, best_m))) {
          best_o = oo; best_m = om; best_lb = ol; found = true;
        }
      }
    } else if (search && act) {
      for (int t = s_begin + sub; t < s_end; t += kGroup) {
        const uint32_t m = s_masks[t];
        if (m & ~emask) continue;
        int32_t qsum = 0;
        uint64_t nmask = 0;
        uint64_t fa = 0, tt = 0;
        uint32_t oc = 0;
#pragma unroll
        for (int a = 0; a < YODA_DEV_CARDS; ++a) {
          const bool ia = (m >> a) & 1u;
          nmask |= ia ? (1ull << numa[a]) : 0ull;
          fa += ia ? ef[a] - r.memory : 0;
          tt += ia ? tot[a] : 0;
          oc += ia ? occ[a] : 0u;
#pragma unroll
          for (int b = a + 1; b < YODA_DEV_CARDS; ++b) {
            const int idx = a * YODA_DEV_CARDS + b;
            const int32_t q = (int32_t)((lq[idx >> 1] >> ((idx & 1) * 16)) & 0xFFFFu);
            qsum += (ia && ((m >> b) & 1u)) ? q : 0;
          }
        }
        const int32_t lb = P ? sdiv_small((P * 10000 - qsum) * 100, P) : 0;
        const int32_t d = __popcll(nmask);
        const int64_t numa_bad = k > 1 ? (int64_t)sdiv_small((d - 1) * 1000000, k - 1) : 0;
        const int64_t leftover = tt ? (int64_t)udiv(fa * 1000000ull, tt) : 0;
        const int64_t fit = r.binpack ? leftover : 1000000 - leftover;
        const int64_t occ_bad = (int64_t)sdiv_small((int32_t)(oc * 100u), k);
        const int64_t o = r.w_link * (int64_t)lb + r.w_numa * numa_bad + r.w_fit * fit + r.w_occ * occ_bad;
        if (!found || better(o, m, best_o, best_m)) {
          best_o = o; best_m = m; best_lb = lb; found = true;
        }
      }
#pragma unroll
      for (int off = 4; off > 0; off >>= 1) {
        const int64_t oo = __shfl_xor(best_o, off, 64);
        const uint32_t om = __shfl_xor(best_m, off, 64);
        const int32_t ol = __shfl_xor(best_lb, off, 64);
        const int of = __shfl_xor((int)found, off, 64);
        if (of && (!found || better(oo, om, best_o, best_m))) {
          best_o = oo; best_m = om; best_lb = ol; found = true;
        }
      }
    } else {
      // keep the shuffles wave-uniform for inactive groups
#pragma unroll
      for (int off = 4; off > 0; off >>= 1) {
        (void)__shfl_xor(best_o, off, 64);
        (void)__shfl_xor(best_m, off, 64);
        (void)__shfl_xor(best_lb, off, 64);
        (void)__shfl_xor((int)found, off, 64);
      }
    }
    const int32_t quality = found ? 10000 - sdiv_small(best_lb, 100) : 10000;
    // ---- yoda raw score (algorithm.go:28-87 with the Q1/Q2/Q3/Q4 fixes); lane sub = card sub
    uint64_t basic = 0, tsum = 0, fsum = 0, asum = 0;
    if (act && sub < ncards) {
      const yoda_dev_card_t cd = nd->cards[sub];
      tsum = cd.total;
      fsum = ef[0];
#pragma unroll
      for (int a = 1; a < YODA_DEV_CARDS; ++a) fsum = sub == a ? ef[a] : fsum;
      asum = cd.reserved;
      if ((emask >> sub) & 1u) {
        basic = udiv((uint64_t)cd.bandwidth * 100, mx0) + udiv((uint64_t)cd.clock * 100, mx1) +
                udiv((uint64_t)cd.core * 100, mx2) + udiv((uint64_t)cd.power * 100, mx4) +
                udiv(fsum * 100, mx3) * 2 + udiv((uint64_t)cd.total * 100, mx5);
      }
    }
    basic = gsum(basic);
    tsum = gsum(tsum);
    fsum = gsum(fsum);
    asum = gsum(asum);
    if (act && sub == 0) {
      int64_t s_out = 0;
      if (yoda_s) {
        const uint64_t actual = tsum ? udiv(fsum * 100, tsum) * 2 : 0;
        const uint64_t allocate = (tsum == 0 || tsum < asum) ? 0 : udiv((tsum - asum) * 100, tsum) * 3;
        uint64_t s = basic + allocate + actual;
        if (r.has_number && r.number > 1 && r.number <= ncards && found)
          s += (uint64_t)(quality / 100) * (uint64_t)r.w_gang_score;
        s_out = s > (uint64_t)LLONG_MAX ? 0 : (int64_t)s;
        const unsigned long long us = (unsigned long long)s_out;
        lo = us < lo ? us : lo;
        hi = us > hi ? us : hi;
      }
      // upstream default scores (engine.cpp Engine::score_nodes)
      const int64_t rc = nd->nz_cpu + nz_cpu, rm = nd->nz_mem + nz_mem;
      const int64_t ac = nd->alloc_cpu, am = nd->alloc_mem;
      int64_t least = 0, most = 0, extra = r.w_const;
      if (ac > 0 && rc <= ac) least += (int64_t)udiv((uint64_t)(ac - rc) * 100, (uint64_t)ac);
      if (am > 0 && rm <= am) least += (int64_t)udiv((uint64_t)(am - rm) * 100, (uint64_t)am);
      if (ac > 0) most += (int64_t)udiv((uint64_t)(rc < ac ? rc : ac) * 100, (uint64_t)ac);
      if (am > 0) most += (int64_t)udiv((uint64_t)(rm < am ? rm : am) * 100, (uint64_t)am);
      extra += r.w_least * (least / 2) + r.w_most * (most / 2);
      if (r.w_balanced) {
        const double cf = ac > 0 ? (double)rc / (double)ac : 1.0;
        const double mf = am > 0 ? (double)rm / (double)am : 1.0;
        const int64_t b = (cf >= 1 || mf >= 1) ? 0 : (int64_t)((1.0 - fabs(cf - mf)) * 100);
        extra += r.w_balanced * b;
      }
      raw[i] = s_out;
      total_out[i] = extra;
      mask_out[i] = best_m;
      quality_out[i] = quality;
    }
  }
  // wave-level min/max of the raw score (lanes that scored nothing hold the identities)
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long ol = __shfl_xor(lo, off, 64), oh = __shfl_xor(hi, off, 64);
    lo = ol < lo ? ol : lo;
    hi = oh > hi ? oh : hi;
  }
  if (lane == 0) {
    s_lo[wave] = lo;
    s_hi[wave] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0 && yoda_s) {
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
  yoda_dev_result_t *h_res = nullptr, *d_res_map = nullptr;
  yoda_dev_result_t *h_resb = nullptr, *d_resb = nullptr;   // batched cycles: one slot per pod
  Globals* d_g = nullptr;
  float last_us = 0;
  int grid = 1024;
  bool timing = false;        // event timing of each cycle (benchmarks); off in the scheduler
  int direct_atomics = -1;    // -1: by grid size; 0/1 forced (YODA_DEV_DIRECT_ATOMICS)
  int fuse_max = kFuseSelectMax;   // YODA_DEV_FUSE_MAX overrides (A/B of the fused select)
  PatchArgs pend{};           // dirty rows waiting to ride in the next filter launch
};

#define CK(x)                               \
  do {                                      \
    hipError_t e__ = (x);                   \
    if (e__ != hipSuccess) return (int)e__; \
  } while (0)

// launch the pending rows on their own (before a bulk scatter or a debug read)
int flush_pending(Ctx* c) {
  if (c->pend.n == 0) return 0;
  hipLaunchKernelGGL(k_patch, dim3(1), dim3(32 * kPatchRows), 0, c->stream, c->pend, c->d_nodes);
  c->pend.n = 0;
  CK(hipGetLastError());
  return 0;
}

// Wait for the device to publish the result: spin on the mapped `feasible` field (written
// last, system-scope release), polling the stream now and then so a failed launch or a
// result that never comes cannot hang the scheduler.
int wait_result(Ctx* c) {
  volatile int32_t* flag = &c->h_res->feasible;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) >= 0) return 0;
    if ((spin & 4095) == 0) {
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) >= 0 ? 0 : -4;
      if (q != hipErrorNotReady) return (int)q;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) return -5;
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
  hipFree(c->d_total); hipFree(c->d_mask); hipFree(c->d_quality); hipHostFree(c->h_res); hipHostFree(c->h_resb); hipFree(c->d_g);
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
  memcpy(c->h_stage, rows, (size_t)n * sizeof(yoda_dev_node_t));
  memcpy(c->h_idx, idx, (size_t)n * sizeof(int32_t));
  CK(hipMemcpyAsync(c->d_stage, c->h_stage, (size_t)n * sizeof(yoda_dev_node_t), hipMemcpyHostToDevice, c->stream));
  CK(hipMemcpyAsync(c->d_idx, c->h_idx, (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  const int per_block = 8;   // 8 records × 32 lanes = 256 threads
  hipLaunchKernelGGL(k_scatter, dim3((n + per_block - 1) / per_block), dim3(256), 0, c->stream, c->d_stage, c->d_idx,
                     n, c->d_nodes);
  CK(hipGetLastError());
  CK(hipStreamSynchronize(c->stream));   // staging buffers are reused by the next upload
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
  c->pend.n = 0;
  hipLaunchKernelGGL(k_score, dim3(grid), dim3(kBlock), 0, c->stream, c->d_nodes, n, r, c->d_feas, c->d_elig,
                     c->d_raw, c->d_total, c->d_mask, c->d_quality, c->d_g, out, fuse);
  if (!fuse)
    hipLaunchKernelGGL(k_select, dim3(grid_sel), dim3(kBlock), 0, c->stream, n, r, c->d_feas, c->d_raw, c->d_total,
                       c->d_mask, c->d_quality, c->d_g, out, c->d_nodes);
  CK(hipGetLastError());
  return 0;
}

// Spin until `slot->feasible` is published (see wait_result).
int wait_slot(Ctx* c, yoda_dev_result_t* slot) {
  volatile int32_t* flag = &slot->feasible;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 1;; ++spin) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) >= 0) return 0;
    if ((spin & 4095) == 0) {
      const hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) return __atomic_load_n(flag, __ATOMIC_ACQUIRE) >= 0 ? 0 : -4;
      if (q != hipErrorNotReady) return (int)q;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) return -5;
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

// B consecutive cycles enqueued back to back: each cycle's winner is assumed on the
// device (its node row updated in place by the publishing block), so cycle b+1 sees cycle
// b's reservation exactly as sequential host cycles would — no host round trip between
// pods. Candidates are not supported here (callers use yoda_dev_schedule for those).
int yoda_dev_schedule_batch(void* p, int n, int B, const yoda_dev_req_t* reqs, yoda_dev_result_t* out) {
  Ctx* c = (Ctx*)p;
  if (n <= 0 || n > c->cap || B < 0) return -1;
  CK(hipSetDevice(c->device));
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
    const int w = wait_slot(c, &c->h_resb[m - 1]);
    if (w != 0) return w;
    for (int j = 0; j < m; ++j)
      if (__atomic_load_n(&c->h_resb[j].feasible, __ATOMIC_ACQUIRE) < 0) return -4;
    memcpy(out + base, c->h_resb, (size_t)m * sizeof(yoda_dev_result_t));
  }
  return 0;
}

void yoda_dev_set_timing(void* p, int on) {
  if (p) ((Ctx*)p)->timing = on != 0;
}

int yoda_dev_debug(void* p, int n, uint8_t* feas, int64_t* raw, int64_t* total, uint32_t* mask, int32_t* quality) {
  Ctx* c = (Ctx*)p;
  if (n <= 0 || n > c->cap) return -1;
  CK(hipSetDevice(c->device));
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

}  // extern "C"
