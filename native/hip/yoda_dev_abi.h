// Shared C ABI between the native engine (g++, native/core) and the gfx950 device scorer
// (hipcc, native/hip/scorer.hip). The engine dlopen()s libyoda_hip.so and resolves the
// yoda_dev_* entry points, so the CPU-only build never links HIP.
//
// Layout: one 512-byte record per node (AoS, 16-byte aligned) — a wave handles one node,
// lanes 0..7 its GPU slots, so a node's cards are read as one contiguous 256-byte burst.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define YODA_DEV_CARDS 8
#define YODA_DEV_REASONS 16
// k_batch per-batch score columns (yoda_dev_batch_extras): up to 2 PodTopologySpread soft
// constraint sets ("spread slots") and 2 ImageLocality image sets ("image slots") per batch
#define YODA_DEV_SPREAD_SLOTS 2
#define YODA_DEV_IMAGE_SLOTS 2
#define YODA_DEV_DOMAINS 64          // distinct values of a spread slot's non-hostname key
#define YODA_DEV_DOM_NONE 0xFF       // the node lacks one of the slot's topology keys (ignored)

enum {
  YODA_DEV_ALIVE = 1,
  YODA_DEV_HAS_SCV = 2,
  YODA_DEV_STALE = 4,
  YODA_DEV_UNSCHEDULABLE = 8,
};

typedef struct {
  uint32_t total, free, reserved, pending;   // MB
  uint32_t clock, bandwidth, core, power;
} yoda_dev_card_t;   // 32 B

typedef struct {
  yoda_dev_card_t cards[YODA_DEV_CARDS];     // 256
  uint16_t linkq[YODA_DEV_CARDS][YODA_DEV_CARDS];   // 128, card-pair xGMI quality (1e-4), host-resolved
  uint16_t occ[YODA_DEV_CARDS];              // 16, CU occupancy (1e-4)
  uint8_t healthy[YODA_DEV_CARDS];           // 8
  uint8_t phys[YODA_DEV_CARDS];              // 8
  uint8_t numa[YODA_DEV_CARDS];              // 8
  int64_t alloc_cpu, alloc_mem, alloc_pods;  // 24
  int64_t req_cpu, req_mem, pod_count;       // 24
  uint32_t card_number;                      // 4  (Scv.Status.CardNumber)
  uint8_t ncards, nphys, flags, pad0;        // 4
  int64_t nz_cpu, nz_mem;                    // 16 Σ non-zero requests (scores)
  int64_t ext_alloc, ext_used;               // 16 the device's one extended resource (engine: dev_ext_res_)
} yoda_dev_node_t;   // 512 B
#ifdef __cplusplus
static_assert(sizeof(yoda_dev_node_t) == 512, "node record must stay 512 B");
#endif

typedef struct {
  uint64_t number;        // effective GPU count (1 when the label is absent)
  uint64_t memory;        // MB per GPU (0 when absent)
  uint64_t clock;         // exact-match clock (0 when absent)
  uint64_t clock_min;
  int64_t cpu_m, mem;     // pod requests (fit)
  int64_t nz_cpu_m, nz_mem;   // pod non-zero requests (Least/Most/Balanced scores)
  int64_t w_yoda, w_least, w_balanced, w_most, w_const;   // score weights; w_const added to every node
  int64_t w_link, w_numa, w_fit, w_occ, w_gang_score;
  int64_t w_minlink;      // bottleneck xGMI pair term (engine.hpp Weights::w_minlink)
  uint32_t has_number, has_memory, has_clock, binpack;
  uint32_t filters;       // engine FilterBit mask (only UNSCHEDULABLE/RESOURCES/YODA are evaluated here)
  uint32_t tolerates_unschedulable;
  uint32_t use_candidates;   // 1: per-node first-failing NodeName/Affinity/Taint reason uploaded
  uint32_t perm_mul, perm_add, perm_inv;   // random tie-break: p(i) = (i*mul + add) mod 2^24
  uint32_t dev_flags;     // set by the device context, not the engine
  int64_t ext;            // request of the device's extended resource (0: none)
  // k_batch only (the per-pod launch chain has no score columns: the engine never sends it a
  // pod with a slot). PodTopologySpread soft constraints of slot `spread_slot` (-1: none), in
  // the engine's constraint order: ckind 0 = kubernetes.io/hostname (the node's own count),
  // 1 = the slot's domain key (its domain's count); maxSkew per constraint; the score weight
  int32_t spread_w;
  int8_t spread_slot, img_slot;   // img_slot: ImageLocality column (weighted), -1: none
  uint8_t spread_nc;              // constraints (1..2)
  uint8_t match_mask;             // bit s: once assumed, this pod counts for slot s's selector
  uint8_t ckind[2];
  uint8_t pad2[2];
  int32_t cskew[2];
} yoda_dev_req_t;

typedef struct {
  int32_t node;           // chosen node index, -1 = none feasible
  int32_t feasible;
  int64_t score;
  uint32_t mask;          // chosen GPU set on `node` (bit i = card i)
  int32_t quality;        // xGMI pair quality of the set, 0..10000
  int32_t reasons[YODA_DEV_REASONS];
  uint64_t maxima[6];     // bandwidth, clock, core, free, power, total
  int64_t raw_lo, raw_hi;
} yoda_dev_result_t;

// returns an opaque context or NULL (err filled)
void* yoda_dev_create(int device, int capacity, char* err, int err_len);
void yoda_dev_destroy(void* ctx);
int yoda_dev_capacity(void* ctx);
// copy `n` node records into slots idx[0..n)
int yoda_dev_upload(void* ctx, int n, const int32_t* idx, const yoda_dev_node_t* rows);
// candidates: NULL or `n_nodes` bytes (0 = pass, else engine Reason code)
int yoda_dev_schedule(void* ctx, int n_nodes, const yoda_dev_req_t* req, const uint8_t* candidates,
                      yoda_dev_result_t* out);
// debug/parity: per-node arrays from the last schedule call
// B cycles back to back, each winner assumed on the device before the next (no candidates)
int yoda_dev_schedule_batch(void* ctx, int n_nodes, int B, const yoda_dev_req_t* reqs, yoda_dev_result_t* out);
int yoda_dev_debug(void* ctx, int n_nodes, uint8_t* feas, int64_t* raw, int64_t* total, uint32_t* mask,
                   int32_t* quality);
// Score columns for the next yoda_dev_schedule_batch call (consumed by it): for each of
// n_spread slots, per node the slot selector's matching pods (`cnt`, [slot][n]) and the node's
// domain id (`dom`, [slot][n], YODA_DEV_DOM_NONE: a key is missing), and per domain the
// matching pods over the nodes with every key (`zc`, [slot][YODA_DEV_DOMAINS]); for each of
// n_img slots, per node the weighted ImageLocality score (`img`, [slot][n]). 0 = accepted.
int yoda_dev_batch_extras(void* ctx, int n, int n_spread, const int32_t* cnt, const uint8_t* dom, const int32_t* zc,
                          int n_img, const int32_t* img);
// last kernel time of yoda_dev_schedule in microseconds (device events)
float yoda_dev_last_us(void* ctx);
// per-cycle event timing (yoda_dev_last_us); off by default — it adds a stream sync
void yoda_dev_set_timing(void* ctx, int on);

#ifdef __cplusplus
}
#endif
