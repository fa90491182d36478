// amd-smi telemetry collector for MI355X nodes — the native replacement of the reference's
// external NVML-based SCV sniffer (readme.md:9-10,15).
//
// One sample per GPU: HBM total/used (amdsmi_get_gpu_vram_usage), GFX clock cur/max
// (amdsmi_get_clock_info), CU count (amdsmi_get_gpu_asic_info), HBM max bandwidth
// (amdsmi_get_gpu_vram_info), power limit + current power (amdsmi_get_power_info), gfx/umc
// activity (amdsmi_get_gpu_activity), ECC totals (amdsmi_get_gpu_total_ecc_count), NUMA node,
// compute/memory partition, xGMI link status and per-link read/write counters
// (amdsmi_get_link_metrics) turned into per-peer rates/load by differencing successive samples.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace yoda {

struct LinkSample {
  std::string peer_bdf;
  int type = 0;              // amdsmi_link_type_t (2 = XGMI)
  uint32_t bit_rate = 0;     // Gb/s
  uint32_t max_bw = 0;       // Gb/s
  uint64_t read_kb = 0, write_kb = 0;   // cumulative counters
  double read_kbps = 0, write_kbps = 0; // rates since the previous sample
  double load = 0;           // (read+write rate) / (2 × max bandwidth), clamped to [0, 1]
};

// amd-smi topology to another GPU of the node (amdsmi_topo_get_link_type / _weight)
struct TopoPeer {
  int peer = 0;              // amd-smi index of the peer
  int type = 0;              // amdsmi_link_type_t (2 = XGMI, 1 = PCIe)
  uint64_t hops = 0;
  uint64_t weight = 0;
};

struct GpuSample {
  int index = 0;
  std::string bdf;
  std::string model;
  // identity: amd-smi index is BDF order; HIP/ROCr enumerate in KFD order, which can
  // differ (and partitions add logical GPUs per BDF) — the UUIDs are the stable names
  std::string uuid;          // amdsmi_get_gpu_device_uuid
  std::string hip_uuid;      // amdsmi_get_gpu_enumeration_info (what ROCR_VISIBLE_DEVICES accepts)
  int hip_id = -1, hsa_id = -1, drm_render = -1, drm_card = -1;
  int kfd_node = -1, partition_id = -1;
  // tenants: processes with a context on this GPU and the CUs their queues occupy
  int processes = -1;
  uint32_t proc_cus = 0;     // Σ amdsmi_proc_info_t.cu_occupancy
  uint64_t proc_vram_mb = 0;
  std::vector<TopoPeer> topo;
  uint32_t vram_total_mb = 0, vram_used_mb = 0;
  uint32_t sclk_cur = 0, sclk_max = 0, mclk_max = 0;
  uint32_t cus = 0;
  uint64_t hbm_bw_gbps = 0;
  uint32_t power_limit_w = 0, power_w = 0;
  uint32_t gfx_activity = 0, umc_activity = 0;
  uint64_t ecc_uncorrectable = 0, ecc_correctable = 0;
  int numa = -1;
  std::string compute_partition, memory_partition;
  int links_up = 0, links_down = 0;
  std::vector<LinkSample> links;
  double t = 0;              // unix seconds
  std::vector<std::string> errors;   // fields amd-smi could not read
};

class Collector {
 public:
  Collector() = default;
  ~Collector();
  Collector(const Collector&) = delete;
  Collector& operator=(const Collector&) = delete;

  // Initialise amd-smi and enumerate GPU processors. Returns false (with a message) if
  // the library or driver is unavailable (e.g. a CPU-only build box).
  bool init(std::string* err);
  int count() const { return (int)handles_.size(); }
  std::vector<GpuSample> sample();
  void shutdown();

 private:
  std::vector<void*> handles_;
  bool inited_ = false;
  // previous link counters for rate estimation: (gpu, link) → (t, read, write)
  std::map<std::pair<int, int>, std::tuple<double, uint64_t, uint64_t>> prev_;
};

std::string to_json(const std::vector<GpuSample>& s);

}  // namespace yoda
