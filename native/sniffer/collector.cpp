// amd-smi collector implementation (see collector.hpp).
#include "collector.hpp"

#include <cmath>

#include <amd_smi/amdsmi.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <sstream>
#include <tuple>

namespace yoda {

namespace {

double now_s() {
  using namespace std::chrono;
  return duration<double>(system_clock::now().time_since_epoch()).count();
}

std::string bdf_str(const amdsmi_bdf_t& b) {
  char buf[32];
  snprintf(buf, sizeof buf, "%04llx:%02llx:%02llx.%llx", (unsigned long long)b.domain_number,
           (unsigned long long)b.bus_number, (unsigned long long)b.device_number,
           (unsigned long long)b.function_number);
  return buf;
}

// JSON string body: escape quotes/backslashes, drop control characters, and replace bytes
// that are not part of a well-formed UTF-8 sequence (driver strings are not guaranteed
// UTF-8; the Python side decodes the JSON strictly).
std::string esc(const std::string& s) {
  std::string o;
  o.reserve(s.size());
  const size_t n = s.size();
  for (size_t i = 0; i < n;) {
    const unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      if (c == '"' || c == '\\') o += '\\';
      if (c >= 0x20) o += (char)c;
      ++i;
      continue;
    }
    int len = (c >= 0xC2 && c <= 0xDF) ? 2 : (c >= 0xE0 && c <= 0xEF) ? 3 : (c >= 0xF0 && c <= 0xF4) ? 4 : 0;
    bool ok = len > 0 && i + len <= n;
    for (int k = 1; ok && k < len; ++k) ok = ((unsigned char)s[i + k] & 0xC0) == 0x80;
    if (ok && len == 3) {
      const unsigned char c1 = (unsigned char)s[i + 1];
      ok = !(c == 0xE0 && c1 < 0xA0) && !(c == 0xED && c1 >= 0xA0);   // overlong / surrogates
    } else if (ok && len == 4) {
      const unsigned char c1 = (unsigned char)s[i + 1];
      ok = !(c == 0xF0 && c1 < 0x90) && !(c == 0xF4 && c1 >= 0x90);
    }
    if (ok) {
      o.append(s, i, len);
      i += len;
    } else {
      o += '?';
      ++i;
    }
  }
  return o;
}

}  // namespace

Collector::~Collector() { shutdown(); }

void Collector::shutdown() {
  if (inited_) {
    amdsmi_shut_down();
    inited_ = false;
  }
  handles_.clear();
}

bool Collector::init(std::string* err) {
  if (inited_) return true;
  amdsmi_status_t st = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
  if (st != AMDSMI_STATUS_SUCCESS) {
    const char* msg = nullptr;
    amdsmi_status_code_to_string(st, &msg);
    if (err) *err = std::string("amdsmi_init: ") + (msg ? msg : "error");
    return false;
  }
  inited_ = true;
  uint32_t nsock = 0;
  if (amdsmi_get_socket_handles(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS) {
    if (err) *err = "amdsmi_get_socket_handles failed";
    return false;
  }
  std::vector<amdsmi_socket_handle> socks(nsock);
  amdsmi_get_socket_handles(&nsock, socks.data());
  for (uint32_t s = 0; s < nsock; ++s) {
    uint32_t n = 0;
    if (amdsmi_get_processor_handles(socks[s], &n, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> hs(n);
    amdsmi_get_processor_handles(socks[s], &n, hs.data());
    for (auto h : hs) handles_.push_back(h);
  }
  // stable order by PCI address (amd-smi/rocm-smi index order)
  std::vector<std::pair<uint64_t, void*>> order;
  for (void* h : handles_) {
    amdsmi_bdf_t b{};
    amdsmi_get_gpu_device_bdf((amdsmi_processor_handle)h, &b);
    order.emplace_back(b.as_uint, h);
  }
  std::sort(order.begin(), order.end(), [](auto& a, auto& b) { return a.first < b.first; });
  handles_.clear();
  for (auto& p : order) handles_.push_back(p.second);
  if (handles_.empty()) {
    if (err) *err = "no AMD GPU processors found";
    return false;
  }
  return true;
}

std::vector<GpuSample> Collector::sample() {
  std::vector<GpuSample> out;
  for (int i = 0; i < (int)handles_.size(); ++i) {
    auto h = (amdsmi_processor_handle)handles_[i];
    GpuSample g;
    g.index = i;
    g.t = now_s();
    amdsmi_bdf_t b{};
    if (amdsmi_get_gpu_device_bdf(h, &b) == AMDSMI_STATUS_SUCCESS) g.bdf = bdf_str(b);
    else g.errors.push_back("bdf");
    char uuid[AMDSMI_GPU_UUID_SIZE + 8] = {0};
    unsigned int ulen = sizeof(uuid);
    if (amdsmi_get_gpu_device_uuid(h, &ulen, uuid) == AMDSMI_STATUS_SUCCESS) g.uuid = uuid;
    else g.errors.push_back("uuid");
    amdsmi_enumeration_info_t en{};
    if (amdsmi_get_gpu_enumeration_info(h, &en) == AMDSMI_STATUS_SUCCESS) {
      g.hip_id = (int)en.hip_id;
      g.hsa_id = (int)en.hsa_id;
      g.drm_render = (int)en.drm_render;
      g.drm_card = (int)en.drm_card;
      g.hip_uuid = en.hip_uuid;
    } else {
      g.errors.push_back("enumeration");
    }
    amdsmi_kfd_info_t kf{};
    if (amdsmi_get_gpu_kfd_info(h, &kf) == AMDSMI_STATUS_SUCCESS) {
      if (kf.node_id != 0xFFFFFFFFu) g.kfd_node = (int)kf.node_id;
      if (kf.current_partition_id != 0xFFFFFFFFu) g.partition_id = (int)kf.current_partition_id;
    }
    uint32_t np = 0;
    if (amdsmi_get_gpu_process_list(h, &np, nullptr) == AMDSMI_STATUS_SUCCESS ||
        np > 0) {
      std::vector<amdsmi_proc_info_t> procs(np + 4);
      uint32_t cap = (uint32_t)procs.size();
      amdsmi_status_t pst = amdsmi_get_gpu_process_list(h, &cap, procs.data());
      if (pst == AMDSMI_STATUS_SUCCESS || pst == AMDSMI_STATUS_OUT_OF_RESOURCES) {
        uint32_t n = std::min<uint32_t>(cap, (uint32_t)procs.size());
        g.processes = (int)cap;
        for (uint32_t k = 0; k < n; ++k) {
          g.proc_cus += procs[k].cu_occupancy;
          g.proc_vram_mb += procs[k].memory_usage.vram_mem >> 20;
        }
      }
    } else {
      g.errors.push_back("process_list");
    }
    for (int j = 0; j < (int)handles_.size(); ++j) {
      if (j == i) continue;
      TopoPeer tp;
      tp.peer = j;
      amdsmi_link_type_t lt{};
      uint64_t hops = 0;
      if (amdsmi_topo_get_link_type(h, (amdsmi_processor_handle)handles_[j], &hops, &lt) != AMDSMI_STATUS_SUCCESS)
        continue;
      tp.type = (int)lt;
      tp.hops = hops;
      uint64_t w = 0;
      if (amdsmi_topo_get_link_weight(h, (amdsmi_processor_handle)handles_[j], &w) == AMDSMI_STATUS_SUCCESS)
        tp.weight = w;
      g.topo.push_back(tp);
    }
    amdsmi_vram_usage_t vu{};
    if (amdsmi_get_gpu_vram_usage(h, &vu) == AMDSMI_STATUS_SUCCESS) {
      g.vram_total_mb = vu.vram_total;
      g.vram_used_mb = vu.vram_used;
    } else {
      g.errors.push_back("vram_usage");
    }
    amdsmi_clk_info_t ci{};
    if (amdsmi_get_clock_info(h, AMDSMI_CLK_TYPE_GFX, &ci) == AMDSMI_STATUS_SUCCESS) {
      g.sclk_cur = ci.clk;
      g.sclk_max = ci.max_clk;
    } else {
      g.errors.push_back("clock_gfx");
    }
    amdsmi_clk_info_t mi{};
    if (amdsmi_get_clock_info(h, AMDSMI_CLK_TYPE_MEM, &mi) == AMDSMI_STATUS_SUCCESS) g.mclk_max = mi.max_clk;
    amdsmi_asic_info_t ai{};
    if (amdsmi_get_gpu_asic_info(h, &ai) == AMDSMI_STATUS_SUCCESS) {
      g.model = ai.market_name;
      g.cus = ai.num_of_compute_units == 0xFFFFFFFFu ? 0 : ai.num_of_compute_units;
    } else {
      g.errors.push_back("asic_info");
    }
    amdsmi_vram_info_t vi{};
    if (amdsmi_get_gpu_vram_info(h, &vi) == AMDSMI_STATUS_SUCCESS) g.hbm_bw_gbps = vi.vram_max_bandwidth;
    else g.errors.push_back("vram_info");
    amdsmi_power_info_t pi{};
    if (amdsmi_get_power_info(h, &pi) == AMDSMI_STATUS_SUCCESS) {
      // ROCm 7.2 reports power_limit in µW on MI355X (1.4e9 for a 1400 W cap) although the
      // header says W; normalise anything implausibly large for watts.
      uint64_t lim = pi.power_limit;
      while (lim > 100000) lim /= 1000;
      g.power_limit_w = (uint32_t)lim;
      g.power_w = pi.current_socket_power ? pi.current_socket_power : pi.average_socket_power;
    } else {
      g.errors.push_back("power_info");
    }
    amdsmi_engine_usage_t eu{};
    if (amdsmi_get_gpu_activity(h, &eu) == AMDSMI_STATUS_SUCCESS) {
      g.gfx_activity = eu.gfx_activity;
      g.umc_activity = eu.umc_activity;
    } else {
      g.errors.push_back("activity");
    }
    amdsmi_error_count_t ec{};
    if (amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS) {
      g.ecc_uncorrectable = ec.uncorrectable_count;
      g.ecc_correctable = ec.correctable_count;
    } else {
      g.errors.push_back("ecc");
    }
    uint32_t numa = 0;
    if (amdsmi_topo_get_numa_node_number(h, &numa) == AMDSMI_STATUS_SUCCESS) g.numa = (int)numa;
    char part[64] = {0};
    if (amdsmi_get_gpu_compute_partition(h, part, sizeof part) == AMDSMI_STATUS_SUCCESS) g.compute_partition = part;
    char mpart[64] = {0};
    if (amdsmi_get_gpu_memory_partition(h, mpart, sizeof mpart) == AMDSMI_STATUS_SUCCESS) g.memory_partition = mpart;
    amdsmi_xgmi_link_status_t xs{};
    if (amdsmi_get_gpu_xgmi_link_status(h, &xs) == AMDSMI_STATUS_SUCCESS) {
      for (uint32_t l = 0; l < xs.total_links && l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
        if (xs.status[l] == AMDSMI_XGMI_LINK_UP) ++g.links_up;
        else if (xs.status[l] == AMDSMI_XGMI_LINK_DOWN) ++g.links_down;
      }
    }
    amdsmi_link_metrics_t lm{};
    if (amdsmi_get_link_metrics(h, &lm) == AMDSMI_STATUS_SUCCESS) {
      for (uint32_t l = 0; l < lm.num_links && l < AMDSMI_MAX_NUM_XGMI_PHYSICAL_LINK; ++l) {
        LinkSample ls;
        ls.peer_bdf = bdf_str(lm.links[l].bdf);
        ls.type = (int)lm.links[l].link_type;
        ls.bit_rate = lm.links[l].bit_rate;
        ls.max_bw = lm.links[l].max_bandwidth;
        ls.read_kb = lm.links[l].read;
        ls.write_kb = lm.links[l].write;
        auto key = std::make_pair(i, (int)l);
        auto it = prev_.find(key);
        if (it != prev_.end()) {
          double dt = g.t - std::get<0>(it->second);
          if (dt > 0) {
            ls.read_kbps = (double)(ls.read_kb - std::min(ls.read_kb, std::get<1>(it->second))) / dt;
            ls.write_kbps = (double)(ls.write_kb - std::min(ls.write_kb, std::get<2>(it->second))) / dt;
            // Gb/s → KB/s per direction
            double cap = (double)ls.max_bw * 1e9 / 8.0 / 1024.0;
            if (cap > 0) ls.load = std::min(1.0, (ls.read_kbps + ls.write_kbps) / (2.0 * cap));
          }
        }
        prev_[key] = std::make_tuple(g.t, ls.read_kb, ls.write_kb);
        g.links.push_back(ls);
      }
    }
    out.push_back(std::move(g));
  }
  return out;
}

// JSON has no NaN/Inf literals
static double finite(double v) { return std::isfinite(v) ? v : 0.0; }

std::string to_json(const std::vector<GpuSample>& s) {
  std::ostringstream o;
  o.precision(17);
  o << "[";
  for (size_t i = 0; i < s.size(); ++i) {
    const GpuSample& g = s[i];
    if (i) o << ",";
    o << "{\"index\":" << g.index << ",\"bdf\":\"" << esc(g.bdf) << "\",\"model\":\"" << esc(g.model)
      << "\",\"uuid\":\"" << esc(g.uuid) << "\",\"hipUuid\":\"" << esc(g.hip_uuid) << "\",\"hipId\":" << g.hip_id
      << ",\"hsaId\":" << g.hsa_id << ",\"drmRender\":" << g.drm_render << ",\"drmCard\":" << g.drm_card
      << ",\"kfdNode\":" << g.kfd_node << ",\"partitionId\":" << g.partition_id
      << ",\"processes\":" << g.processes << ",\"processCUs\":" << g.proc_cus
      << ",\"processVramMB\":" << g.proc_vram_mb << ",\"topo\":[";
    for (size_t k = 0; k < g.topo.size(); ++k) {
      const TopoPeer& t = g.topo[k];
      o << (k ? "," : "") << "{\"peer\":" << t.peer << ",\"type\":" << t.type << ",\"hops\":" << t.hops
        << ",\"weight\":" << t.weight << "}";
    }
    o << "],\"vramTotalMB\":" << g.vram_total_mb << ",\"vramUsedMB\":" << g.vram_used_mb
      << ",\"sclkMHz\":" << g.sclk_cur << ",\"sclkMaxMHz\":" << g.sclk_max << ",\"mclkMaxMHz\":" << g.mclk_max
      << ",\"computeUnits\":" << g.cus << ",\"hbmBandwidthGBps\":" << g.hbm_bw_gbps
      << ",\"powerLimitW\":" << g.power_limit_w << ",\"powerW\":" << g.power_w
      << ",\"gfxActivity\":" << g.gfx_activity << ",\"umcActivity\":" << g.umc_activity
      << ",\"eccUncorrectable\":" << g.ecc_uncorrectable << ",\"eccCorrectable\":" << g.ecc_correctable
      << ",\"numaNode\":" << g.numa << ",\"computePartition\":\"" << esc(g.compute_partition)
      << "\",\"memoryPartition\":\"" << esc(g.memory_partition) << "\",\"xgmiLinksUp\":" << g.links_up
      << ",\"xgmiLinksDown\":" << g.links_down << ",\"time\":" << finite(g.t) << ",\"links\":[";
    for (size_t l = 0; l < g.links.size(); ++l) {
      const LinkSample& x = g.links[l];
      if (l) o << ",";
      o << "{\"peerBdf\":\"" << esc(x.peer_bdf) << "\",\"type\":" << x.type << ",\"bitRateGbps\":" << x.bit_rate
        << ",\"maxBandwidthGbps\":" << x.max_bw << ",\"readKB\":" << x.read_kb << ",\"writeKB\":" << x.write_kb
        << ",\"readKBps\":" << finite(x.read_kbps) << ",\"writeKBps\":" << finite(x.write_kbps)
        << ",\"load\":" << finite(x.load) << "}";
    }
    o << "],\"errors\":[";
    for (size_t e = 0; e < g.errors.size(); ++e) o << (e ? "," : "") << "\"" << esc(g.errors[e]) << "\"";
    o << "]}";
  }
  o << "]";
  return o.str();
}

}  // namespace yoda
