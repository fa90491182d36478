"""Telemetry backends for the Scv sniffer and the sample → ``Scv`` mapping.

* :class:`AmdSmiBackend` — the C++ amd-smi collector (``native/sniffer``), the MI355X
  replacement of the reference's external NVML sniffer.
* :class:`FakeBackend` — synthetic MI355X node with fault injection (ECC errors, xGMI
  link down, HBM pressure, busy CUs) for CPU tests and benches.

Field mapping: ``totalMemory``=vram_total, ``freeMemory``=total −
used, ``clock``=GFX max sclk, ``core``=compute units, ``bandwidth``=HBM GB/s (measured
by the HIP probe when available, else amd-smi's max bandwidth), ``power``=power limit,
``health``="Healthy" iff no uncorrectable ECC, no xGMI link down and the HBM pattern
probe (if run) found no errors.
"""
from __future__ import annotations

import importlib
import json
import random
import time
from dataclasses import dataclass, field
from typing import Optional

from ..models.device import MI355X, GpuSpec, numa_of
from ..models.scv import HEALTHY, Card, Scv, ScvStatus, XgmiLink

UNHEALTHY = "Unhealthy"


class AmdSmiBackend:
    name = "amd-smi"

    def __init__(self) -> None:
        from ..ops.native import load_native
        mod = load_native("sniffer", "yoda_scheduler_amd._native._yoda_sniffer")
        self._c = mod.Collector()
        ok, err = self._c.init()
        if not ok:
            raise RuntimeError(f"amd-smi unavailable: {err}")

    @property
    def count(self) -> int:
        return self._c.count

    def sample(self) -> list[dict]:
        return json.loads(self._c.sample_json())

    def close(self) -> None:
        self._c.shutdown()


@dataclass
class FakeGpuState:
    used_mb: int = 0
    gfx_activity: int = 0
    ecc_uncorrectable: int = 0
    links_down: int = 0
    link_load: dict = field(default_factory=dict)   # peer index → load 0..1


class FakeBackend:
    """Synthetic amd-smi samples for an MI355X node (same JSON shape as the C++ collector)."""
    name = "fake"

    def __init__(self, gpus: int = 8, spec: GpuSpec = MI355X, partition: str = "SPX", seed: int = 0,
                 hip_order: Optional[list[int]] = None, partitions_per_gpu: int = 1, node: str = "node") -> None:
        """``hip_order[i]``: HIP ordinal of amd-smi index ``i`` (a permutation, as when the
        KFD enumerates GPUs in another order than PCI address); ``partitions_per_gpu`` > 1
        models CPX/DPX/QPX: ``gpus`` logical GPUs, consecutive ones sharing a physical BDF."""
        self.spec = spec
        self.gpus = gpus
        self.partition = partition
        self.ppg = max(1, partitions_per_gpu)
        self.hip_order = list(hip_order) if hip_order is not None else list(range(gpus))
        if sorted(self.hip_order) != list(range(gpus)):
            raise ValueError("hip_order must be a permutation of range(gpus)")
        self.node = node
        self.tenants: dict[int, tuple[int, int]] = {}     # index → (processes, CUs held)
        self.state = [FakeGpuState() for _ in range(gpus)]
        self.rng = random.Random(seed)
        self._counters = [[[0, 0] for _ in range(gpus)] for _ in range(gpus)]
        self._last_t = time.time()

    @property
    def count(self) -> int:
        return self.gpus

    def sample(self) -> list[dict]:
        t = time.time()
        dt = max(t - self._last_t, 1e-3)
        self._last_t = t
        out = []
        cap_kbps = self.spec.xgmi_link_gbps * 8 * 1e9 / 8 / 1024   # GB/s → KB/s per direction
        for i, st in enumerate(self.state):
            links = []
            for j in range(self.gpus):
                if j == i:
                    continue
                load = st.link_load.get(j, 0.0)
                rate = load * cap_kbps
                self._counters[i][j][0] += int(rate * dt)
                self._counters[i][j][1] += int(rate * dt)
                if self.ppg > 1 and j // self.ppg == i // self.ppg:
                    continue              # partitions of one GPU share its links
                links.append({"peerBdf": self._bdf(j), "type": 2, "bitRateGbps": 32,
                              "maxBandwidthGbps": int(self.spec.xgmi_link_gbps * 8),
                              "readKB": self._counters[i][j][0], "writeKB": self._counters[i][j][1],
                              "readKBps": rate, "writeKBps": rate, "load": load})
            procs, cus = self.tenants.get(i, (0, 0))
            hid = self.hip_order[i]
            out.append({
                "index": i, "bdf": self._bdf(i), "model": self.spec.model,
                "uuid": self.uuid(i), "hipUuid": f"GPU-{self.uuid(i)[-16:]}", "hipId": hid, "hsaId": hid + 1,
                "drmRender": 128 + hid, "drmCard": hid + 1, "kfdNode": hid + 1,
                "partitionId": i % self.ppg if self.ppg > 1 else -1,
                "processes": procs, "processCUs": cus, "processVramMB": st.used_mb if procs else 0,
                "topo": [{"peer": j, "type": 2, "hops": 1, "weight": 15} for j in range(self.gpus) if j != i],
                "vramTotalMB": self.spec.hbm_mb, "vramUsedMB": st.used_mb,
                "sclkMHz": self.spec.max_sclk_mhz if st.gfx_activity else 150, "sclkMaxMHz": self.spec.max_sclk_mhz,
                "mclkMaxMHz": 2000, "computeUnits": self.spec.cus, "hbmBandwidthGBps": self.spec.hbm_bw_gbps,
                "powerLimitW": self.spec.power_w, "powerW": 200 + 10 * st.gfx_activity,
                "gfxActivity": st.gfx_activity, "umcActivity": 0,
                "eccUncorrectable": st.ecc_uncorrectable, "eccCorrectable": 0,
                "numaNode": numa_of(i, self.gpus), "computePartition": self.partition, "memoryPartition": "NPS1",
                "xgmiLinksUp": self.gpus - 1 - st.links_down, "xgmiLinksDown": st.links_down,
                "time": t, "links": links, "errors": [],
            })
        return out

    def close(self) -> None:
        return None

    def _bdf(self, i: int) -> str:
        return _bdf(i // self.ppg, i % self.ppg)

    def uuid(self, i: int) -> str:
        """Stable per logical GPU (node name, physical slot, partition)."""
        import hashlib
        h = hashlib.sha1(f"{self.node}/{i // self.ppg}/{i % self.ppg}".encode()).hexdigest()
        return f"{h[:8]}-{h[8:12]}-{h[12:16]}-{h[16:20]}-{h[20:32]}"


def _bdf(i: int, fn: int = 0) -> str:
    return f"0000:{0x05 + 0x10 * i:02x}:00.{fn}"


def _phys_key(bdf: str) -> str:
    """Partitions of one physical GPU differ only in the PCI function number."""
    return bdf.rsplit(".", 1)[0] if bdf else bdf


def samples_to_scv(node: str, samples: list[dict], interval_ms: int = 1000, measured_bw: Optional[dict] = None,
                   probe_errors: Optional[dict] = None, sniffer: str = "amd-smi") -> Scv:
    """Map one collector sample of every GPU on ``node`` to an ``Scv`` object."""
    phys_ids: dict[str, int] = {}
    for s in samples:
        phys_ids.setdefault(_phys_key(s.get("bdf", "")), len(phys_ids))
    bdf_to_phys = {_phys_key(s.get("bdf", "")): phys_ids[_phys_key(s.get("bdf", ""))] for s in samples}
    cards = []
    for s in samples:
        i = int(s["index"])
        total = int(s.get("vramTotalMB", 0))
        used = min(int(s.get("vramUsedMB", 0)), total)
        perr = (probe_errors or {}).get(i, 0)
        healthy = int(s.get("eccUncorrectable", 0)) == 0 and int(s.get("xgmiLinksDown", 0)) == 0 and perr == 0
        phys = phys_ids[_phys_key(s.get("bdf", ""))]
        links = []
        for l in s.get("links") or []:
            if int(l.get("type", 2)) != 2:
                continue
            peer = bdf_to_phys.get(_phys_key(l.get("peerBdf", "")))
            if peer is None or peer == phys:
                continue
            links.append(XgmiLink(peer=peer, load=float(l.get("load", 0.0)), read_kbps=float(l.get("readKBps", 0.0)),
                                  write_kbps=float(l.get("writeKBps", 0.0)),
                                  max_bandwidth_gbps=float(l.get("maxBandwidthGbps", 0)) / 8.0,
                                  up=int(l.get("bitRateGbps", 1)) > 0))
        bw = int((measured_bw or {}).get(i, s.get("hbmBandwidthGBps", 0)) or 0)
        cus = int(s.get("computeUnits", 0))
        procs = int(s.get("processes", -1))
        if procs >= 0 and cus > 0:
            occ, occ_src = min(100.0, 100.0 * int(s.get("processCUs", 0)) / cus), "process-cus"
        else:
            occ, occ_src = float(s.get("gfxActivity", 0)), "gfx-activity"
        cards.append(Card(
            id=i, health=HEALTHY if healthy else UNHEALTHY, model=s.get("model", ""),
            power=int(s.get("powerLimitW", 0)), total_memory=total, clock=int(s.get("sclkMaxMHz", 0)),
            free_memory=total - used, core=int(s.get("computeUnits", 0)), bandwidth=bw,
            physical_id=phys, bdf=s.get("bdf", ""), numa_node=max(int(s.get("numaNode", 0)), 0),
            compute_partition=s.get("computePartition") or "SPX", memory_partition=s.get("memoryPartition") or "NPS1",
            cu_occupancy=occ, gfx_activity=float(s.get("gfxActivity", 0)), occupancy_source=occ_src,
            sclk_mhz=int(s.get("sclkMHz", 0)),
            ecc_uncorrectable=int(s.get("eccUncorrectable", 0)), xgmi_links_up=int(s.get("xgmiLinksDown", 0)) == 0,
            xgmi=links, uuid=str(s.get("uuid", "")), hip_uuid=str(s.get("hipUuid", "")),
            hip_id=int(s.get("hipId", -1)), render_node=int(s.get("drmRender", -1)),
            partition_id=int(s.get("partitionId", -1)), processes=procs))
    st = ScvStatus(card_list=cards, update_time=max((float(s.get("time", 0)) for s in samples), default=time.time()),
                   sniffer=sniffer)
    st.recompute_sums()
    return Scv(name=node, status=st, update_interval_ms=interval_ms)
