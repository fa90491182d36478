"""MI355X device / node model used by the fake amd-smi backend, benches and tests.

An MI355X node is 8 GPUs in a full xGMI mesh: every GPU has 7 point-to-point links
(≈153 GB/s each), so every pair is one hop and "locality" means *idle links*, not hop
count (distributed comm backend row). Partition modes (CPX/DPX/QPX) expose
several logical GPUs per physical GPU; logical GPUs of one physical device share its
links and its HBM stack.
"""
from __future__ import annotations

import random
from dataclasses import dataclass

from .scv import HEALTHY, Card, Scv, ScvStatus, XgmiLink


@dataclass(frozen=True)
class GpuSpec:
    model: str
    hbm_mb: int
    max_sclk_mhz: int
    cus: int
    power_w: int
    hbm_bw_gbps: int
    xgmi_link_gbps: float
    xgmi_links: int


MI355X = GpuSpec("AMD Instinct MI355X", 288 * 1024, 2400, 256, 1400, 8000, 153.6, 7)
MI350X = GpuSpec("AMD Instinct MI350X", 288 * 1024, 2200, 256, 1000, 8000, 153.6, 7)

PARTITION_FACTOR = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}


def numa_of(phys_id: int, gpus_per_node: int) -> int:
    """Typical 2-socket host: first half of the GPUs on socket 0."""
    return 0 if gpus_per_node <= 1 else int(phys_id >= (gpus_per_node + 1) // 2)


def make_cards(spec: GpuSpec = MI355X, gpus: int = 8, partition: str = "SPX",
               used_mb: list[int] | None = None, link_load: float = 0.0,
               occupancy: float = 0.0, rng: random.Random | None = None,
               jitter: bool = False) -> list[Card]:
    """Synthetic SCV card list for one node (logical GPUs in partition order)."""
    f = PARTITION_FACTOR[partition]
    cards: list[Card] = []
    for p in range(gpus):
        for s in range(f):
            i = p * f + s
            total = spec.hbm_mb // f
            used = (used_mb[i] if used_mb and i < len(used_mb) else 0)
            if jitter and rng is not None:
                used += rng.randint(0, 512)
            links = [XgmiLink(peer=q, load=(rng.random() * link_load if (jitter and rng) else link_load),
                              max_bandwidth_gbps=spec.xgmi_link_gbps)
                     for q in range(gpus) if q != p]
            cards.append(Card(
                id=i, health=HEALTHY, model=spec.model, power=spec.power_w,
                total_memory=total, clock=spec.max_sclk_mhz, free_memory=max(total - used, 0),
                core=spec.cus // f, bandwidth=spec.hbm_bw_gbps // f,
                physical_id=p, bdf=f"0000:{0x05 + 0x10 * p:02x}:00.{s}", numa_node=numa_of(p, gpus),
                compute_partition=partition, memory_partition="NPS1",
                cu_occupancy=occupancy, sclk_mhz=spec.max_sclk_mhz, xgmi=links))
    return cards


def make_scv(node: str, spec: GpuSpec = MI355X, gpus: int = 8, partition: str = "SPX",
             update_time: float | None = None, sniffer: str = "fake", **kw) -> Scv:
    st = ScvStatus(card_list=make_cards(spec, gpus, partition, **kw), update_time=update_time,
                   sniffer=sniffer)
    st.recompute_sums()
    return Scv(name=node, status=st)


def make_node(name: str, cpu: str = "192", memory: str = "2Ti", pods: int = 1100,
              labels: dict | None = None, taints: list | None = None,
              unschedulable: bool = False) -> dict:
    """A minimal v1.Node object as the apiserver would return it."""
    lab = {"kubernetes.io/hostname": name, "kubernetes.io/os": "linux"}
    lab.update(labels or {})
    return {
        "apiVersion": "v1", "kind": "Node",
        "metadata": {"name": name, "labels": lab},
        "spec": {"unschedulable": unschedulable, "taints": list(taints or [])},
        "status": {"allocatable": {"cpu": cpu, "memory": memory, "pods": str(pods)},
                   "capacity": {"cpu": cpu, "memory": memory, "pods": str(pods)},
                   "conditions": [{"type": "Ready", "status": "True"}]},
    }
