"""``Scv`` node-telemetry CRD (``scvs.core.run-linux.com/v1``), wire-compatible.

The reference consumes ``github.com/NJUPT-ISL/SCV/api/v1`` (``go.mod:6``); only the
fields it touches are load-bearing: ``Status.CardNumber``,
``CardList``, ``FreeMemorySum``, ``TotalMemorySum`` and per card ``Health``,
``FreeMemory``, ``TotalMemory``, ``Clock``, ``Bandwidth``, ``Core``, ``Power``.
Field names live in ONE place (``_CARD_FIELDS`` / ``_STATUS_FIELDS``) so the CRD
schema, the sniffer publisher and the scheduler cache agree.

MI355X additions are an additive ``status.amd`` block: per-GPU physical id, PCI BDF,
identity (amd-smi UUID, HIP/ROCr UUID and ordinal, render node, partition id), NUMA
node, compute/memory partition, CU occupancy + GFX activity, tenant process count, sclk
and per-peer xGMI link load, plus the sample timestamp used for staleness-based health.
"""
from __future__ import annotations

import datetime as _dt
import time
from dataclasses import dataclass, field
from collections.abc import Sequence
from typing import Any

GROUP = "core.run-linux.com"
VERSION = "v1"
API_VERSION = f"{GROUP}/{VERSION}"
KIND = "Scv"
PLURAL = "scvs"
HEALTHY = "Healthy"

_CARD_FIELDS = {
    # python attr : json key
    "id": "id",
    "health": "health",
    "model": "model",
    "power": "power",
    "total_memory": "totalMemory",
    "clock": "clock",
    "free_memory": "freeMemory",
    "core": "core",
    "bandwidth": "bandwidth",
}

_STR_FIELDS = frozenset(("health", "model"))

_AMD_CARD_FIELDS = {
    "physical_id": "physicalId",
    "bdf": "bdf",
    "numa_node": "numaNode",
    "compute_partition": "computePartition",
    "memory_partition": "memoryPartition",
    "cu_occupancy": "cuOccupancy",
    "gfx_activity": "gfxActivity",
    "occupancy_source": "occupancySource",
    "sclk_mhz": "sclkMhz",
    "ecc_uncorrectable": "eccUncorrectable",
    "xgmi_links_up": "xgmiLinksUp",
    # identity (amd-smi index = BDF order ≠ HIP/ROCr order in general; UUIDs are stable)
    "uuid": "uuid",
    "hip_uuid": "hipUuid",
    "hip_id": "hipId",
    "render_node": "renderNode",
    "partition_id": "partitionId",
    "processes": "processes",
}


@dataclass
class XgmiLink:
    peer: int                 # physical id of the peer GPU
    load: float = 0.0         # 0..1 utilisation estimated from counter deltas
    read_kbps: float = 0.0
    write_kbps: float = 0.0
    max_bandwidth_gbps: float = 0.0
    up: bool = True

    def to_json(self) -> dict:
        return {"peer": self.peer, "load": round(self.load, 6), "readKBps": self.read_kbps,
                "writeKBps": self.write_kbps, "maxBandwidthGBps": self.max_bandwidth_gbps,
                "up": self.up}

    @classmethod
    def from_json(cls, d: dict) -> "XgmiLink":
        return cls(peer=int(d.get("peer", 0)), load=float(d.get("load", 0.0)),
                   read_kbps=float(d.get("readKBps", 0.0)), write_kbps=float(d.get("writeKBps", 0.0)),
                   max_bandwidth_gbps=float(d.get("maxBandwidthGBps", 0.0)), up=bool(d.get("up", True)))


class LazyLinks(Sequence):
    """A card's ``status.amd.cards[i].xgmi`` as decoded JSON, turned into ``XgmiLink``
    objects only when something iterates it: the scheduler's hot path (``link_matrix``)
    reads the raw dicts (``raw``), so an Scv update does not build 56 objects per node."""
    __slots__ = ("raw", "_links")

    def __init__(self, raw: list) -> None:
        self.raw = raw
        self._links: list | None = None

    def _get(self) -> list:
        if self._links is None:
            self._links = [XgmiLink.from_json(l) for l in self.raw]
        return self._links

    def __getitem__(self, i):
        return self._get()[i]

    def __len__(self) -> int:
        return len(self.raw)

    def __iter__(self):
        return iter(self._get())

    def __eq__(self, other) -> bool:
        return list(self) == list(other)


@dataclass
class Card:
    id: int = 0
    health: str = HEALTHY
    model: str = ""
    power: int = 0            # W
    total_memory: int = 0     # MB
    clock: int = 0            # MHz
    free_memory: int = 0      # MB
    core: int = 0             # compute units
    bandwidth: int = 0        # GB/s (HBM)
    # --- amd extension (status.amd.cards[i]) ---
    physical_id: int | None = None
    bdf: str = ""
    numa_node: int = 0
    compute_partition: str = "SPX"
    memory_partition: str = "NPS1"
    # CU occupancy %: Σ per-process CUs held (amd-smi process list) / CUs when the driver
    # reports it ("process-cus"), else the GFX-engine busy % as a proxy ("gfx-activity")
    cu_occupancy: float = 0.0
    gfx_activity: float = 0.0   # 0..100 GFX engine busy %
    occupancy_source: str = "gfx-activity"
    sclk_mhz: int = 0           # current sclk
    ecc_uncorrectable: int = 0
    xgmi_links_up: bool = True
    xgmi: list[XgmiLink] = field(default_factory=list)
    uuid: str = ""              # amd-smi device UUID
    hip_uuid: str = ""          # HIP/ROCr UUID ("GPU-…", accepted by ROCR_VISIBLE_DEVICES)
    hip_id: int = -1            # HIP ordinal on the node (-1: unknown)
    render_node: int = -1       # /dev/dri/renderD<n>
    partition_id: int = -1      # compute partition of a CPX/DPX/QPX logical GPU
    processes: int = -1         # processes with a context on the GPU (-1: unknown)

    @property
    def phys(self) -> int:
        return self.id if self.physical_id is None else self.physical_id

    def base_json(self) -> dict:
        return {j: getattr(self, a) for a, j in _CARD_FIELDS.items()}

    def amd_json(self) -> dict:
        d = {j: getattr(self, a) for a, j in _AMD_CARD_FIELDS.items()}
        d["physicalId"] = self.phys
        d["id"] = self.id
        d["xgmi"] = [l.to_json() for l in self.xgmi]
        return d


@dataclass
class ScvStatus:
    card_list: list[Card] = field(default_factory=list)
    total_memory_sum: int = 0
    free_memory_sum: int = 0
    card_number: int = 0
    update_time: float | None = None     # unix seconds (serialised RFC3339)
    sniffer: str = ""                    # producer id (amd-smi / fake / nvml)

    def recompute_sums(self) -> None:
        self.card_number = len(self.card_list)
        self.total_memory_sum = sum(c.total_memory for c in self.card_list)
        self.free_memory_sum = sum(c.free_memory for c in self.card_list)


@dataclass
class Scv:
    name: str
    status: ScvStatus = field(default_factory=ScvStatus)
    update_interval_ms: int = 1000
    resource_version: str = ""
    labels: dict = field(default_factory=dict)

    # ------------------------------------------------------------------ JSON
    def to_json(self) -> dict:
        st = self.status
        status: dict[str, Any] = {
            "cardList": [c.base_json() for c in st.card_list],
            "totalMemorySum": st.total_memory_sum,
            "freeMemorySum": st.free_memory_sum,
            "cardNumber": st.card_number,
        }
        if st.update_time is not None:
            status["updateTime"] = rfc3339(st.update_time)
        status["amd"] = {
            "sniffer": st.sniffer,
            "cards": [c.amd_json() for c in st.card_list],
        }
        meta: dict[str, Any] = {"name": self.name}
        if self.resource_version:
            meta["resourceVersion"] = self.resource_version
        if self.labels:
            meta["labels"] = dict(self.labels)
        return {"apiVersion": API_VERSION, "kind": KIND, "metadata": meta,
                "spec": {"updateInterval": self.update_interval_ms}, "status": status}

    @classmethod
    def from_json(cls, obj: dict) -> "Scv":
        meta = obj.get("metadata") or {}
        status = obj.get("status") or {}
        amd = status.get("amd") or {}
        amd_cards = {int(c.get("id", i)): c for i, c in enumerate(amd.get("cards") or [])}
        cards: list[Card] = []
        for i, cj in enumerate(status.get("cardList") or []):
            # one constructor call per card (telemetry updates are the scheduler's most
            # frequent event: ≈100/s per 1000 nodes)
            kw = {a: (v if a in _STR_FIELDS else int(v)) for a, j in _CARD_FIELDS.items()
                  if (v := cj.get(j)) is not None}
            ext = amd_cards.get(kw.get("id", 0)) or amd_cards.get(i)
            if ext:
                for a, j in _AMD_CARD_FIELDS.items():
                    v = ext.get(j)
                    if v is not None:
                        kw[a] = v
                if "gfxActivity" not in ext and "cuOccupancy" in ext:      # pre-r2 producers
                    kw["gfx_activity"] = float(ext["cuOccupancy"])
                kw["physical_id"] = int(ext.get("physicalId", kw.get("id", 0)))
                kw["xgmi"] = LazyLinks(ext.get("xgmi") or [])
            cards.append(Card(**kw))
        st = ScvStatus(
            card_list=cards,
            total_memory_sum=int(status.get("totalMemorySum", 0) or 0),
            free_memory_sum=int(status.get("freeMemorySum", 0) or 0),
            card_number=int(status.get("cardNumber", 0) or 0),
            update_time=parse_rfc3339(status.get("updateTime")),
            sniffer=str(amd.get("sniffer", "")),
        )
        spec = obj.get("spec") or {}
        return cls(name=meta.get("name", ""), status=st,
                   update_interval_ms=int(spec.get("updateInterval", 1000) or 1000),
                   resource_version=str(meta.get("resourceVersion", "")),
                   labels=dict(meta.get("labels") or {}))

    def is_stale(self, now: float | None = None, factor: float = 3.0) -> bool:
        """Fresh iff sampled within ``factor`` × update interval (SURVEY §5 health)."""
        t = self.status.update_time
        if t is None:
            return False   # producers that do not stamp (reference SCV) are never stale
        now = time.time() if now is None else now
        return (now - t) * 1000.0 > factor * max(self.update_interval_ms, 1)


def card_vis(ids: list) -> list:
    """Per card position of ``(id, amd-smi UUID, ROCr UUID, HIP ordinal)`` identities: the
    ROCr-visible id (ROCr UUID, else HIP ordinal, else the amd-smi index) and the UUID."""
    return [(c[2] if c[2] else (str(c[3]) if c[3] >= 0 else str(c[0])), c[1]) for c in ids]


class LazyScv:
    """An ``Scv`` as the informer delivered it (decoded JSON), turned into the dataclass
    tree only when something reads it. The scheduler's per-update path needs neither: the
    engine view (``engine_view``: card tuples, sums, link matrix — computed straight from the
    dict by ``ops.native.scv_engine_view``) and the freshness fields are kept here. A 1000-node
    cluster sends ≈100 Scv updates/s, most of which are never read by anything else."""
    __slots__ = ("name", "update_time", "update_interval_ms", "card_number", "engine_view", "_obj", "_scv",
                 "_idents", "_vis", "ann_memo")

    def __init__(self, obj: dict, engine_view, idents: list | None = None) -> None:
        meta = obj.get("metadata") or {}
        status = obj.get("status") or {}
        spec = obj.get("spec") or {}
        self.name = meta.get("name", "")
        self.update_time = parse_rfc3339(status.get("updateTime"))
        self.update_interval_ms = int(spec.get("updateInterval", 1000) or 1000)
        self.card_number = int(status.get("cardNumber", 0) or 0)
        self.engine_view = engine_view
        self._obj = obj
        self._scv = None
        self._idents = idents
        self._vis = card_vis(idents) if idents is not None else None   # at ingest, off the bind path
        self.ann_memo: dict = {}       # the scheduler's Binding annotations per (GPU set, HBM)

    def card_vis(self) -> list:
        """Per card position: (ROCr-visible id, amd-smi UUID) as the Binding annotations spell
        them (``card_vis``), computed once per Scv version."""
        if self._vis is None:
            self._vis = card_vis(self.card_idents())
        return self._vis

    def card_idents(self) -> list:
        """Per card position: (id, amd-smi UUID, HIP/ROCr UUID, HIP ordinal) — what a Binding's
        device annotations need — read from the JSON (same matching and defaults as
        ``Scv.from_json``) without decoding the rest."""
        if self._scv is not None:
            return [(c.id, c.uuid, c.hip_uuid, c.hip_id) for c in self._scv.status.card_list]
        if self._idents is None:
            status = self._obj.get("status") or {}
            amd = status.get("amd") or {}
            amd_cards = {int(c.get("id", i)): c for i, c in enumerate(amd.get("cards") or [])}
            out = []
            for i, cj in enumerate(status.get("cardList") or []):
                cid = int(cj["id"]) if cj.get("id") is not None else 0
                ext = amd_cards.get(cid) or amd_cards.get(i) or {}
                u, hu, hid = ext.get("uuid"), ext.get("hipUuid"), ext.get("hipId")
                out.append((cid, u if u is not None else "", hu if hu is not None else "",
                            hid if hid is not None else -1))
            self._idents = out
        return self._idents

    def decoded(self) -> "Scv":
        if self._scv is None:
            self._scv = Scv.from_json(self._obj)
        return self._scv

    def __getattr__(self, attr):       # status, labels, resource_version, to_json, ...
        return getattr(self.decoded(), attr)

    def is_stale(self, now: float | None = None, factor: float = 3.0) -> bool:
        t = self.update_time
        if t is None:
            return False
        now = time.time() if now is None else now
        return (now - t) * 1000.0 > factor * max(self.update_interval_ms, 1)


_rfc_sec = [-1, ""]


def rfc3339(t: float) -> str:
    """RFC 3339 with microseconds (k8s MicroTime). The whole-second prefix is cached:
    bursts stamp thousands of objects within the same second."""
    sec = int(t)
    if sec != _rfc_sec[0]:
        _rfc_sec[0], _rfc_sec[1] = sec, time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(sec))
    return f"{_rfc_sec[1]}.{int((t - sec) * 1e6):06d}Z"


def parse_rfc3339(s: Any) -> float | None:
    if s is None or s == "":
        return None
    if isinstance(s, (int, float)):
        return float(s)
    s = str(s)
    try:   # C fast path (py3.10 fromisoformat needs an explicit offset)
        return _dt.datetime.fromisoformat(s[:-1] + "+00:00" if s.endswith("Z") else s).timestamp()
    except ValueError:
        pass
    import calendar
    base, frac = s.rstrip("Z"), 0.0
    if "." in base:
        base, f = base.split(".", 1)
        frac = float("0." + f) if f else 0.0
    return calendar.timegm(time.strptime(base, "%Y-%m-%dT%H:%M:%S")) + frac


def crd_manifest() -> dict:
    """CustomResourceDefinition for scvs.core.run-linux.com (cluster-scoped, status subresource)."""
    int_t = {"type": "integer", "format": "int64", "minimum": 0}
    card_props = {j: ({"type": "string"} if a in ("health", "model") else dict(int_t))
                  for a, j in _CARD_FIELDS.items()}
    schema = {
        "type": "object",
        "properties": {
            "spec": {"type": "object", "properties": {"updateInterval": {"type": "integer"}}},
            "status": {
                "type": "object",
                "properties": {
                    "cardList": {"type": "array", "items": {"type": "object", "properties": card_props}},
                    "totalMemorySum": dict(int_t),
                    "freeMemorySum": dict(int_t),
                    "cardNumber": dict(int_t),
                    "updateTime": {"type": "string", "format": "date-time"},
                    "amd": {"type": "object", "x-kubernetes-preserve-unknown-fields": True},
                },
            },
        },
    }
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{PLURAL}.{GROUP}"},
        "spec": {
            "group": GROUP,
            "scope": "Cluster",
            "names": {"plural": PLURAL, "singular": "scv", "kind": KIND, "listKind": "ScvList"},
            "versions": [{"name": VERSION, "served": True, "storage": True,
                          "subresources": {"status": {}},
                          "schema": {"openAPIV3Schema": schema}}],
        },
    }
