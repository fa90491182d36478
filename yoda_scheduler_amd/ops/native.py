"""Loader + marshalling for the native scheduling engine (``_yoda_core``).

The engine is mandatory: there is no silent Python fallback on the hot path. If the
extension is missing it is built in-tree on first import (hipcc/g++ are in the image);
if that fails the import raises.
"""
from __future__ import annotations

import importlib
import threading
import weakref

from ..models.pod import PF_CLAIMS, NodeInfo, PodInfo
from ..models.scv import HEALTHY, LazyLinks, LazyScv, Scv

_lock = threading.Lock()
_core = None


def core():
    """Return the ``_yoda_core`` extension module, building it in-tree if needed."""
    global _core
    if _core is not None:
        return _core
    with _lock:
        if _core is None:
            _core = load_native("core", "yoda_scheduler_amd._native._yoda_core")
    return _core


def load_native(name: str, module: str):
    """Import a pybind artefact after making sure it was built from this tree's sources
    (rebuilt in-tree if its recorded build id is stale), then check the id compiled into
    the module actually loaded (``ops/build.py``: build provenance)."""
    from . import build
    build.ensure_fresh(name)
    importlib.invalidate_caches()
    mod = importlib.import_module(module)
    bid = getattr(mod, "build_id", None)
    if (build.NATIVE / "common" / "build_id.h").exists():
        build.verify_loaded(name, bid() if bid is not None else "")
    return mod


def card_tuples(scv: Scv) -> list[tuple]:
    out = []
    for c in scv.status.card_list:
        out.append((int(c.total_memory) & 0xFFFFFFFFFFFFFFFF, int(c.free_memory) & 0xFFFFFFFFFFFFFFFF,
                    int(c.clock) & 0xFFFFFFFFFFFFFFFF, int(c.bandwidth) & 0xFFFFFFFFFFFFFFFF,
                    int(c.core) & 0xFFFFFFFFFFFFFFFF, int(c.power) & 0xFFFFFFFFFFFFFFFF,
                    c.health == HEALTHY and c.ecc_uncorrectable == 0 and c.xgmi_links_up,
                    int(c.phys), int(c.numa_node), int(round(float(c.cu_occupancy) * 100))))
    return out


def compat_card_tuples(scv: Scv) -> list[tuple]:
    """Reference semantics: health is exactly ``Health == "Healthy"``."""
    return [t[:6] + (c.health == HEALTHY,) + t[7:] for t, c in zip(card_tuples(scv), scv.status.card_list)]


# Quality of an idle xGMI link relative to two partitions of the same physical GPU (1e-4
# units; same physical GPU = 10000 in the engine and the device rows). One xGMI link is
# ≈153 GB/s while partitions of one MI355X talk over the on-package fabric, so on
# partitioned (DPX/QPX/CPX) nodes a gang prefers partitions of fewer physical GPUs. On SPX
# nodes every pair crosses xGMI, so this only shifts all subsets' link term equally.
XGMI_IDLE_QUALITY = 9000


def link_matrix(scv: Scv) -> tuple[int, list[int]]:
    """Pair quality in 1e-4 units between physical GPUs: ``XGMI_IDLE_QUALITY × (1 − load)``
    for an up link (idle when unreported), 0 for a down one."""
    cards = scv.status.card_list
    nphys = max((c.phys for c in cards), default=-1) + 1
    q = [XGMI_IDLE_QUALITY] * (nphys * nphys)
    for a in range(nphys):
        q[a * nphys + a] = 10000
    for c in cards:
        row = c.phys * nphys
        links = c.xgmi
        if isinstance(links, LazyLinks):      # decoded JSON: read the dicts, build no objects
            for d in links.raw:
                peer = int(d.get("peer", 0))
                if 0 <= peer < nphys:
                    load = float(d.get("load", 0.0))
                    q[row + peer] = 0 if not d.get("up", True) else \
                        int(round(XGMI_IDLE_QUALITY * (1.0 - (0.0 if load < 0.0 else 1.0 if load > 1.0 else load))))
        else:
            for l in links:
                if 0 <= l.peer < nphys:
                    v = 0 if not l.up else int(round(XGMI_IDLE_QUALITY * (1.0 - min(max(l.load, 0.0), 1.0))))
                    q[row + l.peer] = v
    # symmetrise with the worse direction (a ring uses both)
    for a in range(nphys):
        ra = a * nphys
        for b in range(a + 1, nphys):
            x, y = q[ra + b], q[b * nphys + a]
            q[ra + b] = q[b * nphys + a] = x if x < y else y
    return nphys, q


_M64 = 0xFFFFFFFFFFFFFFFF


def scv_engine_view(obj: dict, compat: bool, idents: list | None = None) -> tuple:
    """What ``push_scv`` sends the engine for an Scv given as decoded JSON — the card tuples
    (``card_tuples`` / ``compat_card_tuples``), CardNumber / memory sums, sample time and the
    link matrix (``link_matrix``) — computed from the dict without building the dataclasses
    (same field defaults and conversions as ``Scv.from_json``; equivalence pinned by
    ``tests/test_control_plane.py::test_scv_engine_view_matches_dataclass_path``). With
    ``idents`` the same pass appends each card's (id, amd-smi UUID, ROCr UUID, HIP ordinal)
    (``LazyScv.card_idents``): the Binding annotations then never walk the JSON again."""
    status = obj.get("status") or {}
    amd = status.get("amd") or {}
    amd_cards = {int(c.get("id", i)): c for i, c in enumerate(amd.get("cards") or [])}
    cards, raw_links = [], []
    for i, cj in enumerate(status.get("cardList") or []):
        g = cj.get
        cid = int(g("id")) if g("id") is not None else 0
        ext = amd_cards.get(cid) or amd_cards.get(i)
        v = g("health")
        health = v if v is not None else HEALTHY
        num = [int(g(k)) if g(k) is not None else 0
               for k in ("totalMemory", "freeMemory", "clock", "bandwidth", "core", "power")]
        if idents is not None:
            x = ext or {}
            u, hu, hid = x.get("uuid"), x.get("hipUuid"), x.get("hipId")
            idents.append((cid, u if u is not None else "", hu if hu is not None else "", hid if hid is not None else -1))
        if ext:
            e = ext.get
            phys = int(ext.get("physicalId", cid))
            numa = e("numaNode") if e("numaNode") is not None else 0
            occ = e("cuOccupancy") if e("cuOccupancy") is not None else 0.0
            ecc = e("eccUncorrectable") if e("eccUncorrectable") is not None else 0
            up = e("xgmiLinksUp") if e("xgmiLinksUp") is not None else True
            raw_links.append((phys, ext.get("xgmi") or []))
        else:
            phys, numa, occ, ecc, up = cid, 0, 0.0, 0, True
            raw_links.append((phys, []))
        healthy = health == HEALTHY if compat else (health == HEALTHY and ecc == 0 and bool(up))
        cards.append((num[0] & _M64, num[1] & _M64, num[2] & _M64, num[3] & _M64, num[4] & _M64, num[5] & _M64,
                      healthy, int(phys), int(numa), int(round(float(occ) * 100))))
    nphys = max((p for p, _ in raw_links), default=-1) + 1
    q = [XGMI_IDLE_QUALITY] * (nphys * nphys)
    for a in range(nphys):
        q[a * nphys + a] = 10000
    for phys, links in raw_links:
        row = phys * nphys
        for d in links:
            peer = int(d.get("peer", 0))
            if 0 <= peer < nphys:
                load = float(d.get("load", 0.0))
                q[row + peer] = 0 if not bool(d.get("up", True)) else \
                    int(round(XGMI_IDLE_QUALITY * (1.0 - (0.0 if load < 0.0 else 1.0 if load > 1.0 else load))))
    for a in range(nphys):
        ra = a * nphys
        for b in range(a + 1, nphys):
            x, y = q[ra + b], q[b * nphys + a]
            q[ra + b] = q[b * nphys + a] = x if x < y else y
    ut = status.get("updateTime")
    from ..models.scv import parse_rfc3339
    return (cards, int(status.get("cardNumber", 0) or 0) & _M64, int(status.get("freeMemorySum", 0) or 0) & _M64,
            int(status.get("totalMemorySum", 0) or 0) & _M64, float(parse_rfc3339(ut) or 0.0), nphys, q)


def push_scv(engine, idx: int, scv, compat: bool, stale: bool = False) -> None:
    view = getattr(scv, "engine_view", None) if isinstance(scv, LazyScv) else None
    if view is not None:
        cards, cn, fs, ts, ut, nphys, q = view
        engine.set_cards(idx, cards, cn, fs, ts, stale, ut)
        if nphys:
            engine.set_links(idx, nphys, q)
        return
    st = scv.status
    cards = compat_card_tuples(scv) if compat else card_tuples(scv)
    engine.set_cards(idx, cards, int(st.card_number) & _M64, int(st.free_memory_sum) & _M64,
                     int(st.total_memory_sum) & _M64, stale, float(st.update_time or 0.0))
    nphys, q = link_matrix(scv)
    if nphys:
        engine.set_links(idx, nphys, q)


def push_node(engine, info: NodeInfo) -> int:
    idx = engine.upsert_node(info.name)
    engine.set_node_meta(idx, info.unschedulable, list(info.labels.items()), list(info.taints),
                         info.cpu_m, info.mem, info.pods)
    if info.images or info.ext_alloc or info.avoid:
        engine.set_node_extras(idx, list(info.images.items()), list(info.ext_alloc.items()), avoid_controllers(info.avoid))
    else:
        engine.set_node_extras(idx, [], [], [])
    return idx


def avoid_controllers(raw) -> list:
    """(kind, uid) of every ``podSignature.podController`` in a node's
    ``scheduler.alpha.kubernetes.io/preferAvoidPods`` annotation (plugins/node_extras.py
    NodePreferAvoidPods reads the same); an unparsable annotation avoids nothing."""
    if not raw:
        return []
    import json
    try:
        items = json.loads(raw).get("preferAvoidPods") or []
    except (ValueError, AttributeError):
        return []
    out = []
    for a in items if isinstance(items, list) else ():
        pc = ((a.get("podSignature") or {}).get("podController")) or {} if isinstance(a, dict) else {}
        if pc.get("kind") in ("ReplicationController", "ReplicaSet"):
            out.append((pc["kind"], str(pc.get("uid") or "")))
    return out


_shared_reqs: list = [None, {}]      # [weakref to the engine, {template key: PodReq}]


def pod_req(engine, pi: PodInfo):
    """Build (and cache on the PodInfo) the engine's PodReq.

    Pods stamped from one template (a ReplicaSet's, a Job's, a burst's) share a PodReq: the
    engine only ever reads it (``const PodReq&``), so a pod without node-side constraints,
    extended resources or spread / affinity terms takes the PodReq of the last pod with the
    same requests, labels, namespace, images and owner instead of two extension calls."""
    if pi.native_owner is engine and pi.native_req is not None:
        return pi.native_req
    key = None
    if not (pi.node_name or pi.node_selector or pi.required_terms or pi.preferred_terms or pi.tolerations
            or pi.ext or pi.spread or pi.pod_aff or pi.host_ports or pi.flags & PF_CLAIMS):
        key = (pi.gpu, pi.cpu_m, pi.mem, pi.nz_cpu_m, pi.nz_mem, pi.namespace, tuple(pi.labels.items()),
               tuple(pi.images), pi.containers, pi.owner, pi.avoid, pi.deleting, pi.priority)
        shared = _shared_reqs
        if shared[0] is None or shared[0]() is not engine:   # weak: a shut-down engine is freed
            shared[0], shared[1] = weakref.ref(engine), {}
        r = shared[1].get(key)
        if r is not None:
            pi.native_req, pi.native_owner = r, engine
            return r
    g = pi.gpu
    r = engine.make_req(g.has_number, g.number, g.has_memory, g.memory, g.has_clock, g.clock,
                        g.clock_min, g.priority, pi.node_name, pi.cpu_m, pi.mem,
                        list(pi.node_selector.items()), pi.required_terms, pi.preferred_terms,
                        pi.tolerations, pi.nz_cpu_m, pi.nz_mem)
    engine.set_req_extras(r, pi.namespace, list(pi.labels.items()), pi.deleting, pi.images, pi.containers,
                          list(pi.ext.items()), pi.owner, pi.avoid, pi.spread, pi.pod_aff)
    if pi.priority:
        r.pod_priority = pi.priority      # spec.priority: what DefaultPreemption compares on the ledger
    if pi.host_ports:
        from ..plugins.defaults import host_port_set
        engine.set_req_ports(r, [(port, proto, ip) for ip, proto, port in sorted(host_port_set(pi.host_ports))])
    if pi.flags & PF_CLAIMS:
        # the ledger keeps every pod's PVC claims per node: the lane's NodeVolumeLimits counts them
        from ..plugins.volumes import pvc_claim_keys
        engine.set_req_claims(r, pvc_claim_keys(pi), False)
    pi.native_req, pi.native_owner = r, engine
    if key is not None:
        cache = _shared_reqs[1]
        if len(cache) >= 4096:
            cache.clear()
        cache[key] = r
    return r
