"""Scheduler cache: nodes, Scv telemetry, bound + assumed pods — backed by the native
engine's node table and per-GPU HBM reservation ledger.

Upstream semantics kept: a selected pod is *assumed* into the cache
before its asynchronous bind, so the very next cycle already sees it (the reference's
Allocate score depends on this, ``pkg/yoda/score/algorithm.go:74-80``); an assumed pod
is confirmed when the informer reports it bound, forgotten on bind failure, and
expires if the confirmation never arrives.

MI355X additions: assumed/bound pods reserve ``scv/memory`` MB on each assigned GPU
(quirk Q10 fixed), the assignment travels as the ``scv.amd.com/gpus`` annotation and
is rebuilt from it on restart (SURVEY §5 checkpoint/resume), and an ``Scv`` whose
sample is older than ``staleFactor × updateInterval`` makes its node unschedulable for
GPU pods.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Callable, Optional

from ..models.labels import ANNOTATION_GPUS
from ..models.pod import PF_REQ_ANTI, NodeInfo, PodInfo
from ..models.scv import LazyScv, Scv
from ..ops.native import pod_req, push_node, push_scv, scv_engine_view


@dataclass
class PodState:
    info: PodInfo
    node: str
    cards: list[int]
    assumed: bool
    deadline: Optional[float] = None      # assumed + binding finished → expiry
    lane: bool = False                    # mirrored from the native lane (it owns the reservation)


_CSI_ALLOC = "attachable-volumes-csi-"


def _csi_attach_limits(obj: dict) -> list:
    """CSI drivers the node's allocatable limits (``attachable-volumes-csi-<driver>``)."""
    alloc = (obj.get("status") or {}).get("allocatable") or {}
    return [k[len(_CSI_ALLOC):] for k in alloc if k.startswith(_CSI_ALLOC)]


class SchedulerCache:
    def __init__(self, engine, compat: bool = False, stale_factor: float = 3.0,
                 assume_ttl: float = 30.0, clock: Callable[[], float] = time.monotonic,
                 wall: Callable[[], float] = time.time) -> None:
        self.engine = engine
        self.compat = compat
        self.stale_factor = stale_factor
        self.assume_ttl = assume_ttl
        self.clock = clock
        self.wall = wall
        self.nodes: dict[str, NodeInfo] = {}
        self.scvs: dict[str, Scv] = {}
        self._stale: dict[str, bool] = {}
        self.pods: dict[str, PodState] = {}
        self.node_pods: dict[str, set[str]] = {}
        self._anti: set[str] = set()
        self._anti_terms: Optional[list] = None     # required anti-affinity terms of self._anti
        self._anti_parsed: dict[str, list] = {}     # uid → [(topologyKey, namespaces, LabelSelector)]
        self.image_nodes: dict[str, int] = {}    # image → number of nodes holding it (ImageLocality)
        self.avoid_nodes: set[str] = set()       # nodes with a preferAvoidPods annotation
        # CSI driver → nodes whose allocatable limits it (attachable-volumes-csi-<driver>; NodeVolumeLimits)
        self.csi_limit_drivers: dict[str, int] = {}
        self.node_ext_used: dict[str, dict[str, int]] = {}   # node → extended resource → requested
        self.generation = 0
        self.node_generation = 0                 # node add/remove only (engine index → name stays valid)
        self.lane = None                         # native lane (core.Lane) whose reserved pods sync_lane mirrors
        self.on_anti_change = None               # called when the set of required-anti-affinity pods changes
        self._lane_uids: dict[int, str] = {}     # lane ledger id → uid of the mirrored pod
        self.lane_synced_at: Optional[float] = None   # clock() of the last sync_lane
        self.lane_census_at: Optional[float] = None   # clock() of the last lane_counts
        self.lane_never_flags = 0                # pod flags no lane pod carries (NativeLane.refresh)

    # ------------------------------------------------------------------ nodes
    def _index_node(self, info: NodeInfo, sign: int) -> None:
        for im in info.images:
            c = self.image_nodes.get(im, 0) + sign
            if c > 0:
                self.image_nodes[im] = c
            else:
                self.image_nodes.pop(im, None)
        for d in _csi_attach_limits(info.obj):
            c = self.csi_limit_drivers.get(d, 0) + sign
            if c > 0:
                self.csi_limit_drivers[d] = c
            else:
                self.csi_limit_drivers.pop(d, None)
        if sign > 0 and info.avoid:
            self.avoid_nodes.add(info.name)
        elif sign < 0:
            self.avoid_nodes.discard(info.name)

    def add_node(self, obj: dict) -> None:
        info = NodeInfo.from_obj(obj)
        old = self.nodes.get(info.name)
        if old is not None:
            self._index_node(old, -1)
        self._index_node(info, +1)
        self.nodes[info.name] = info
        idx = push_node(self.engine, info)
        if old is None:
            self.node_generation += 1
        self.node_pods.setdefault(info.name, set())
        scv = self.scvs.get(info.name)
        if scv is not None:
            push_scv(self.engine, idx, scv, self.compat, self._stale.get(info.name, False))
        self.generation += 1

    update_node = add_node

    def remove_node(self, name: str) -> None:
        self.node_ext_used.pop(name, None)
        old = self.nodes.pop(name, None)
        if old is not None:
            self._index_node(old, -1)
        idx = self.engine.node_index(name)
        if idx >= 0:
            self.engine.remove_node(idx)
        self.node_generation += 1
        for uid in list(self.node_pods.pop(name, ())):
            self.pods.pop(uid, None)
        self.generation += 1

    # ------------------------------------------------------------------ telemetry
    def set_scv(self, scv: Scv) -> None:
        self.scvs[scv.name] = scv
        stale = (not self.compat) and scv.is_stale(self.wall(), self.stale_factor)
        self._stale[scv.name] = stale
        idx = self.engine.node_index(scv.name)
        if idx >= 0:
            push_scv(self.engine, idx, scv, self.compat, stale)
        self.generation += 1

    def add_scv(self, obj: dict) -> None:
        # engine view (and the cards' identities) straight from the JSON; the Scv
        # dataclasses are built only if read
        idents: list = []
        self.set_scv(LazyScv(obj, scv_engine_view(obj, self.compat, idents), idents))

    update_scv = add_scv

    def remove_scv(self, name: str) -> None:
        self.scvs.pop(name, None)
        self._stale.pop(name, None)
        idx = self.engine.node_index(name)
        if idx >= 0:
            self.engine.clear_scv(idx)
        self.generation += 1

    def refresh_staleness(self) -> list[str]:
        """Re-evaluate sample freshness; returns nodes whose state flipped."""
        if self.compat:
            return []
        now, flipped = self.wall(), []
        for name, scv in self.scvs.items():
            st = scv.is_stale(now, self.stale_factor)
            if st != self._stale.get(name):
                self._stale[name] = st
                idx = self.engine.node_index(name)
                if idx >= 0:
                    push_scv(self.engine, idx, scv, self.compat, st)
                flipped.append(name)
        return flipped

    # ------------------------------------------------------------------ pods
    def _ext(self, ps: PodState, sign: int) -> None:
        used = self.node_ext_used.setdefault(ps.node, {})
        for k, v in ps.info.ext.items():
            used[k] = used.get(k, 0) + sign * v

    def _track(self, ps: PodState) -> None:
        if ps.info.ext:
            self._ext(ps, +1)
        self.pods[ps.info.uid] = ps
        self.node_pods.setdefault(ps.node, set()).add(ps.info.uid)
        if ps.info.flags & PF_REQ_ANTI:
            if ps.info.uid not in self._anti:
                self._anti_parsed.pop(ps.info.uid, None)
                self._anti.add(ps.info.uid)
                self._anti_changed(True)
        else:
            self._anti_drop(ps.info.uid)

    def _anti_drop(self, uid: str) -> None:
        if uid in self._anti:
            self._anti.discard(uid)
            self._anti_parsed.pop(uid, None)
            self._anti_changed(False)

    def _anti_changed(self, grew: bool) -> None:
        """InterPodAffinity's cluster gate (required anti-affinity symmetry) may have flipped:
        the native lane re-decides which pods it may take (``grew``: a holder was added — the
        lane must learn it before it places another pod; a removal may be applied later)."""
        self._anti_terms = None
        if self.on_anti_change is not None:
            self.on_anti_change(grew)

    def hide(self, uids) -> list:
        """Drop pods from the Python-side views (``pods`` / ``node_pods`` / extended-resource
        usage) without touching the engine ledger: the preemption what-if of upstream's
        ``RemovePod`` on a NodeInfo copy. ``unhide`` puts them back."""
        out = []
        for uid in uids:
            ps = self.pods.pop(uid, None)
            if ps is None:
                continue
            self.node_pods.get(ps.node, set()).discard(uid)
            if ps.info.ext:
                self._ext(ps, -1)
            out.append(ps)
        return out

    def unhide(self, states) -> None:
        for ps in states:
            self._track(ps)

    def pods_with_required_anti_affinity(self) -> int:
        """Bound/assumed pods whose required anti-affinity can reject new pods (symmetry)."""
        if self._anti:
            pods = self.pods
            gone = [u for u in self._anti if u not in pods]   # O(holders), not O(pods)
            if gone:
                self._anti.difference_update(gone)
                self._anti_terms = None
        return len(self._anti)

    def _anti_of(self, uid: str) -> list:
        """The parsed required anti-affinity terms of a bound/assumed pod (once per pod)."""
        r = self._anti_parsed.get(uid)
        if r is None:
            from ..models.selectors import LabelSelector
            info = self.pods[uid].info
            aff = ((info.obj.get("spec") or {}).get("affinity") or {}).get("podAntiAffinity") or {}
            r = self._anti_parsed[uid] = [
                (t.get("topologyKey", ""), tuple(t.get("namespaces") or (info.namespace,)),
                 LabelSelector(t.get("labelSelector")))
                for t in aff.get("requiredDuringSchedulingIgnoredDuringExecution") or ()]
        return r

    def anti_terms(self) -> list:
        """(namespaces, LabelSelector) of every required anti-affinity term of a bound/assumed
        pod: an incoming pod matching none of them is unaffected by the symmetric rule."""
        if self.pods_with_required_anti_affinity() == 0:
            if self._anti_parsed:
                self._anti_parsed.clear()
            return []
        if self._anti_terms is None:
            if len(self._anti_parsed) > 2 * len(self._anti) + 16:
                self._anti_parsed = {u: v for u, v in self._anti_parsed.items() if u in self._anti}
            self._anti_terms = [(ns, sel) for uid in self._anti for _k, ns, sel in self._anti_of(uid)]
        return self._anti_terms

    def anti_holders(self):
        """(pod info, node, [(topologyKey, namespaces, LabelSelector)]) of every bound/assumed pod
        with required anti-affinity (InterPodAffinity's symmetric rule), terms parsed once."""
        if self.pods_with_required_anti_affinity() == 0:
            return
        for uid in list(self._anti):
            ps = self.pods.get(uid)
            if ps is not None:
                yield ps.info, ps.node, self._anti_of(uid)

    def lane_counts(self, queries: list, skip_deleting: bool = False) -> list:
        """Per query (a list of native terms, all of which a pod must match): lane pods holding a
        reservation counted per node (``core.Lane.count_matching``); empty dicts without a lane.
        Plugins that count matching pods add these to their walk over the Python-owned pods
        (lane mirrors skipped), so they need no Python copy of the lane's pods."""
        if self.lane is None or not queries:
            return [{} for _ in queries]
        self.lane_census_at = self.clock()
        return self.lane.count_matching(queries, skip_deleting)

    def assumed(self, pi: PodInfo, node: str, cards: list[int]) -> None:
        """Record a pod the engine reserved during ``schedule(assume=True)``."""
        self._track(PodState(pi, node, list(cards), True))

    def assume(self, pi: PodInfo, node: str, cards: list[int]) -> bool:
        idx = self.engine.node_index(node)
        if idx < 0 or not self.engine.reserve(pi.num_id, pod_req(self.engine, pi), idx, list(cards)):
            return False
        self.assumed(pi, node, cards)
        return True

    def finish_binding(self, pi: PodInfo) -> None:
        ps = self.pods.get(pi.uid)
        if ps is not None and ps.assumed:
            ps.deadline = self.clock() + self.assume_ttl

    def forget(self, pi: PodInfo) -> None:
        ps = self.pods.pop(pi.uid, None)
        self._anti_drop(pi.uid)
        if ps is not None:
            self.node_pods.get(ps.node, set()).discard(pi.uid)
            if ps.info.ext:
                self._ext(ps, -1)
        self.engine.release(pi.num_id)

    def add_pod(self, obj: dict) -> None:
        """A bound pod observed by the informer (confirms an assumed pod)."""
        meta = obj.get("metadata") or {}
        ps = self.pods.get(meta.get("uid"))
        if ps is not None and ps.assumed and ps.node == (obj.get("spec") or {}).get("nodeName"):
            ps.assumed, ps.deadline = False, None      # fast confirm: no re-parse
            ps.info.obj = obj
            return
        self._add_bound(PodInfo.from_obj(obj))

    def add_pod_native(self, ev, uid: str, node: str) -> None:
        """``add_pod`` for a native transport ``PodEvent`` (decoded only when not a confirm)."""
        ps = self.pods.get(uid)
        if ps is not None and ps.assumed and ps.node == node:
            ps.assumed, ps.deadline = False, None
            ps.info.set_source(ev)
            return
        self._add_bound(PodInfo.from_native(ev))

    def update_pod_native(self, ev, uid: str, node: str, same_spec: bool = False) -> None:
        ps = self.pods.get(uid)
        if ps is None or ps.node != node:
            self.add_pod_native(ev, uid, node)
        elif same_spec:
            ps.info.set_source(ev)         # status-only update (kubelet): nothing to re-parse
        else:
            self._replace_info(ps, PodInfo.from_native(ev))

    def _replace_info(self, ps: PodState, pi: PodInfo) -> None:
        """A bound pod's spec / metadata changed: keep its ledger id, and let the engine's copy
        of its labels and deletionTimestamp (what spread constraints count) follow."""
        old = ps.info
        pi.num_id = old.num_id
        ps.info = pi
        if not ps.lane and (pi.labels != old.labels or pi.deleting != old.deleting):
            self.engine.set_pod_meta(pi.num_id, list(pi.labels.items()), pi.deleting)

    def _add_bound(self, pi: PodInfo) -> None:
        node = pi.node_name
        ps = self.pods.get(pi.uid)
        if ps is not None:
            if ps.assumed and ps.node == node:
                ps.assumed, ps.deadline = False, None
                ps.info = pi
                return
            self.forget(ps.info)
        idx = self.engine.node_index(node)
        cards = parse_gpu_annotation(pi.annotations.get(ANNOTATION_GPUS))
        if idx >= 0:
            req = pod_req(self.engine, pi)
            if cards is None:
                ok, sel, _ = self.engine.select_gpus(req, idx)
                cards = sel if ok else []
            if not self.engine.reserve(pi.num_id, req, idx, cards):
                self.engine.reserve(pi.num_id, req, idx, [])
        self._track(PodState(pi, node, cards or [], False))

    def update_pod(self, obj: dict) -> None:
        pi = PodInfo.from_obj(obj)
        ps = self.pods.get(pi.uid)
        if ps is None or ps.node != pi.node_name:
            self.add_pod(obj)
        else:
            self._replace_info(ps, pi)

    def remove_pod(self, uid: str) -> None:
        ps = self.pods.pop(uid, None)
        self._anti_drop(uid)
        if ps is not None:
            self.node_pods.get(ps.node, set()).discard(uid)
            if ps.info.ext:
                self._ext(ps, -1)
            self.engine.release(ps.info.num_id)

    def cleanup_expired(self) -> list[PodInfo]:
        now, out = self.clock(), []
        for uid, ps in list(self.pods.items()):
            if ps.assumed and ps.deadline is not None and now > ps.deadline:
                self.forget(ps.info)
                out.append(ps.info)
        return out

    def sync_lane(self) -> int:
        """Mirror the native lane's reserved pods into ``pods`` / ``node_pods`` (only what
        changed since the last call) for the Python plugins that read other pods — pod
        (anti-)affinity, topology spread, preemption. The lane keeps owning them: their
        ``num_id`` is the lane's ledger id and nothing here releases them. Returns the
        number of changes applied."""
        lane = self.lane
        if lane is None:
            return 0
        self.lane_synced_at = self.clock()
        full, changes = lane.changes()
        if full:
            for uid in list(self._lane_uids.values()):
                self._untrack_lane(uid)
            self._lane_uids.clear()
        for lid, add, ev, node, cards in changes:
            if add:
                old = self._lane_uids.pop(lid, None)
                if old is not None:
                    self._untrack_lane(old)
                pi = PodInfo.from_native(ev)
                cur = self.pods.get(pi.uid)
                if cur is not None and not cur.lane:
                    continue        # Python's own state of the pod (it took the pod over) wins
                pi.num_id = lid
                self._track(PodState(pi, node, list(cards), False, lane=True))
                self._lane_uids[lid] = pi.uid
            else:
                uid = self._lane_uids.pop(lid, None)
                if uid is not None:
                    self._untrack_lane(uid)
        if changes or full:
            self.generation += 1
        return len(changes)

    def drop_lane_mirror(self) -> int:
        """Forget every mirrored lane pod and turn the lane's change log off: no Python-path
        cycle has read the mirror for a while, so lane Bindings stop paying for it (the next
        Python cycle resyncs from a full snapshot). Returns the number of pods dropped."""
        n = 0
        for uid in list(self._lane_uids.values()):
            n += self._untrack_lane(uid)
        self._lane_uids.clear()
        if self.lane is not None:
            self.lane.stop_log()
        if n:
            self.generation += 1
        return n

    def lane_mirrored(self) -> int:
        """Pods in ``pods`` that are mirrors of lane pods (not Python-owned)."""
        n = 0
        for uid in self._lane_uids.values():
            ps = self.pods.get(uid)
            n += ps is not None and ps.lane
        return n

    def python_pods(self) -> int:
        """Bound/assumed pods the Python side owns (lane mirrors excluded)."""
        return len(self.pods) - self.lane_mirrored()

    def _untrack_lane(self, uid: str) -> bool:
        """Drop a lane mirror; a PodState the Python side owns under that uid (it took the pod
        over after a failed lane Binding) is left alone."""
        ps = self.pods.get(uid)
        if ps is None or not ps.lane:
            return False
        self._untrack(uid)
        return True

    def _untrack(self, uid: str) -> None:
        ps = self.pods.pop(uid, None)
        if ps is not None:
            self.node_pods.get(ps.node, set()).discard(uid)
            if ps.info.ext:
                self._ext(ps, -1)

    def is_assumed(self, uid: str) -> bool:
        ps = self.pods.get(uid)
        return ps is not None and ps.assumed

    # ------------------------------------------------------------------ views
    def node_gpu_state(self, name: str) -> list[dict]:
        idx = self.engine.node_index(name)
        if idx < 0:
            return []
        return [{"total": t, "free": f, "reserved": r, "pods": p, "clock": c, "healthy": h, "phys": ph,
                 "pending": pe}
                for (t, f, r, p, c, h, ph, pe) in self.engine.node_cards(idx)]

    def snapshot_counts(self) -> dict:
        return {"nodes": len(self.nodes), "scvs": len(self.scvs), "pods": len(self.pods),
                "assumed": sum(1 for p in self.pods.values() if p.assumed)}


def parse_gpu_annotation(v: Optional[str]) -> Optional[list[int]]:
    if v is None:
        return None
    v = v.strip()
    if not v:
        return []
    try:
        return [int(x) for x in v.split(",") if x.strip()]
    except ValueError:
        return None
