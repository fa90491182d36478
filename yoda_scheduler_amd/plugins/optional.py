"""The in-tree plugins kube-scheduler v1.20 *registers* but does not enable by default —
``NodeLabel``, ``ServiceAffinity``, ``SelectorSpread`` and ``RequestedToCapacityRatio``.
The reference's binary is the full upstream scheduler plus ``yoda``
(``pkg/register/register.go:9-13``), so a profile (or a legacy Policy file, see
``framework/policy.py``) may turn any of them on; SURVEY §2.2 U6.

All four are Python plugins. The first three are conditional (``is_noop_for``): a pod
they cannot affect stays on the native cycle. ``RequestedToCapacityRatio`` scores every
pod, so a profile that enables it runs the hybrid cycle (native filters, Python score).
Semantics follow upstream v1.20 (``pkg/scheduler/framework/plugins/{nodelabel,
serviceaffinity,selectorspread,noderesources/requested_to_capacity_ratio.go}``); the
reference tree holds no copy of that code, so parity is pinned by the hand-computed
vectors in ``tests/test_plugins_optional.py``.
"""
from __future__ import annotations

import math
from collections import defaultdict
from typing import Optional

from ..framework.interfaces import (CycleState, FilterPlugin, NodeScore, PreFilterPlugin, PreScorePlugin, ScorePlugin,
                                    StateData, Status, MAX_NODE_SCORE)
from ..models.pod import PF_CONTROLLER
from ..models.selectors import LabelSelector

LABEL_ZONE = ("failure-domain.beta.kubernetes.io/zone", "topology.kubernetes.io/zone")
LABEL_REGION = ("failure-domain.beta.kubernetes.io/region", "topology.kubernetes.io/region")
ZONE_WEIGHTING = 2.0 / 3.0


def _node_labels(handle, node: str) -> dict:
    n = handle.cache.nodes.get(node)
    return n.labels if n is not None else {}


def zone_key(labels: dict) -> str:
    """upstream ``utilnode.GetZoneKey``: beta labels first, ``region:\\x00:zone``."""
    zone = labels.get(LABEL_ZONE[0], labels.get(LABEL_ZONE[1], ""))
    region = labels.get(LABEL_REGION[0], labels.get(LABEL_REGION[1], ""))
    if not region and not zone:
        return ""
    return region + ":\x00:" + zone


def _deleting(pod) -> bool:
    return bool((pod.obj.get("metadata") or {}).get("deletionTimestamp"))


def pod_services(handle, pod) -> list[dict]:
    """upstream ``helper.GetPodServices``: services of the pod's namespace whose (non-nil)
    selector matches the pod's labels, in name order."""
    out = []
    for key in sorted(handle.lister("services")):
        svc = handle.lister("services")[key]
        meta = svc.get("metadata") or {}
        if (meta.get("namespace") or "default") != pod.namespace:
            continue
        sel = (svc.get("spec") or {}).get("selector")
        if sel is None:
            continue                                  # nil selector matches nothing
        if all(pod.labels.get(k) == v for k, v in sel.items()):
            out.append(svc)
    return out


class _Selector:
    """A merged label selector: equality requirements plus LabelSelector requirement sets
    (``labels.Selector`` with ``Add``). Empty ⇒ matches nothing for counting purposes."""
    __slots__ = ("eq", "sels")

    def __init__(self) -> None:
        self.eq: dict = {}
        self.sels: list[LabelSelector] = []

    @property
    def empty(self) -> bool:
        return not self.eq and not self.sels

    def matches(self, labels: dict) -> bool:
        return all(labels.get(k) == v for k, v in self.eq.items()) and all(s.matches(labels) for s in self.sels)

    def native_query(self, namespaces=None) -> list:
        """The conjunction as native terms (``core.Lane.count_matching``): a pod counts when it
        matches every one."""
        ns = None if namespaces is None else tuple(namespaces)
        return [(ns, False, tuple(self.eq.items()), ())] + [s.native(namespaces) for s in self.sels]


_OWNER_KINDS = {("v1", "ReplicationController"): "replicationcontrollers",
                ("apps/v1", "ReplicaSet"): "replicasets",
                ("apps/v1", "StatefulSet"): "statefulsets"}


def default_selector(handle, pod) -> _Selector:
    """upstream ``helper.DefaultSelector``: the union of the selectors of the services
    matching the pod and of its controller (RC map selector; RS / StatefulSet
    LabelSelector requirements)."""
    s = _Selector()
    for svc in pod_services(handle, pod):
        s.eq.update((svc.get("spec") or {}).get("selector") or {})
    for ref in (pod.obj.get("metadata") or {}).get("ownerReferences") or ():
        if not ref.get("controller"):
            continue
        res = _OWNER_KINDS.get((ref.get("apiVersion", ""), ref.get("kind", "")))
        if res is None:
            break
        owner = handle.lister(res).get(f"{pod.namespace}/{ref.get('name', '')}")
        if owner is None:
            break
        sel = (owner.get("spec") or {}).get("selector")
        if res == "replicationcontrollers":
            s.eq.update(sel or {})
        elif sel is not None:
            ls = LabelSelector(sel)
            if not ls.empty:
                s.sels.append(ls)
        break
    return s


def _count(handle, namespace: str, sel: _Selector, node: str) -> int:
    if sel.empty:
        return 0
    cache = handle.cache
    n = 0
    for uid in cache.node_pods.get(node, ()):
        ps = cache.pods.get(uid)
        if ps is not None and ps.info.namespace == namespace and not _deleting(ps.info) \
                and sel.matches(ps.info.labels):
            n += 1
    return n


# ============================================================== NodeLabel
class NodeLabel(FilterPlugin, ScorePlugin):
    """Filter: the node has every ``presentLabels`` key and none of ``absentLabels``.
    Score: 100 per satisfied ``presentLabelsPreference`` / ``absentLabelsPreference``
    key, averaged over the preference keys."""
    name = "NodeLabel"
    pod_flags = None          # applies to every pod once configured
    reads_flags = 0  # other pods' features this plugin reads (needs_lane_mirror)

    def __init__(self, args: Optional[dict] = None, handle=None) -> None:
        super().__init__(args, handle)
        a = self.args
        self.present = list(a.get("presentLabels") or [])
        self.absent = list(a.get("absentLabels") or [])
        self.present_pref = list(a.get("presentLabelsPreference") or [])
        self.absent_pref = list(a.get("absentLabelsPreference") or [])
        for x, y in ((self.present, self.absent), (self.present_pref, self.absent_pref)):
            both = sorted(set(x) & set(y))
            if both:
                raise ValueError(f"NodeLabel: label {both[0]!r} is in both the present {x} and absent {y} lists")

    def is_noop_for(self, pod) -> bool:
        return not (self.present or self.absent or self.present_pref or self.absent_pref)

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        labels = _node_labels(self.handle, node_name)
        if all(k in labels for k in self.present) and not any(k in labels for k in self.absent):
            return Status.ok()
        return Status.unschedulable("node(s) didn't have the requested labels", plugin=self.name)

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        size = len(self.present_pref) + len(self.absent_pref)
        if size == 0:
            return 0, Status.ok()
        labels = _node_labels(self.handle, node_name)
        s = MAX_NODE_SCORE * (sum(1 for k in self.present_pref if k in labels)
                              + sum(1 for k in self.absent_pref if k not in labels))
        return s // size, Status.ok()


# ============================================================== ServiceAffinity
class _ServiceAffinityState(StateData):
    def __init__(self, pods: list, services: list) -> None:
        self.pods, self.services = pods, services

    def clone(self) -> "_ServiceAffinityState":
        return self


class ServiceAffinity(PreFilterPlugin, FilterPlugin, ScorePlugin):
    """Filter (``affinityLabels``): the pod lands on nodes whose values for those labels
    equal the ones of the node already running the first pod of its service (or the
    pod's own nodeSelector values). Score (``antiAffinityLabelsPreference``): fewer
    service pods in the node's label domain scores higher."""
    name = "ServiceAffinity"
    KEY = "PreFilterServiceAffinity"
    watches = ("services",)
    pod_flags = None

    def __init__(self, args: Optional[dict] = None, handle=None) -> None:
        super().__init__(args, handle)
        self.affinity_labels = list(self.args.get("affinityLabels") or [])
        self.anti_prefs = list(self.args.get("antiAffinityLabelsPreference") or [])

    def is_noop_for(self, pod) -> bool:
        return not self.affinity_labels and not self.anti_prefs

    def pre_filter(self, state: CycleState, pod) -> Status:
        services = pod_services(self.handle, pod)
        pods = []
        if pod.labels:                     # an empty selector selects nothing here (filteredPod)
            cache = self.handle.cache
            for node, uids in cache.node_pods.items():
                for uid in uids:
                    ps = cache.pods.get(uid)
                    if ps is not None and ps.info.namespace == pod.namespace and \
                            all(ps.info.labels.get(k) == v for k, v in pod.labels.items()):
                        pods.append(ps)
        state.write(self.KEY, _ServiceAffinityState(pods, services))
        return Status.ok()

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        if not self.affinity_labels:
            return Status.ok()
        try:
            s: _ServiceAffinityState = state.read(self.KEY)
        except KeyError:
            self.pre_filter(state, pod)
            s = state.read(self.KEY)
        want = {k: pod.node_selector[k] for k in self.affinity_labels if k in pod.node_selector}
        if len(want) < len(self.affinity_labels) and s.services and s.pods:
            first = _node_labels(self.handle, s.pods[0].node)
            for k in self.affinity_labels:
                if k not in want and k in first:
                    want[k] = first[k]
        labels = _node_labels(self.handle, node_name)
        if all(labels.get(k) == v for k, v in want.items()):
            return Status.ok()
        return Status.unschedulable("node(s) didn't match service affinity", plugin=self.name)

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        services = pod_services(self.handle, pod)
        if not services:
            return 0, Status.ok()
        sel = _Selector()
        sel.eq.update((services[0].get("spec") or {}).get("selector") or {})
        return _count(self.handle, pod.namespace, sel, node_name), Status.ok()

    def normalize_score(self, state: CycleState, pod, scores: list[NodeScore]) -> Status:
        reduce = [0.0] * len(scores)
        nlab = len(self.anti_prefs)
        for label in self.anti_prefs:
            total = 0
            per_value: dict = defaultdict(int)
            value_of: dict = {}
            for ns in scores:
                total += ns.score
                labels = _node_labels(self.handle, ns.name)
                if label not in labels:
                    continue
                value_of[ns.name] = labels[label]
                per_value[labels[label]] += ns.score
            for i, ns in enumerate(scores):
                v = value_of.get(ns.name)
                if v is None:
                    continue
                f = float(MAX_NODE_SCORE)
                if total > 0:
                    f = MAX_NODE_SCORE * (float(total - per_value[v]) / float(total))
                reduce[i] += f / nlab
        for i, ns in enumerate(scores):
            ns.score = int(reduce[i])
        return Status.ok()


# ============================================================== SelectorSpread
class _SpreadSelector(StateData):
    def __init__(self, sel: _Selector) -> None:
        self.sel = sel

    def clone(self) -> "_SpreadSelector":
        return self


class SelectorSpread(PreScorePlugin, ScorePlugin):
    """Spread the pods of one Service / ReplicationController / ReplicaSet / StatefulSet
    across nodes and zones: score = 100·(max − count)/max per node, blended 1/3 node +
    2/3 zone when nodes carry zone labels. Pods with topologySpreadConstraints are left
    to PodTopologySpread."""
    name = "SelectorSpread"
    KEY = "PreScoreSelectorSpread"
    watches = ("services", "replicationcontrollers", "replicasets", "statefulsets")
    pod_flags = PF_CONTROLLER

    def cluster_active(self) -> bool:
        return bool(self.handle.lister("services"))

    @staticmethod
    def _skip(pod) -> bool:
        return bool((pod.obj.get("spec") or {}).get("topologySpreadConstraints"))

    def _has_controller(self, pod) -> bool:
        return any(r.get("controller") and (r.get("apiVersion", ""), r.get("kind", "")) in _OWNER_KINDS
                   for r in (pod.obj.get("metadata") or {}).get("ownerReferences") or ())

    def is_noop_for(self, pod) -> bool:
        if self._skip(pod):
            return True
        return not self._has_controller(pod) and not pod_services(self.handle, pod)

    def pre_score(self, state: CycleState, pod, nodes: list[str]) -> Status:
        if not self._skip(pod):
            state.write(self.KEY, _SpreadSelector(default_selector(self.handle, pod)))
        return Status.ok()

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        if self._skip(pod):
            return 0, Status.ok()
        try:
            s: _SpreadSelector = state.read(self.KEY)
        except KeyError:
            s = _SpreadSelector(default_selector(self.handle, pod))
            state.write(self.KEY, s)
        return _count(self.handle, pod.namespace, s.sel, node_name), Status.ok()

    def normalize_score(self, state: CycleState, pod, scores: list[NodeScore]) -> Status:
        if self._skip(pod):
            return Status.ok()
        by_zone: dict = defaultdict(int)
        zones = []
        max_node = 0
        for ns in scores:
            max_node = max(max_node, ns.score)
            z = zone_key(_node_labels(self.handle, ns.name))
            zones.append(z)
            if z:
                by_zone[z] += ns.score
        max_zone = max(by_zone.values(), default=0)
        for ns, z in zip(scores, zones):
            f = float(MAX_NODE_SCORE)
            if max_node > 0:
                f = MAX_NODE_SCORE * (float(max_node - ns.score) / float(max_node))
            if by_zone and z:
                zs = float(MAX_NODE_SCORE)
                if max_zone > 0:
                    zs = MAX_NODE_SCORE * (float(max_zone - by_zone[z]) / float(max_zone))
                f = f * (1.0 - ZONE_WEIGHTING) + ZONE_WEIGHTING * zs
            ns.score = int(f)
        return Status.ok()


# ============================================================== RequestedToCapacityRatio
MAX_CUSTOM_PRIORITY_SCORE = 10
MAX_UTILIZATION = 100


def broken_linear(shape: list[tuple[int, int]]):
    """upstream ``buildBrokenLinearFunction``: piecewise-linear through (utilization,
    score) points, flat outside them, integer arithmetic."""
    def f(p: int) -> int:
        for i, (u, s) in enumerate(shape):
            if p <= u:
                if i == 0:
                    return shape[0][1]
                pu, ps = shape[i - 1]
                return ps + (s - ps) * (p - pu) // (u - pu)
        return shape[-1][1]
    return f


class RequestedToCapacityRatio(ScorePlugin):
    """score = Σ_r w_r·shape(utilization_r) / Σ_r w_r over resources with a non-zero shape
    value, utilization = requested (incl. this pod; cpu/memory as NonZeroRequested) ÷
    allocatable in percent; ``shape`` scores 0–10 are scaled to 0–100."""
    name = "RequestedToCapacityRatio"

    def __init__(self, args: Optional[dict] = None, handle=None) -> None:
        super().__init__(args, handle)
        shape = self.args.get("shape") or []
        if not shape:
            raise ValueError("RequestedToCapacityRatio: at least one shape point is required")
        pts, prev = [], -1
        for p in shape:
            u, s = int(p.get("utilization", 0)), int(p.get("score", 0))
            if not 0 <= u <= MAX_UTILIZATION:
                raise ValueError(f"RequestedToCapacityRatio: utilization {u} not in [0, {MAX_UTILIZATION}]")
            if u <= prev:
                raise ValueError("RequestedToCapacityRatio: utilization values must be sorted in increasing order")
            if not 0 <= s <= MAX_CUSTOM_PRIORITY_SCORE:
                raise ValueError(f"RequestedToCapacityRatio: score {s} not in [0, {MAX_CUSTOM_PRIORITY_SCORE}]")
            prev = u
            pts.append((u, s * (MAX_NODE_SCORE // MAX_CUSTOM_PRIORITY_SCORE)))
        self.shape = pts
        self.fn = broken_linear(pts)
        res = self.args.get("resources") or [{"name": "cpu", "weight": 1}, {"name": "memory", "weight": 1}]
        self.weights: list[tuple[str, int]] = []
        for r in res:
            w = int(r.get("weight", 1))
            if not 1 <= w <= 100:
                raise ValueError(f"RequestedToCapacityRatio: resource {r.get('name')!r} weight {w} not in [1, 100]")
            self.weights.append((r.get("name", ""), w))

    def _resource_score(self, requested: int, capacity: int) -> int:
        if capacity == 0 or requested > capacity:
            return self.fn(MAX_UTILIZATION)
        return self.fn(MAX_UTILIZATION - (capacity - requested) * MAX_UTILIZATION // capacity)

    def _node(self, pod, node_name: str) -> dict:
        """resource → (requested incl. pod, allocatable)."""
        cache = self.handle.cache
        node = cache.nodes.get(node_name)
        if node is None:
            return {}
        idx = cache.engine.node_index(node_name)
        nz_cpu, nz_mem = cache.engine.node_usage(idx)[4:6] if idx >= 0 else (0, 0)
        out = {"cpu": (nz_cpu + pod.nz_cpu_m, node.cpu_m), "memory": (nz_mem + pod.nz_mem, node.mem)}
        used = cache.node_ext_used.get(node_name, {})
        for r, _w in self.weights:
            if r not in out:
                out[r] = (used.get(r, 0) + pod.ext.get(r, 0), node.ext_alloc.get(r, 0))
        return out

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        vals = self._node(pod, node_name)
        total = wsum = 0
        for r, w in self.weights:
            req, cap = vals.get(r, (0, 0))
            s = self._resource_score(req, cap)
            if s > 0:
                total += s * w
                wsum += w
        if wsum == 0:
            return 0, Status.ok()
        return int(math.floor(total / wsum + 0.5)), Status.ok()   # Go math.Round (values are >= 0)


OPTIONAL_PLUGINS = (NodeLabel, ServiceAffinity, SelectorSpread, RequestedToCapacityRatio)
