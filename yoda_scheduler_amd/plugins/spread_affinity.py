"""PodTopologySpread and InterPodAffinity (upstream default plugins the reference's profile
keeps), in Python.

Both only matter for pods that declare topology spread constraints / pod (anti-)affinity,
or when bound pods carry required anti-affinity terms (the symmetric rule); for every
other pod ``is_noop_for`` is true and the pod stays on the native fast path. Counting is
done once per cycle in PreFilter over the cache's bound + assumed pods.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Optional

from ..framework.interfaces import (CycleState, FilterPlugin, NodeScore, PreFilterPlugin, PreScorePlugin, ScorePlugin,
                                    StateData, Status, MAX_NODE_SCORE)
from ..models.pod import PF_POD_AFFINITY, PF_SPREAD
from ..models.selectors import LabelSelector


def _spec(pod) -> dict:
    return pod.obj.get("spec") or {}


def _node_labels(handle, node: str) -> dict:
    n = handle.cache.nodes.get(node)
    return n.labels if n is not None else {}


# ============================================================== PodTopologySpread
class _SpreadState(StateData):
    def __init__(self, hard, soft, counts, domains):
        self.hard, self.soft, self.counts, self.domains = hard, soft, counts, domains


class PodTopologySpread(PreFilterPlugin, FilterPlugin, PreScorePlugin, ScorePlugin):
    """topologySpreadConstraints: DoNotSchedule → Filter (skew ≤ maxSkew), ScheduleAnyway →
    Score (fewer matching pods in the domain scores higher)."""
    name = "PodTopologySpread"
    KEY = "PreFilterPodTopologySpread"

    pod_flags = PF_SPREAD

    def is_noop_for(self, pod) -> bool:
        return not _spec(pod).get("topologySpreadConstraints")

    def _constraints(self, pod):
        hard, soft = [], []
        for c in _spec(pod).get("topologySpreadConstraints") or []:
            item = (c.get("topologyKey", ""), int(c.get("maxSkew", 1)), LabelSelector(c.get("labelSelector")))
            (hard if c.get("whenUnsatisfiable", "DoNotSchedule") == "DoNotSchedule" else soft).append(item)
        return hard, soft

    def pre_filter(self, state: CycleState, pod) -> Status:
        hard, soft = self._constraints(pod)
        cache = self.handle.cache
        counts: dict = defaultdict(int)        # (constraint idx, domain value) → matching pods
        domains: dict = defaultdict(set)       # constraint idx → domain values that exist
        allc = hard + soft
        for node, uids in cache.node_pods.items():
            labels = _node_labels(self.handle, node)
            for ci, (key, _skew, sel) in enumerate(allc):
                if key not in labels:
                    continue
                dom = labels[key]
                domains[ci].add(dom)
                for uid in uids:
                    ps = cache.pods.get(uid)
                    if ps is not None and ps.info.namespace == pod.namespace and sel.matches(ps.info.labels):
                        counts[(ci, dom)] += 1
        for node, info in cache.nodes.items():        # nodes without pods are domains too
            for ci, (key, _s, _sel) in enumerate(allc):
                if key in info.labels:
                    domains[ci].add(info.labels[key])
        state.write(self.KEY, _SpreadState(hard, soft, counts, domains))
        return Status.ok()

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        try:
            s: _SpreadState = state.read(self.KEY)
        except KeyError:
            return Status.ok()
        labels = _node_labels(self.handle, node_name)
        for ci, (key, max_skew, sel) in enumerate(s.hard):
            if key not in labels:
                return Status.unschedulable("node(s) didn't match pod topology spread constraints (missing label)",
                                            plugin=self.name)
            self_match = 1 if sel.matches(pod.labels) else 0
            min_count = min((s.counts.get((ci, d), 0) for d in s.domains[ci]), default=0)
            if s.counts.get((ci, labels[key]), 0) + self_match - min_count > max_skew:
                return Status.unschedulable("node(s) didn't match pod topology spread constraints", plugin=self.name)
        return Status.ok()

    def pre_score(self, state: CycleState, pod, nodes: list[str]) -> Status:
        try:
            state.read(self.KEY)
        except KeyError:
            self.pre_filter(state, pod)
        return Status.ok()

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        s: _SpreadState = state.read(self.KEY)
        labels = _node_labels(self.handle, node_name)
        off = len(s.hard)
        total = 0
        for j, (key, _skew, _sel) in enumerate(s.soft):
            if key in labels:
                total += s.counts.get((off + j, labels[key]), 0)
        return total, Status.ok()

    def normalize_score(self, state: CycleState, pod, scores: list[NodeScore]) -> Status:
        if not scores:
            return Status.ok()
        hi, lo = max(x.score for x in scores), min(x.score for x in scores)
        for x in scores:
            x.score = MAX_NODE_SCORE if hi == lo else MAX_NODE_SCORE * (hi - x.score) // (hi - lo)
        return Status.ok()


# ============================================================== InterPodAffinity
def _terms(pod, kind: str, required: bool):
    aff = (_spec(pod).get("affinity") or {}).get(kind) or {}
    if required:
        return [(t, 1) for t in aff.get("requiredDuringSchedulingIgnoredDuringExecution") or []]
    return [(w.get("podAffinityTerm") or {}, int(w.get("weight", 1)))
            for w in aff.get("preferredDuringSchedulingIgnoredDuringExecution") or []]


def _term_matches(term: dict, owner_ns: str, other) -> bool:
    namespaces = term.get("namespaces") or [owner_ns]
    return other.namespace in namespaces and LabelSelector(term.get("labelSelector")).matches(other.labels)


class _AffinityState(StateData):
    def __init__(self, by_node):
        self.by_node = by_node      # node → list[PodInfo]


class InterPodAffinity(PreFilterPlugin, FilterPlugin, PreScorePlugin, ScorePlugin):
    name = "InterPodAffinity"
    KEY = "PreFilterInterPodAffinity"

    pod_flags = PF_POD_AFFINITY

    def cluster_active(self) -> bool:
        """Bound pods with required anti-affinity can reject any new pod (symmetry)."""
        return bool(self.handle.cache.pods_with_required_anti_affinity())

    def is_noop_for(self, pod) -> bool:
        aff = _spec(pod).get("affinity") or {}
        if aff.get("podAffinity") or aff.get("podAntiAffinity"):
            return False
        return not self.handle.cache.pods_with_required_anti_affinity()

    def pre_filter(self, state: CycleState, pod) -> Status:
        cache = self.handle.cache
        by_node = {n: [cache.pods[u].info for u in uids if u in cache.pods] for n, uids in cache.node_pods.items()}
        state.write(self.KEY, _AffinityState(by_node))
        return Status.ok()

    def _pods_in_domain(self, s: _AffinityState, key: str, value: str):
        for node, pods in s.by_node.items():
            if _node_labels(self.handle, node).get(key) == value:
                yield from pods

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        try:
            s: _AffinityState = state.read(self.KEY)
        except KeyError:
            self.pre_filter(state, pod)
            s = state.read(self.KEY)
        labels = _node_labels(self.handle, node_name)
        for term, _w in _terms(pod, "podAffinity", True):
            key = term.get("topologyKey", "")
            if key not in labels:
                return Status.unschedulable("node(s) didn't match pod affinity rules", plugin=self.name)
            if not any(_term_matches(term, pod.namespace, o) for o in self._pods_in_domain(s, key, labels[key])):
                # upstream: the first pod of a self-affine group may land anywhere in a domain
                if not (_term_matches(term, pod.namespace, pod) and
                        not any(_term_matches(term, pod.namespace, o) for ps in s.by_node.values() for o in ps)):
                    return Status.unschedulable("node(s) didn't match pod affinity rules", plugin=self.name)
        for term, _w in _terms(pod, "podAntiAffinity", True):
            key = term.get("topologyKey", "")
            if key in labels and any(_term_matches(term, pod.namespace, o)
                                     for o in self._pods_in_domain(s, key, labels[key])):
                return Status.unschedulable("node(s) didn't match pod anti-affinity rules", plugin=self.name)
        # symmetry: existing pods' required anti-affinity against the incoming pod
        for node, pods in s.by_node.items():
            nl = _node_labels(self.handle, node)
            for o in pods:
                for term, _w in _terms(o, "podAntiAffinity", True):
                    key = term.get("topologyKey", "")
                    if key in nl and nl.get(key) == labels.get(key) and _term_matches(term, o.namespace, pod):
                        return Status.unschedulable("node(s) didn't satisfy existing pods anti-affinity rules",
                                                    plugin=self.name)
        return Status.ok()

    def pre_score(self, state: CycleState, pod, nodes: list[str]) -> Status:
        try:
            state.read(self.KEY)
        except KeyError:
            self.pre_filter(state, pod)
        return Status.ok()

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        s: _AffinityState = state.read(self.KEY)
        labels = _node_labels(self.handle, node_name)
        total = 0
        for kind, sign in (("podAffinity", 1), ("podAntiAffinity", -1)):
            for term, w in _terms(pod, kind, False):
                key = term.get("topologyKey", "")
                if key in labels:
                    n = sum(1 for o in self._pods_in_domain(s, key, labels[key]) if _term_matches(term, pod.namespace, o))
                    total += sign * w * n
        return total, Status.ok()

    def normalize_score(self, state: CycleState, pod, scores: list[NodeScore]) -> Status:
        if not scores:
            return Status.ok()
        hi, lo = max(x.score for x in scores), min(x.score for x in scores)
        for x in scores:
            x.score = 0 if hi == lo else MAX_NODE_SCORE * (x.score - lo) // (hi - lo)
        return Status.ok()
