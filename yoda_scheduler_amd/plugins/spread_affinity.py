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
        # global minimum matching count per hard constraint (computed once, not per node)
        self.min_count = [min((counts.get((ci, d), 0) for d in domains[ci]), default=0) for ci in range(len(hard))]


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
            if s.counts.get((ci, labels[key]), 0) + self_match - s.min_count[ci] > max_skew:
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
    """Topology-pair counts computed once per cycle (upstream ``preFilterState``):
    ``existing_anti``: (key, value) domains where an existing pod's required anti-affinity
    matches the incoming pod; ``affinity`` / ``anti``: per required term of the incoming pod,
    the (key, value) domains holding pods that match it; ``scores``: (key, value) → weight
    for the preferred terms (both directions) and existing pods' required affinity
    (``hardPodAffinityWeight``)."""

    def __init__(self) -> None:
        self.existing_anti: dict = defaultdict(set)     # topology key → values with a blocking pod
        self.affinity: dict = defaultdict(int)
        self.any_affinity_match = False
        self.anti: dict = defaultdict(int)
        self.aff_terms: list = []
        self.anti_terms: list = []
        self.scores: Optional[dict] = None      # topology key → value → weight

    def clone(self) -> "_AffinityState":
        return self


class InterPodAffinity(PreFilterPlugin, FilterPlugin, PreScorePlugin, ScorePlugin):
    """Required pod (anti-)affinity as a filter (incl. the symmetric rule for existing
    pods' required anti-affinity), preferred terms + ``hardPodAffinityWeight`` as a score.
    Each cycle walks the bound/assumed pods once; per-node work is a few dict lookups."""
    name = "InterPodAffinity"
    KEY = "PreFilterInterPodAffinity"

    pod_flags = PF_POD_AFFINITY

    def __init__(self, args=None, handle=None) -> None:
        super().__init__(args, handle)
        self.hard_weight = int(self.args.get("hardPodAffinityWeight", 1))

    def cluster_active(self) -> bool:
        """Bound pods with required anti-affinity can reject any new pod (symmetry)."""
        return bool(self.handle.cache.pods_with_required_anti_affinity())

    def is_noop_for(self, pod) -> bool:
        aff = _spec(pod).get("affinity") or {}
        if aff.get("podAffinity") or aff.get("podAntiAffinity"):
            return False
        return not self.handle.cache.pods_with_required_anti_affinity()

    def _existing(self):
        """(pod info, node labels) for every bound/assumed pod."""
        cache = self.handle.cache
        for node, uids in cache.node_pods.items():
            labels = _node_labels(self.handle, node)
            for u in uids:
                ps = cache.pods.get(u)
                if ps is not None:
                    yield ps.info, labels

    def pre_filter(self, state: CycleState, pod) -> Status:
        st = _AffinityState()
        aff_terms = [t for t, _ in _terms(pod, "podAffinity", True)]
        anti_terms = [t for t, _ in _terms(pod, "podAntiAffinity", True)]
        for o, labels in self._existing():
            for term, _w in _terms(o, "podAntiAffinity", True):
                key = term.get("topologyKey", "")
                if key in labels and _term_matches(term, o.namespace, pod):
                    st.existing_anti[key].add(labels[key])
            if aff_terms and all(_term_matches(t, pod.namespace, o) for t in aff_terms):
                st.any_affinity_match = True
                for t in aff_terms:
                    key = t.get("topologyKey", "")
                    if key in labels:
                        st.affinity[(key, labels[key])] += 1
            for t in anti_terms:
                key = t.get("topologyKey", "")
                if key in labels and _term_matches(t, pod.namespace, o):
                    st.anti[(key, labels[key])] += 1
        st.aff_terms, st.anti_terms = aff_terms, anti_terms
        state.write(self.KEY, st)
        return Status.ok()

    def _state(self, state: CycleState, pod) -> _AffinityState:
        try:
            return state.read(self.KEY)
        except KeyError:
            self.pre_filter(state, pod)
            return state.read(self.KEY)

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        st = self._state(state, pod)
        labels = _node_labels(self.handle, node_name)
        for key, values in st.existing_anti.items():
            if key in labels and labels[key] in values:
                return Status.unschedulable("node(s) didn't satisfy existing pods anti-affinity rules",
                                            plugin=self.name)
        if st.aff_terms:
            ok = all(k in labels and st.affinity.get((k, labels[k]), 0) > 0
                     for k in (t.get("topologyKey", "") for t in st.aff_terms))
            if not ok:
                # upstream: the first pod of a self-affine group may go to any node that has
                # the topology keys, when no existing pod matches the terms yet
                first = (not st.any_affinity_match and all(_term_matches(t, pod.namespace, pod) for t in st.aff_terms)
                         and all(t.get("topologyKey", "") in labels for t in st.aff_terms))
                if not first:
                    return Status.unschedulable("node(s) didn't match pod affinity rules", plugin=self.name)
        for t in st.anti_terms:
            k = t.get("topologyKey", "")
            if k in labels and st.anti.get((k, labels[k]), 0) > 0:
                return Status.unschedulable("node(s) didn't match pod anti-affinity rules", plugin=self.name)
        return Status.ok()

    def pre_score(self, state: CycleState, pod, nodes: list[str]) -> Status:
        st = self._state(state, pod)
        scores: dict = defaultdict(lambda: defaultdict(int))
        pref = [(t, w, 1) for t, w in _terms(pod, "podAffinity", False)] + \
               [(t, w, -1) for t, w in _terms(pod, "podAntiAffinity", False)]
        for o, labels in self._existing():
            for t, w, sign in pref:                     # incoming pod's preferred terms
                key = t.get("topologyKey", "")
                if key in labels and _term_matches(t, pod.namespace, o):
                    scores[key][labels[key]] += sign * w
            if self.hard_weight:                        # existing pods' required affinity
                for t, _w in _terms(o, "podAffinity", True):
                    key = t.get("topologyKey", "")
                    if key in labels and _term_matches(t, o.namespace, pod):
                        scores[key][labels[key]] += self.hard_weight
            for kind, sign in (("podAffinity", 1), ("podAntiAffinity", -1)):   # existing preferred
                for t, w in _terms(o, kind, False):
                    key = t.get("topologyKey", "")
                    if key in labels and _term_matches(t, o.namespace, pod):
                        scores[key][labels[key]] += sign * w
        st.scores = scores
        return Status.ok()

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        st = self._state(state, pod)
        if st.scores is None:
            self.pre_score(state, pod, [])
        labels = _node_labels(self.handle, node_name)
        return sum(by_val.get(labels.get(k), 0) for k, by_val in st.scores.items()), Status.ok()

    def normalize_score(self, state: CycleState, pod, scores: list[NodeScore]) -> Status:
        if not scores:
            return Status.ok()
        hi, lo = max(x.score for x in scores), min(x.score for x in scores)
        for x in scores:
            x.score = 0 if hi == lo else MAX_NODE_SCORE * (x.score - lo) // (hi - lo)
        return Status.ok()
