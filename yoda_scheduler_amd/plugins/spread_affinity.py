"""PodTopologySpread and InterPodAffinity (upstream default plugins the reference's profile
keeps).

PodTopologySpread runs natively (``native/core/engine.cpp``: ``F_SPREAD`` filter, ``S_SPREAD``
score): the engine ledger keeps every reserved pod's namespace, labels and terminating flag, the
engine holds the DefaultSelector sources (Services, RCs, ReplicaSets, StatefulSets), and each
pod's explicit constraints travel in its request — so the System default constraints a real
cluster applies to every Service-selected or controller-owned pod no longer move pods off the
native cycle. The methods below are the executable spec the native code is pinned against
(``tests/test_native_default_plugins.py``).

InterPodAffinity only matters for pods that declare pod (anti)affinity, or match a bound pod's
required anti-affinity term (the symmetric rule); for every other pod ``is_noop_for`` is true
and the pod stays on the native fast path. Counting is done once per cycle in PreFilter over the
cache's bound + assumed pods: the Python-owned ones walked here, the native lane's counted in C++
(``SchedulerCache.lane_counts``: per node, the lane pods matching a selector), so it needs no
Python copy of the lane's pods.
"""
from __future__ import annotations

import math
from collections import defaultdict
from typing import Optional

from ..framework.interfaces import (CycleState, FilterPlugin, NativeBinding, NodeScore, PreFilterPlugin,
                                    PreScorePlugin, ScorePlugin, StateData, Status, MAX_NODE_SCORE)
from ..models.pod import PF_POD_AFFINITY
from ..ops.native import core
from ..models.selectors import LabelSelector, NodeSelector
from .optional import default_selector


def _spec(pod) -> dict:
    return pod.obj.get("spec") or {}


def _node_labels(handle, node: str) -> dict:
    n = handle.cache.nodes.get(node)
    return n.labels if n is not None else {}


# ============================================================== PodTopologySpread
LABEL_HOSTNAME = "kubernetes.io/hostname"
# upstream v1.20 ``systemDefaultConstraints`` (DefaultPodTopologySpread, beta and on in v1.20)
SYSTEM_DEFAULT_CONSTRAINTS = (
    {"topologyKey": LABEL_HOSTNAME, "whenUnsatisfiable": "ScheduleAnyway", "maxSkew": 3},
    {"topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "ScheduleAnyway", "maxSkew": 5},
)


def pod_matches_node_affinity(pod, node_name: str, labels: dict) -> bool:
    """upstream ``helper.PodMatchesNodeSelectorAndAffinityTerms``: ``spec.nodeSelector``
    plus the required node-affinity terms (preferred terms are ignored)."""
    spec = _spec(pod)
    for k, v in (spec.get("nodeSelector") or {}).items():
        if labels.get(k) != v:
            return False
    req = ((spec.get("affinity") or {}).get("nodeAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution")
    if req is not None and not NodeSelector(req).matches(node_name, labels):
        return False
    return True


def _has_keys(labels: dict, constraints) -> bool:
    """upstream ``nodeLabelsMatchSpreadConstraints``: the node carries every topology key."""
    return all(c[0] in labels for c in constraints)


def _count_matching(cache, uids, sel, namespace: str) -> int:
    """upstream ``countPodsMatchSelector``: same namespace, not terminating, selector match —
    over the Python-owned pods (the lane's come from ``_lane_counts``)."""
    n = 0
    for uid in uids:
        ps = cache.pods.get(uid)
        if ps is None or ps.lane:
            continue
        info = ps.info
        if info.namespace != namespace or (info.obj.get("metadata") or {}).get("deletionTimestamp"):
            continue
        if sel.matches(info.labels):
            n += 1
    return n


def _lane_counts(cache, constraints, namespace: str) -> list:
    """Per constraint: node → lane pods matching its selector in ``namespace``, not terminating."""
    counts = getattr(cache, "lane_counts", None)
    if counts is None:                       # a cache without a native lane (tests' stand-ins)
        return [{} for _ in constraints]
    return counts([sel.native_query([namespace]) for _k, _s, sel in constraints], True)


class _SpreadFilterState(StateData):
    """upstream ``preFilterState``: the hard constraints, matching-pod count per
    (key, value) pair over the nodes that pass the pod's node affinity and carry every key,
    and the global minimum per key (``TpKeyToCriticalPaths[key][0]``)."""

    def __init__(self, constraints, pair_counts, min_count):
        self.constraints, self.pair_counts, self.min_count = constraints, pair_counts, min_count

    def clone(self) -> "_SpreadFilterState":
        return self


class _SpreadScoreState(StateData):
    """upstream ``preScoreState``: soft constraints, nodes missing a key (score 0), counts
    per non-hostname pair and ``log(size + 2)`` normalising weights."""

    def __init__(self, constraints, ignored, pair_counts, weights, lane=None):
        self.constraints, self.ignored, self.pair_counts, self.weights = constraints, ignored, pair_counts, weights
        self.lane = lane or []            # per constraint: node → matching lane pods

    def clone(self) -> "_SpreadScoreState":
        return self


def _parse_constraints(items, action: str, selector=None) -> list:
    """upstream ``filterTopologySpreadConstraints``: (topologyKey, maxSkew, selector) of the
    constraints whose ``whenUnsatisfiable`` is ``action``."""
    out = []
    for c in items or ():
        if c.get("whenUnsatisfiable", "DoNotSchedule") != action:
            continue
        sel = selector if selector is not None else LabelSelector(c.get("labelSelector"))
        out.append((c.get("topologyKey", ""), int(c.get("maxSkew", 1)), sel))
    return out


class PodTopologySpread(PreFilterPlugin, FilterPlugin, PreScorePlugin, ScorePlugin):
    """upstream v1.20 ``podtopologyspread``: ``DoNotSchedule`` constraints filter
    (matching pods in the node's domain + self − global minimum ≤ maxSkew; domains and
    counts only over nodes that pass the pod's nodeSelector/required node affinity and
    carry every key), ``ScheduleAnyway`` constraints score (Σ count·log(#domains + 2) +
    maxSkew − 1, normalised ``100·(max + min − s)/max``; nodes missing a key score 0).

    Pods without constraints get the profile's default constraints with the
    ``DefaultSelector`` of their Services / controller: ``defaultingType: System`` (the
    v1.20 default when ``defaultConstraints`` is empty) uses hostname maxSkew 3 and zone
    maxSkew 5, both ``ScheduleAnyway``; ``List`` uses ``args.defaultConstraints``."""
    name = "PodTopologySpread"
    KEY = "PreFilterPodTopologySpread"
    SCORE_KEY = "PreScorePodTopologySpread"
    watches = ("services", "replicationcontrollers", "replicasets", "statefulsets")
    # other pods read: their labels only, counted per node (the lane's natively) — no Python
    # copy of the lane's pods is needed (framework.runtime.Framework.needs_lane_mirror)
    reads_flags = 0

    def native(self):
        return NativeBinding(filter_bit=core().F_SPREAD, score_index=core().S_SPREAD)

    # Pods with these flags stay off the native lane: none. A lane pod's constraints are counted
    # and its reservation made under one engine lock (a pod with DoNotSchedule constraints is
    # never device-eligible, so no device batch drops the lock in between); a Python-path pod
    # assumed later is a later pod in upstream's serial order, which a spread constraint never
    # looks back at. The other direction — a Python-path pod's own constraints — is its
    # declared gate (``own_gate_terms``), and its final engine call re-runs this filter natively.
    lane_flags = 0

    def engine_defaults(self) -> list:
        """The default constraints as the engine takes them (``Engine.set_spread_defaults``)."""
        return [(c.get("topologyKey", ""), int(c.get("maxSkew", 1)), c.get("whenUnsatisfiable", "DoNotSchedule"))
                for c in self.default_constraints]

    def __init__(self, args: Optional[dict] = None, handle=None) -> None:
        super().__init__(args, handle)
        listed = list(self.args.get("defaultConstraints") or [])
        dtype = self.args.get("defaultingType") or ("List" if listed else "System")
        if dtype not in ("System", "List"):
            raise ValueError(f"PodTopologySpread: defaultingType must be System or List, got {dtype!r}")
        if dtype == "System" and listed:
            raise ValueError("PodTopologySpread: when defaultingType is System, defaultConstraints must be empty")
        for c in listed:
            if c.get("labelSelector") is not None:
                raise ValueError("PodTopologySpread: defaultConstraints must not set labelSelector")
            if int(c.get("maxSkew", 0)) <= 0 or not c.get("topologyKey") or \
                    c.get("whenUnsatisfiable") not in ("DoNotSchedule", "ScheduleAnyway"):
                raise ValueError(f"PodTopologySpread: invalid default constraint {c!r}")
        self.defaulting_type = dtype
        self.default_constraints = list(SYSTEM_DEFAULT_CONSTRAINTS) if dtype == "System" else listed

    def is_noop_for(self, pod) -> bool:
        if _spec(pod).get("topologySpreadConstraints"):
            return False
        if not self.default_constraints:
            return True
        return default_selector(self.handle, pod).empty

    def _constraints(self, pod, action: str) -> list:
        explicit = _spec(pod).get("topologySpreadConstraints")
        if explicit:
            return _parse_constraints(explicit, action)
        if not self.default_constraints:
            return []
        sel = default_selector(self.handle, pod)
        if sel.empty:
            return []
        return _parse_constraints(self.default_constraints, action, sel)

    def own_gate_terms(self, pod) -> list:
        """Native queries the lane must not place pods matching while this pod's cycle runs
        unparked: its hard constraints' selectors (a matching lane pod would change a skew)."""
        return [sel.native_query([pod.namespace]) for _k, _s, sel in self._constraints(pod, "DoNotSchedule")]

    def _qualified_nodes(self, pod, constraints):
        """Nodes that pass the pod's node affinity and carry every topology key."""
        for name, info in self.handle.cache.nodes.items():
            labels = info.labels
            if _has_keys(labels, constraints) and pod_matches_node_affinity(pod, name, labels):
                yield name, labels

    # ---------------------------------------------------------------- filter
    def pre_filter(self, state: CycleState, pod) -> Status:
        hard = self._constraints(pod, "DoNotSchedule")
        pair_counts: dict = {}
        min_count: dict = {}
        if hard:
            cache = self.handle.cache
            lane = _lane_counts(cache, hard, pod.namespace)
            for name, labels in self._qualified_nodes(pod, hard):
                uids = cache.node_pods.get(name, ())
                for i, (key, _skew, sel) in enumerate(hard):
                    pair = (key, labels[key])
                    pair_counts[pair] = pair_counts.get(pair, 0) + lane[i].get(name, 0) + (
                        _count_matching(cache, uids, sel, pod.namespace) if uids else 0)
            for (key, _v), n in pair_counts.items():
                if key not in min_count or n < min_count[key]:
                    min_count[key] = n
        state.write(self.KEY, _SpreadFilterState(hard, pair_counts, min_count))
        return Status.ok()

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        try:
            s: _SpreadFilterState = state.read(self.KEY)
        except KeyError:
            self.pre_filter(state, pod)
            s = state.read(self.KEY)
        if not s.constraints:
            return Status.ok()
        labels = _node_labels(self.handle, node_name)
        for key, max_skew, sel in s.constraints:
            if key not in labels:
                return Status.unresolvable("node(s) didn't match pod topology spread constraints "
                                           "(missing required label)", plugin=self.name)
            self_match = 1 if sel.matches(pod.labels) else 0
            skew = s.pair_counts.get((key, labels[key]), 0) + self_match - s.min_count.get(key, 0)
            if skew > max_skew:
                return Status.unschedulable("node(s) didn't match pod topology spread constraints", plugin=self.name)
        return Status.ok()

    # ---------------------------------------------------------------- score
    def pre_score(self, state: CycleState, pod, nodes: list[str]) -> Status:
        soft = self._constraints(pod, "ScheduleAnyway")
        ignored: set = set()
        pair_counts: dict = {}
        weights: list = []
        if soft and nodes:
            sizes = [0] * len(soft)
            for name in nodes:
                labels = _node_labels(self.handle, name)
                if not _has_keys(labels, soft):
                    ignored.add(name)
                    continue
                for i, (key, _skew, _sel) in enumerate(soft):
                    if key == LABEL_HOSTNAME:
                        continue          # per-node counts are taken in Score
                    pair = (key, labels[key])
                    if pair not in pair_counts:
                        pair_counts[pair] = 0
                        sizes[i] += 1
            for i, (key, _skew, _sel) in enumerate(soft):
                size = len(nodes) - len(ignored) if key == LABEL_HOSTNAME else sizes[i]
                weights.append(math.log(size + 2))
            cache = self.handle.cache
            lane = _lane_counts(cache, soft, pod.namespace)
            if pair_counts:
                for name, labels in self._qualified_nodes(pod, soft):
                    uids = cache.node_pods.get(name, ())
                    for i, (key, _skew, sel) in enumerate(soft):
                        pair = (key, labels[key])
                        if pair in pair_counts:
                            pair_counts[pair] += lane[i].get(name, 0) + (
                                _count_matching(cache, uids, sel, pod.namespace) if uids else 0)
        else:
            lane = []
        state.write(self.SCORE_KEY, _SpreadScoreState(soft, ignored, pair_counts, weights, lane))
        return Status.ok()

    def _score_state(self, state: CycleState, pod) -> _SpreadScoreState:
        try:
            return state.read(self.SCORE_KEY)
        except KeyError:
            self.pre_score(state, pod, list(self.handle.cache.nodes))
            return state.read(self.SCORE_KEY)

    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        s = self._score_state(state, pod)
        if not s.constraints or node_name in s.ignored:
            return 0, Status.ok()
        labels = _node_labels(self.handle, node_name)
        total = 0.0
        for i, (key, max_skew, sel) in enumerate(s.constraints):
            if key not in labels:
                continue
            if key == LABEL_HOSTNAME:
                cnt = _count_matching(self.handle.cache, self.handle.cache.node_pods.get(node_name, ()), sel,
                                      pod.namespace) + (s.lane[i].get(node_name, 0) if s.lane else 0)
            else:
                cnt = s.pair_counts.get((key, labels[key]), 0)
            total += cnt * s.weights[i] + (max_skew - 1)
        return int(total), Status.ok()

    def normalize_score(self, state: CycleState, pod, scores: list[NodeScore]) -> Status:
        s = self._score_state(state, pod)
        if not s.constraints or not scores:
            return Status.ok()
        lo, hi = None, 0
        for x in scores:
            if x.name in s.ignored:
                continue
            lo = x.score if lo is None or x.score < lo else lo
            hi = max(hi, x.score)
        for x in scores:
            if x.name in s.ignored:
                x.score = 0
            elif hi == 0:
                x.score = MAX_NODE_SCORE
            else:
                x.score = MAX_NODE_SCORE * (hi + lo - x.score) // hi
        return Status.ok()


# ============================================================== InterPodAffinity
def _terms(pod, kind: str, required: bool):
    aff = (_spec(pod).get("affinity") or {}).get(kind) or {}
    if required:
        return [(t, 1) for t in aff.get("requiredDuringSchedulingIgnoredDuringExecution") or []]
    return [(w.get("podAffinityTerm") or {}, int(w.get("weight", 1)))
            for w in aff.get("preferredDuringSchedulingIgnoredDuringExecution") or []]


# parsed selectors of affinity terms, by the term dict's identity (a pod's terms are read at
# several extension points per cycle, and against every existing pod): the entry keeps the
# dict alive, so an id is never reused while cached
_TERM_CACHE: dict = {}


def _term_entry(term: dict) -> list:
    e = _TERM_CACHE.get(id(term))
    if e is None or e[0] is not term:
        if len(_TERM_CACHE) > 4096:
            _TERM_CACHE.clear()
        e = _TERM_CACHE[id(term)] = [term, LabelSelector(term.get("labelSelector")), None, None]
    return e


def _term_matches(term: dict, owner_ns: str, other) -> bool:
    namespaces = term.get("namespaces") or [owner_ns]
    return other.namespace in namespaces and _term_entry(term)[1].matches(other.labels)


def _native_term(term: dict, owner_ns: str) -> tuple:
    e = _term_entry(term)
    if e[2] != owner_ns or e[3] is None:     # the native form depends on the owner's namespace
        e[2], e[3] = owner_ns, e[1].native(term.get("namespaces") or [owner_ns])
    return e[3]


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

    Runs natively (``native/core/engine.cpp`` ``F_INTERPOD`` / ``S_INTERPOD``, round 5): the engine
    ledger keeps every reserved pod's namespace, labels and (anti-)affinity terms, so neither an
    affinity pod nor a bound pod's required anti-affinity moves pods off the native cycle or the
    native lane, and a Python-path cycle's final engine call re-checks the rule against every pod
    placed meanwhile. The methods below are the executable spec the native code is pinned against
    (``tests/test_native_default_plugins.py``); each cycle walks the bound/assumed pods once."""
    name = "InterPodAffinity"
    KEY = "PreFilterInterPodAffinity"
    # other pods read: labels and affinity terms, which the engine ledger holds for every pod
    reads_flags = 0
    lane_flags = 0

    def __init__(self, args=None, handle=None) -> None:
        super().__init__(args, handle)
        self.hard_weight = int(self.args.get("hardPodAffinityWeight", 1))

    def native(self):
        return NativeBinding(filter_bit=core().F_INTERPOD, score_index=core().S_INTERPOD)

    def is_noop_for(self, pod) -> bool:
        aff = _spec(pod).get("affinity") or {}
        if aff.get("podAffinity") or aff.get("podAntiAffinity"):
            return False
        return not any(pod.namespace in ns and sel.matches(pod.labels) for ns, sel in self.handle.cache.anti_terms())

    def _existing(self, flags: int = 0, owned_only: bool = False):
        """(pod info, node labels) for the bound/assumed pods (with any of ``flags`` if given;
        Python-owned only if ``owned_only`` — the lane's are counted natively)."""
        cache = self.handle.cache
        for node, uids in cache.node_pods.items():
            labels = None
            for u in uids:
                ps = cache.pods.get(u)
                if ps is None or (owned_only and ps.lane) or (flags and not ps.info.flags & flags):
                    continue
                if labels is None:
                    labels = _node_labels(self.handle, node)
                yield ps.info, labels

    def _by_topology(self, counts: dict, key: str, out, weight: int = 1) -> None:
        """Add per-node lane counts into ``out[(key, value)]`` by the nodes' topology labels."""
        for node, n in counts.items():
            labels = _node_labels(self.handle, node)
            if key in labels:
                out[(key, labels[key])] += weight * n

    def pre_filter(self, state: CycleState, pod) -> Status:
        st = _AffinityState()
        aff_terms = [t for t, _ in _terms(pod, "podAffinity", True)]
        anti_terms = [t for t, _ in _terms(pod, "podAntiAffinity", True)]
        cache = self.handle.cache
        # existing pods' required anti-affinity against this pod: only pods flagged with it
        # carry such terms (the lane never takes them)
        for _o, node, terms in cache.anti_holders():
            labels = _node_labels(self.handle, node)
            for key, ns, sel in terms:
                if key in labels and pod.namespace in ns and sel.matches(pod.labels):
                    st.existing_anti[key].add(labels[key])
        # the incoming pod's terms against every existing pod: the lane's in one native pass
        queries = ([[_native_term(t, pod.namespace) for t in aff_terms]] if aff_terms else []) + \
            [[_native_term(t, pod.namespace)] for t in anti_terms]
        lane = cache.lane_counts(queries) if queries and hasattr(cache, "lane_counts") else [{} for _ in queries]
        if aff_terms:
            if lane[0]:
                for t in aff_terms:
                    self._by_topology(lane[0], t.get("topologyKey", ""), st.affinity)
            lane = lane[1:]
        for t, counts in zip(anti_terms, lane):
            self._by_topology(counts, t.get("topologyKey", ""), st.anti)
        for o, labels in (self._existing(owned_only=True) if aff_terms or anti_terms else ()):
            if aff_terms and all(_term_matches(t, pod.namespace, o) for t in aff_terms):
                for t in aff_terms:
                    key = t.get("topologyKey", "")
                    if key in labels:
                        st.affinity[(key, labels[key])] += 1
            for t in anti_terms:
                key = t.get("topologyKey", "")
                if key in labels and _term_matches(t, pod.namespace, o):
                    st.anti[(key, labels[key])] += 1
        # upstream topologyToMatchedAffinityTerms is empty: no matching pod sits on a node that
        # carries the terms' topology keys (matching pods on unlabeled nodes do not count)
        st.any_affinity_match = any(v > 0 for v in st.affinity.values())
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
        cache = self.handle.cache
        if pref:
            # incoming pod's preferred terms: the lane's pods natively, Python-owned pods below
            queries = [[_native_term(t, pod.namespace)] for t, _w, _s in pref]
            lane = cache.lane_counts(queries) if hasattr(cache, "lane_counts") else [{} for _ in queries]
            for (t, w, sign), counts in zip(pref, lane):
                key = t.get("topologyKey", "")
                for node, n in counts.items():
                    labels = _node_labels(self.handle, node)
                    if key in labels:
                        scores[key][labels[key]] += sign * w * n
            for o, labels in self._existing(owned_only=True):
                for t, w, sign in pref:
                    key = t.get("topologyKey", "")
                    if key in labels and _term_matches(t, pod.namespace, o):
                        scores[key][labels[key]] += sign * w
        for o, labels in self._existing(PF_POD_AFFINITY):
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
        # upstream v1.20 NormalizeScore: maxCount / minCount start at 0, float64 scale truncated
        hi = max(0, max(x.score for x in scores))
        lo = min(0, min(x.score for x in scores))
        for x in scores:
            x.score = int(float(MAX_NODE_SCORE) * ((x.score - lo) / (hi - lo))) if hi - lo > 0 else 0
        return Status.ok()
