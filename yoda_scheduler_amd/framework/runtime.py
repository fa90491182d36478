"""Per-profile framework: instantiates the profile's plugins and splits every extension
point into a *native* part (one engine call evaluates all nodes) and a *Python* part
(out-of-tree plugins written against :mod:`interfaces`).

A profile whose non-inert plugins are all native (the shipped yoda profile + upstream
defaults) takes the fully native cycle: one C++ call per pod — or per batch of pods —
does Filter → PreScore → Score → Normalize → selectHost → Reserve. Otherwise the
hybrid runner interleaves native node sets with the Python plugins.
"""
from __future__ import annotations

import logging
from typing import Optional

from .config import Profile
from .interfaces import (EXTENSION_POINTS, POINT_TYPES, BindPlugin, CycleState, FilterPlugin, NodeScore,
                         PermitPlugin, PostBindPlugin, PostFilterPlugin, PreBindPlugin, PreFilterPlugin,
                         PreScorePlugin, QueueSortPlugin, ReservePlugin, ScorePlugin, Status, MAX_NODE_SCORE)
from .registry import Registry

log = logging.getLogger("yoda.framework")



class Framework:
    def __init__(self, profile: Profile, registry: Registry, handle) -> None:
        self.profile = profile
        self.name = profile.scheduler_name
        self.handle = handle
        self.plugins: dict[str, object] = {}
        self.points: dict[str, list[tuple[object, int]]] = {p: [] for p in EXTENSION_POINTS}
        plugins = dict(profile.plugins)
        multi = plugins.pop("multiPoint", [])
        for point in EXTENSION_POINTS:
            refs = list(plugins.get(point, []))
            for ref in multi:
                inst = self._get(ref.name, registry)
                if isinstance(inst, POINT_TYPES[point]) and all(r.name != ref.name for r in refs):
                    refs.append(ref)
            for ref in refs:
                inst = self._get(ref.name, registry)
                if getattr(inst, "inert", False):
                    continue
                if point in ("preFilter", "preScore", "reserve") and not isinstance(inst, POINT_TYPES[point]):
                    continue   # pre-work folded into the plugin's filter/score (or the native cycle)

                if not isinstance(inst, POINT_TYPES[point]):
                    raise ValueError(f"profile {self.name}: plugin {ref.name} does not implement {point}")
                self.points[point].append((inst, ref.weight))
        qs = self.points["queueSort"]
        if len(qs) != 1:
            raise ValueError(f"profile {self.name}: exactly one queueSort plugin required, got {len(qs)}")
        self.queue_sort: QueueSortPlugin = qs[0][0]
        self.bind_plugins: list[BindPlugin] = [p for p, _ in self.points["bind"]]
        if not self.bind_plugins:
            raise ValueError(f"profile {self.name}: at least one bind plugin required")

        # native split
        from ..ops.native import core
        self.filter_mask = 0
        self.score_w = [0] * core().S_NUM
        self.filter_py: list[FilterPlugin] = []
        self.score_py: list[tuple[ScorePlugin, int]] = []
        for p, _ in self.points["filter"]:
            nb = p.native()
            if nb is not None and nb.filter_bit:
                self.filter_mask |= nb.filter_bit
                if getattr(p, "python_filter_too", False):
                    self.filter_py.append(p)      # native half + a conditional Python half
            else:
                self.filter_py.append(p)
        for p, w in self.points["score"]:
            nb = p.native()
            if nb is not None and nb.score_index >= 0:
                self.score_w[nb.score_index] += w
            else:
                self.score_py.append((p, w))
        self.pre_filter: list[PreFilterPlugin] = [p for p, _ in self.points["preFilter"] if p.native() is None]
        self.pre_score: list[PreScorePlugin] = [p for p, _ in self.points["preScore"] if p.native() is None]
        self.post_filter: list[PostFilterPlugin] = [p for p, _ in self.points["postFilter"]]
        self.reserve: list[ReservePlugin] = [p for p, _ in self.points["reserve"] if p.native() is None]
        self.permit: list[PermitPlugin] = [p for p, _ in self.points["permit"]]
        self.pre_bind: list[PreBindPlugin] = [p for p, _ in self.points["preBind"]]
        self.post_bind: list[PostBindPlugin] = [p for p, _ in self.points["postBind"]]
        self.yoda = self.plugins.get("yoda")
        # Python plugins that are no-ops for most pods (NodePorts without hostPorts,
        # PodTopologySpread without constraints, InterPodAffinity without terms) keep a
        # pod on the native path unless they actually apply to it.
        py_plugins = (self.filter_py + [p for p, _ in self.score_py] + self.pre_filter + self.pre_score + self.reserve
                      + self.permit)
        self.conditional = list({id(p): p for p in py_plugins if hasattr(p, "is_noop_for")}.values())
        static = [p for p in py_plugins if not hasattr(p, "is_noop_for")]
        self.reserve_static = [p for p in self.reserve if not hasattr(p, "is_noop_for")]
        self.fully_native_static = not static
        self.waiting: dict = {}            # pod uid → WaitingPod
        self.fully_native = self.fully_native_static and not self.conditional
        # one-mask fast path: valid when every conditional plugin declares its pod flags
        # (it is a no-op for pods without them unless its cluster gate is active)
        self._flag_mask: Optional[int] = 0
        for p in self.conditional:
            f = getattr(p, "pod_flags", None)
            if f is None:
                self._flag_mask = None
                break
            self._flag_mask |= f
        self._gates = [p.cluster_active for p in self.conditional if hasattr(p, "cluster_active")]
        # gates the native lane applies per pod from selectors (InterPodAffinity's symmetric rule)
        self._term_gates = [p for p in self.conditional if hasattr(p, "gate_terms")]
        self._plain_gates = [p.cluster_active for p in self.conditional
                             if hasattr(p, "cluster_active") and not hasattr(p, "gate_terms")]
        # native plugins that still keep some pods off the native lane (``lane_flags``: pod
        # flags, or None: no lane for this profile) and that declare gate terms for a Python
        # cycle running beside the lane (PodTopologySpread's hard constraints)
        native_plugins = {id(p): p for p, _ in self.points["filter"] + self.points["score"]
                          if p.native() is not None}.values()
        self.lane_flags: Optional[int] = 0
        for p in native_plugins:
            lf = getattr(p, "lane_flags", 0)
            if lf is None:
                self.lane_flags = None
                break
            self.lane_flags |= lf
        self._native_gaters = [p for p in native_plugins if hasattr(p, "own_gate_terms")]
        spread = self.plugins.get("PodTopologySpread")
        self._spread_defaults = spread.engine_defaults() if spread is not None and hasattr(spread, "engine_defaults") \
            else []

    def native_mask(self, lane: bool = False) -> Optional[int]:
        """For a batch of pods: the pod-flag mask such that ``native_for(pod)`` is exactly
        ``not (pod.flags & mask)``, or None when that shortcut does not hold right now (a
        plugin without declared flags, or a cluster gate is active). Evaluated once per batch
        instead of once per pod. ``lane``: for the native lane, which applies selector gates
        (``gate_terms``) per pod itself, so only the other gates count."""
        if not self.fully_native_static:
            return None
        m = self._flag_mask
        if m is None or any(g() for g in (self._plain_gates if lane else self._gates)):
            return None
        return m

    def gate_terms(self) -> tuple:
        """Native terms of the active selector gates: a pod matching one is not for the lane."""
        return tuple(t for p in self._term_gates for t in p.gate_terms())

    def own_gate_terms(self, pod) -> Optional[list]:
        """The lane gates (native queries) under which ``pod``'s Python cycle may run while
        the lane keeps placing other pods: every applying Python plugin must either ignore
        other pods or declare the pods it is sensitive to (``own_gate_terms``). None when a
        plugin cannot say (the lane must be parked for the whole cycle)."""
        out: list = []
        for p in self._native_gaters:
            out.extend(p.own_gate_terms(pod))
        for p in self._act(self._py_points(), pod):
            f = getattr(p, "own_gate_terms", None)
            if f is not None:
                out.extend(f(pod))
            elif getattr(p, "reads_flags", None) is None:
                return None
        return out

    def needs_lane_mirror(self, pod, lane_never_flags: int) -> bool:
        """Does a Python plugin that applies to ``pod`` read other pods in a way only a Python
        copy of the lane's pods can serve? Plugins declare ``reads_flags``: the features of
        other pods they read (pods of the lane never carry ``lane_never_flags``); plugins that
        count pods by selector do the lane's natively (``reads_flags = 0``). A plugin without
        the declaration (or preemption) needs the mirror."""
        for p in self._act(self._py_points(), pod):
            rf = getattr(p, "reads_flags", None)
            if rf is None or rf & ~lane_never_flags:
                return True
        return False

    def claims_ok(self) -> bool:
        """May the native lane run this profile's pods whose only lane-excluding feature is
        PF_CLAIMS, when every claim is in the lane's claim table (plugins/volumes.py::claim_lane)?
        Yes when every plugin that acts on claims — conditional or PreBind — declares that such
        claims make it a no-op or an engine filter (``claim_inert_ok``)."""
        from ..models.pod import PF_CLAIMS
        for p in list(self.conditional) + list(self.pre_bind):
            pf = getattr(p, "pod_flags", None)
            if pf is None or (pf & PF_CLAIMS and not getattr(p, "claim_inert_ok", False)):
                return False
        return any(getattr(p, "claim_inert_ok", False) for p in self.conditional)

    def direct_bind_mask(self) -> Optional[int]:
        """Likewise for ``direct_binder_for``: pods without these flags get the single bind
        plugin directly; None when the shortcut does not hold (ask per pod)."""
        if len(self.bind_plugins) != 1:
            return None
        m = 0
        for p in self.pre_bind:
            pf = getattr(p, "pod_flags", None)
            if pf is None or getattr(p, "cluster_active", None) is not None and p.cluster_active():
                return None
            m |= pf
        return m

    def native_for(self, pod) -> bool:
        if not self.fully_native_static:
            return False
        m = self._flag_mask
        if m is not None and not (pod.flags & m) and not any(g() for g in self._gates):
            return True
        # every conditional plugin a no-op for the pod: the declared-flags test first (what
        # ``_applies`` does at every extension point), ``is_noop_for`` only past it
        memo = pod.applies_memo
        if memo is not None:
            r = memo.get("native")
            if r is None:
                r = memo["native"] = not any(self._applies(p, pod) for p in self.conditional)
            return r
        return not any(self._applies_now(p, pod) for p in self.conditional)

    def _py_points(self) -> list:
        """Every plugin of the Python extension points a cycle runs, each once (built once: a
        plugin at several points would otherwise declare its gate terms several times)."""
        pts = self.__dict__.get("_py_points_l")
        if pts is None:
            seen: set = set()
            pts = self._py_points_l = [
                p for p in (self.pre_filter + self.filter_py + [q for q, _ in self.score_py] + self.pre_score
                            + self.reserve + self.permit)
                if not (id(p) in seen or seen.add(id(p)))]
        return pts

    def _act(self, plugins: list, pod) -> list:
        """The plugins of ``plugins`` (an extension point's list) that apply to ``pod``; within a
        cycle (``memo_cycle``) computed once per point."""
        memo = pod.applies_memo
        if memo is None:
            return [p for p in plugins if self._applies_now(p, pod)]
        k = ("act", id(plugins))
        r = memo.get(k)
        if r is None:
            r = memo[k] = [p for p in plugins if self._applies(p, pod)]
        return r

    @staticmethod
    def _applies(p, pod) -> bool:
        memo = pod.applies_memo
        if memo is not None:
            r = memo.get(id(p))
            if r is None:
                r = memo[id(p)] = Framework._applies_now(p, pod)
            return r
        return Framework._applies_now(p, pod)

    @staticmethod
    def memo_cycle(pod):
        """Memoise which plugins apply to ``pod`` for one scheduling cycle (a hybrid cycle asks
        the same plugin about the same pod at every extension point): a context manager."""
        import contextlib

        @contextlib.contextmanager
        def scope():
            memo = pod.applies_memo
            if memo is not None and not memo.pop("_adopt", False):   # nested (preemption inside a cycle)
                yield
                return
            if memo is None:
                pod.applies_memo = {}
            try:
                yield
            finally:
                pod.applies_memo = None
        return scope()

    @staticmethod
    def _applies_now(p, pod) -> bool:
        # one flag test for plugins that declare the pod features they act on (unless a
        # cluster-wide gate makes them relevant to every pod)
        pf = getattr(p, "pod_flags", None)
        if pf is not None and not (pod.flags & pf):
            gate = getattr(p, "cluster_active", None)
            if gate is None or not gate():
                return False
        f = getattr(p, "is_noop_for", None)
        return f is None or not f(pod)

    def _get(self, name: str, registry: Registry):
        inst = self.plugins.get(name)
        if inst is None:
            inst = registry.create(name, self.profile.plugin_config.get(name, {}), self.handle)
            if hasattr(inst, "bind_framework"):
                inst.bind_framework(self)
            self.plugins[name] = inst
        return inst

    # ------------------------------------------------------------------ engine config
    def apply(self, engine) -> None:
        engine.filters = self.filter_mask
        for i, w in enumerate(self.score_w):
            engine.set_score_weight(i, w)
        for most, name in ((False, "NodeResourcesLeastAllocated"), (True, "NodeResourcesMostAllocated")):
            p = self.plugins.get(name)
            engine.set_alloc_weights(most, *(p.alloc_weights() if p is not None else (1, 1, 0)))
        engine.set_spread_defaults(self._spread_defaults)
        ipa = self.plugins.get("InterPodAffinity")
        engine.set_hard_pod_affinity_weight(getattr(ipa, "hard_weight", 1) if ipa is not None else 1)
        fit = self.plugins.get("NodeResourcesFit")
        engine.set_ext_ignored(*(fit.engine_ignored() if fit is not None and hasattr(fit, "engine_ignored")
                                 else ([], [])))
        if self.yoda is not None:
            self.yoda.configure_engine(engine)

    # ------------------------------------------------------------------ Python points
    def run_pre_filter(self, state: CycleState, pod) -> Status:
        for p in self._act(self.pre_filter, pod):
            st = p.pre_filter(state, pod)
            if not st.is_success():
                st.plugin = st.plugin or p.name
                return st
        return Status.ok()

    def passes_py_filters(self, pod, node: str) -> bool:
        """Upstream ``PodPassesFiltersOnNode`` for the Python side of a profile: PreFilter
        over the cache as it stands (state rebuilt, which equals upstream's AddPod /
        RemovePod extensions applied to the cycle state), then the Python filters on
        ``node``. The native filters are checked by the caller."""
        state = CycleState()
        if not self.run_pre_filter(state, pod).is_success():
            return False
        ok, _ = self.run_filter_py(state, pod, [node])
        return bool(ok)

    def has_active_filter_py(self, pod) -> bool:
        return bool(self._act(self.filter_py, pod))

    def run_filter_py(self, state: CycleState, pod, nodes: list[str],
                      limit: Optional[int] = None) -> tuple[list[str], dict]:
        """Python filters over the native-feasible ``nodes``; stops once ``limit`` nodes
        passed (numFeasibleNodesToFind)."""
        if not self.filter_py:
            return nodes, {}
        out, failed = [], {}
        active = self._act(self.filter_py, pod)
        if not active:
            return nodes, {}
        for n in nodes:
            if limit is not None and len(out) >= limit:
                break
            for p in active:
                st = p.filter(state, pod, n)
                if not st.is_success():
                    failed[n] = st
                    break
            else:
                out.append(n)
        return out, failed

    def run_score_py(self, state: CycleState, pod, nodes: list[str]) -> list[int]:
        total = [0] * len(nodes)
        for p in self._act(self.pre_score, pod):
            st = p.pre_score(state, pod, nodes)
            if not st.is_success():
                raise RuntimeError(f"preScore {p.name}: {st.message()}")
        for p, w in self.score_py:
            if not self._applies(p, pod):
                continue
            scores = []
            for n in nodes:
                s, st = p.score(state, pod, n)
                if not st.is_success():
                    raise RuntimeError(f"score {p.name}: {st.message()}")
                scores.append(NodeScore(n, s))
            if p.has_normalize():
                st = p.normalize_score(state, pod, scores)
                if not st.is_success():
                    raise RuntimeError(f"normalize {p.name}: {st.message()}")
            for i, ns in enumerate(scores):
                if not 0 <= ns.score <= MAX_NODE_SCORE:
                    raise RuntimeError(f"plugin {p.name} returned out-of-range score {ns.score}")
                total[i] += ns.score * w
        return total

    def run_reserve(self, state: CycleState, pod, node: str) -> Status:
        active = self._act(self.reserve, pod)
        for i, p in enumerate(active):
            st = p.reserve(state, pod, node)
            if not st.is_success():
                for q in reversed(active[:i]):
                    q.unreserve(state, pod, node)
                return st
        return Status.ok()

    def run_unreserve(self, state: CycleState, pod, node: str) -> None:
        for p in reversed(self.reserve):
            if self._applies(p, pod):
                p.unreserve(state, pod, node)

    def run_permit(self, state: CycleState, pod, node: str) -> tuple[Status, float]:
        """Returns success, a rejection, or WAIT (the pod is registered in ``waiting``;
        the binding cycle awaits it)."""
        from .interfaces import Code, WaitingPod
        wait, waiters = 0.0, set()
        for p in self._act(self.permit, pod):
            st, t = p.permit(state, pod, node)
            if st.code == Code.WAIT:
                waiters.add(p.name)
                wait = max(wait, t)
            elif not st.is_success():
                st.plugin = st.plugin or p.name
                return st, 0.0
        if waiters:
            self.waiting[pod.uid] = WaitingPod(pod, node, waiters, wait)
            return Status(Code.WAIT, [], ""), wait
        return Status.ok(), 0.0

    def get_waiting_pod(self, uid: str):
        return self.waiting.get(uid)

    def iterate_waiting_pods(self):
        return list(self.waiting.values())

    async def wait_on_permit(self, pod) -> Status:
        wp = self.waiting.get(pod.uid)
        if wp is None:
            return Status.ok()
        try:
            return await wp.wait()
        finally:
            self.waiting.pop(pod.uid, None)

    def direct_binder_for(self, pod):
        """``direct_binder`` for one pod: PreBind plugins that are no-ops for it do not count."""
        if len(self.bind_plugins) != 1:
            return None
        for p in self.pre_bind:
            if self._applies(p, pod):
                return None
        return self.bind_plugins[0]

    def direct_binder(self):
        """The single bind plugin when nothing runs around it (no PreBind plugins): the
        bind workers then await it directly instead of going through ``run_bind``."""
        if not self.pre_bind and len(self.bind_plugins) == 1:
            return self.bind_plugins[0]
        return None

    async def run_bind(self, state: CycleState, pod, node: str, extender=None) -> Status:
        for p in self.pre_bind:
            if not self._applies(p, pod):
                continue
            st = await p.pre_bind(state, pod, node)
            if not st.is_success():
                return st
        if extender is not None:           # upstream extendersBinding: the extender binds
            try:
                await extender.bind(pod, node)
            except Exception as e:  # noqa: BLE001 - surfaced as a bind failure
                return Status.error(f"extender bind: {e}")
            return Status.ok()
        for p in self.bind_plugins:
            st = await p.bind(state, pod, node)
            if st.code.name == "SKIP":
                continue
            return st
        return Status.error("no bind plugin bound the pod")

    @property
    def post_bind_noop(self) -> bool:
        return not self.post_bind

    def run_post_bind(self, state: CycleState, pod, node: str) -> None:
        for p in self.post_bind:
            p.post_bind(state, pod, node)
