"""In-tree default plugins (the upstream v1.20 set the reference's profile keeps).

Hot filters/scores are *native*: they declare an engine binding and run inside the
C++ cycle (``native/core/engine.cpp``). The object-dependent ones — topology spread and
inter-pod affinity (``spread_affinity.py``), the volume plugins (``volumes.py``),
ImageLocality and NodePreferAvoidPods (``node_extras.py``) — are Python plugins that are
no-ops for pods they do not apply to, so those pods stay on the native path. The
registered-but-not-default v1.20 plugins (NodeLabel, ServiceAffinity, SelectorSpread,
RequestedToCapacityRatio) live in ``optional.py``, CinderLimits in ``volumes.py``. Only
``CSILimits`` (a pre-1.17 name of NodeVolumeLimits) is registered as inert so older
configs still load.
"""
from __future__ import annotations

import time

from typing import Optional

from ..framework.interfaces import (BindPlugin, CycleState, FilterPlugin, NativeBinding, Plugin,
                                    PostFilterPlugin, PostFilterResult, QueueSortPlugin, ScorePlugin, Status)
from ..models.labels import ANNOTATION_GPU_UUIDS, ANNOTATION_GPUS, ANNOTATION_RESERVED, ANNOTATION_VISIBLE
from ..models.scv import LazyScv, card_vis
from ..ops.native import core


def _c():
    return core()


class PrioritySort(QueueSortPlugin):
    """``.spec.priority`` desc, then enqueue order (upstream PrioritySort)."""
    name = "PrioritySort"

    def sort_key(self, pi) -> tuple:
        return (-pi.priority,)


class NodeUnschedulable(FilterPlugin):
    name = "NodeUnschedulable"

    def native(self):
        return NativeBinding(filter_bit=_c().F_NODE_UNSCHEDULABLE)


class NodeName(FilterPlugin):
    name = "NodeName"

    def native(self):
        return NativeBinding(filter_bit=_c().F_NODE_NAME)


class NodeResourcesFit(FilterPlugin):
    """Natively: cpu / memory / pod count and everything else a pod requests (``amd.com/gpu``
    from the AMD device plugin, ``ephemeral-storage``, hugepages, other extended resources)
    against the node's allocatable and the engine ledger's per-node usage
    (``native/core/engine.cpp`` ``RS_EXT_RESOURCES``), so ``PF_EXTENDED`` pods stay on the
    native cycle and the native lane. ``ignoredResources`` / ``ignoredResourceGroups`` args as
    upstream (``Engine.set_ext_ignored``). ``filter`` below is the executable spec of the
    extended-resource check (``tests/test_native_default_plugins.py``)."""
    name = "NodeResourcesFit"
    reads_flags = 0  # other pods' features this plugin reads (needs_lane_mirror)

    def __init__(self, args: Optional[dict] = None, handle=None) -> None:
        super().__init__(args, handle)
        self.ignored = set(self.args.get("ignoredResources") or [])
        self.ignored_groups = set(self.args.get("ignoredResourceGroups") or [])

    def native(self):
        return NativeBinding(filter_bit=_c().F_NODE_RESOURCES_FIT)

    def _checked(self, res: str) -> bool:
        return res not in self.ignored and res.split("/", 1)[0] not in self.ignored_groups

    def engine_ignored(self) -> tuple[list, list]:
        return sorted(self.ignored), sorted(self.ignored_groups)

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        cache = self.handle.cache
        node = cache.nodes.get(node_name)
        alloc = node.ext_alloc if node is not None else {}
        used = cache.node_ext_used.get(node_name, {})
        short = [r for r, v in pod.ext.items() if self._checked(r) and used.get(r, 0) + v > alloc.get(r, 0)]
        if short:
            return Status.unschedulable(*(f"Insufficient {r}" for r in sorted(short)), plugin=self.name)
        return Status.ok()


class NodeAffinity(FilterPlugin, ScorePlugin):
    name = "NodeAffinity"

    def native(self):
        return NativeBinding(filter_bit=_c().F_NODE_AFFINITY, score_index=_c().S_NODE_AFFINITY)


class TaintToleration(FilterPlugin, ScorePlugin):
    name = "TaintToleration"

    def native(self):
        return NativeBinding(filter_bit=_c().F_TAINT_TOLERATION, score_index=_c().S_TAINT_TOLERATION)


def _alloc_weights(args: dict) -> tuple[int, int, int]:
    """``resources: [{name, weight}]`` → (cpu, memory, Σ others); default cpu=memory=1."""
    res = args.get("resources")
    if not res:
        return 1, 1, 0
    w = {r.get("name", ""): int(r.get("weight", 1)) for r in res}
    return w.pop("cpu", 0), w.pop("memory", 0), sum(w.values())


class NodeResourcesLeastAllocated(ScorePlugin):
    name = "NodeResourcesLeastAllocated"

    def alloc_weights(self) -> tuple[int, int, int]:
        return _alloc_weights(self.args)

    def native(self):
        return NativeBinding(score_index=_c().S_LEAST_ALLOCATED)


class NodeResourcesMostAllocated(ScorePlugin):
    name = "NodeResourcesMostAllocated"

    def alloc_weights(self) -> tuple[int, int, int]:
        return _alloc_weights(self.args)

    def native(self):
        return NativeBinding(score_index=_c().S_MOST_ALLOCATED)


class NodeResourcesBalancedAllocation(ScorePlugin):
    name = "NodeResourcesBalancedAllocation"

    def native(self):
        return NativeBinding(score_index=_c().S_BALANCED_ALLOCATION)


class NodePorts(FilterPlugin):
    """Host-port conflicts with the pods on the node, natively (engine ``F_NODE_PORTS``: the
    ledger keeps every reserved pod's host ports per node), so hostPort / hostNetwork pods —
    multi-node training pods on RDMA fabrics run with ``hostNetwork: true``, which gives every
    container port a host port — stay on the native cycle and the native lane. ``filter``
    below is the executable spec (upstream v1.20 ``HostPortInfo.CheckConflict``), pinned by
    ``tests/test_native_default_plugins.py``."""
    name = "NodePorts"
    reads_flags = 0  # other pods' features this plugin reads (needs_lane_mirror): native

    def native(self):
        return NativeBinding(filter_bit=_c().F_NODE_PORTS)

    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        want = host_port_set(pod.host_ports)
        if not want:
            return Status.ok()
        cache = self.handle.cache
        used: set = set()
        for uid in cache.node_pods.get(node_name, ()):
            ps = cache.pods.get(uid)
            if ps is not None:
                used |= host_port_set(ps.info.host_ports)
        any_ip = {(proto, port) for _ip, proto, port in used}
        for ip, proto, port in want:
            if ip == "0.0.0.0":
                hit = (proto, port) in any_ip
            else:
                hit = ("0.0.0.0", proto, port) in used or (ip, proto, port) in used
            if hit:
                return Status.unschedulable("node(s) didn't have free ports for the requested pod ports",
                                            plugin=self.name)
        return Status.ok()


def host_port_set(ports) -> set:
    """(hostIP, protocol, hostPort) of a pod's host ports as upstream HostPortInfo keeps them:
    hostIP "" → "0.0.0.0", protocol "" → "TCP", ports <= 0 dropped."""
    out = set()
    for port, proto, ip in ports or ():
        if isinstance(port, int) and not isinstance(port, bool) and 0 < port <= 0x7FFFFFFF:
            out.add((ip or "0.0.0.0", proto or "TCP", port))
    return out


class _Inert(Plugin):
    inert = True


def _inert(name: str):
    return type(name, (_Inert,), {"name": name})


INERT_PLUGINS = ["CSILimits"]


def visible_device_ids(scv, cards: list) -> tuple[str, str]:
    """(ROCR_VISIBLE_DEVICES value, amd-smi UUID list) for the assigned card positions of a
    node's Scv. Per card: ROCr UUID, else HIP ordinal, else the amd-smi index."""
    if scv is None:
        per = ()
    elif isinstance(scv, LazyScv):             # computed once per Scv version
        per = scv.card_vis()
    else:
        per = card_vis([(c.id, c.uuid, c.hip_uuid, c.hip_id) for c in scv.status.card_list])
    n = len(per)
    vis, uuids = [], []
    for c in cards:
        if 0 <= c < n:
            v, u = per[c]
            vis.append(v)
            if u:
                uuids.append(u)
        else:
            vis.append(str(c))
    return ",".join(vis), (",".join(uuids) if len(uuids) == len(cards) else "")


def bind_annotations(pod, scvs: Optional[dict] = None, node: str = "") -> list:
    """(key, value) pairs the Binding carries: the GPU assignment (amd-smi indices, the
    ROCr-visible ids, the device UUIDs) and the per-GPU HBM reserve."""
    cards = getattr(pod, "assigned_cards", None)
    if cards is None:
        return []
    ann = [(ANNOTATION_GPUS, ",".join(map(str, cards)))]
    vis, uuids = visible_device_ids((scvs or {}).get(node), cards)
    ann.append((ANNOTATION_VISIBLE, vis))
    if uuids:
        ann.append((ANNOTATION_GPU_UUIDS, uuids))
    if pod.gpu.has_memory:
        ann.append((ANNOTATION_RESERVED, str(pod.gpu.memory)))
    return ann


class DefaultBinder(BindPlugin):
    """POST pods/{name}/binding; the GPU assignment rides on the Binding's annotations,
    which the apiserver copies onto the pod (one round trip, no extra patch). With the
    native transport the scheduler submits this same POST directly (``native_bind``)."""
    name = "DefaultBinder"
    native_bind = True

    async def bind(self, state: CycleState, pod, node_name: str) -> Status:
        ann = dict(bind_annotations(pod, self.handle.cache.scvs, node_name))
        try:
            await self.handle.client.bind(pod.namespace, pod.name, pod.uid, node_name, ann)
        except Exception as e:  # noqa: BLE001 - surfaced as a bind failure
            return Status.error(f"binding rejected: {e}", plugin=self.name)
        return Status.ok()


class DefaultPreemption(PostFilterPlugin):
    """Evict lower-priority pods so a high-priority pod fits (GPU-aware), upstream v1.20
    ``selectVictimsOnNode`` + ``pickOneNodeForPreemption`` semantics on the native ledger:

    * per node: take every lower-priority pod off the ledger (a what-if); if the pod still
      does not fit, the node is no candidate. Otherwise *reprieve* victims, PDB-violating
      ones first and then by descending priority, re-adding each one that leaves the pod
      still fitting — what remains are the victims;
    * candidates are ranked by fewest PodDisruptionBudget violations, lowest highest-victim
      priority, lowest sum of victim priorities, fewest victims;
    * a pod whose nominated node still has terminating lower-priority pods waits instead
      of preempting again (``PodEligibleToPreemptOthers``).

    Victims are deleted through the API and the preemptor is nominated to the node; the
    ledger is restored exactly before returning. When the pod uses a Python filter plugin
    of the profile (pod (anti-)affinity, topology spread, host ports, volumes) each what-if
    also hides the removed pods from the cache and re-runs PreFilter + those filters, so a
    victim whose removal satisfies e.g. required anti-affinity is found (upstream's
    ``RunPreFilterExtensionRemovePod`` / ``AddPod``).
    """
    name = "DefaultPreemption"
    watches = ("poddisruptionbudgets",)
    framework = None
    # process-wide: PostFilter calls, the ones that nominated a node, victims, seconds spent
    # (bench.py --mix-preempt reports them)
    stats = {"calls": 0, "nominated": 0, "victims": 0, "seconds": 0.0}

    def bind_framework(self, fw) -> None:
        self.framework = fw

    def _pdbs(self) -> list:
        from ..models.selectors import LabelSelector
        out = []
        for o in self.handle.lister("poddisruptionbudgets").values():
            m = o.get("metadata") or {}
            allowed = int(((o.get("status") or {}).get("disruptionsAllowed")) or 0)
            out.append((m.get("namespace", "default"), LabelSelector((o.get("spec") or {}).get("selector") or {}),
                        allowed))
        return out

    def _eligible(self, pod) -> bool:
        if (pod.obj.get("spec") or {}).get("preemptionPolicy") == "Never":
            return False
        nominated = ((pod.obj.get("status") or {}).get("nominatedNodeName")) or ""
        if not nominated:
            return True
        cache = self.handle.cache
        for u in cache.node_pods.get(nominated, ()):
            ps = cache.pods.get(u)
            if ps is not None and ps.info.priority < pod.priority and \
                    (ps.info.obj.get("metadata") or {}).get("deletionTimestamp"):
                return False
        return True

    def _python_filters(self, pod) -> bool:
        """A Python filter or PreFilter of the profile applies to the pod: the what-if must
        re-run them (the Python path below); otherwise the engine's native search decides."""
        fw = self.framework
        return fw is not None and (fw.has_active_filter_py(pod) or any(fw._applies(p, pod) for p in fw.pre_filter))

    def needs_mirror(self, pod) -> bool:
        """The Python what-if walks the cache's pods (lane pods mirrored into it); the native
        search reads the engine ledger, which holds every pod."""
        return self._python_filters(pod) or not hasattr(self.handle.engine, "preempt")

    def _native(self, pod, req, pdbs) -> tuple[Optional[PostFilterResult], Status]:
        """upstream v1.20 preemption in the engine (Engine::preempt): nodesWherePreemptionMightHelp
        (nodes whose first failing filter is UnschedulableAndUnresolvable are skipped), at most
        max(minCandidateNodesPercentage % of them, minCandidateNodesAbsolute) candidates dry-run
        from a random offset, selectVictimsOnNode's reprieve order (PDB-violating first, then by
        importance) and pickOneNodeForPreemption's ranking — on the ledger, lane pods included."""
        h = self.handle
        eng, cache = h.engine, h.cache
        pct = int(self.args.get("minCandidateNodesPercentage", 10))
        absolute = int(self.args.get("minCandidateNodesAbsolute", 100))
        native_pdbs = [(ns, sel.native(), allowed) for ns, sel, allowed in pdbs]
        node_idx, ids, cards, _viol, *_ = eng.preempt(req, pod.priority, native_pdbs, pct, absolute)
        if node_idx < 0:
            return None, Status.unschedulable("preemption: no node can be freed", plugin=self.name)
        node = eng.node_name(node_idx)
        want = set(ids)
        victims = []
        for uid in cache.node_pods.get(node, ()):        # Python-owned pods on the node
            ps = cache.pods.get(uid)
            if ps is not None and ps.info.num_id in want:
                victims.append(ps.info)
                want.discard(ps.info.num_id)
        lane = getattr(cache, "lane", None)
        if want and lane is not None:                   # lane-owned pods: the lane's store
            from ..models.pod import PodInfo
            for lid in sorted(want):
                got = lane.lookup_id(lid)
                if got is not None:
                    victims.append(PodInfo.from_native(got[0]))
        h.preempt(pod, node, victims)
        DefaultPreemption.stats["victims"] += len(victims)
        return PostFilterResult(node, list(cards)), Status.ok()

    def post_filter(self, state: CycleState, pod, statuses: dict) -> tuple[Optional[PostFilterResult], Status]:
        t0 = time.perf_counter()
        r, st = self._post_filter(state, pod, statuses)
        S = DefaultPreemption.stats
        S["calls"] += 1
        S["seconds"] += time.perf_counter() - t0
        if r is not None and r.nominated_node:
            S["nominated"] += 1
        return r, st

    def _post_filter(self, state: CycleState, pod, statuses: dict) -> tuple[Optional[PostFilterResult], Status]:
        h = self.handle
        if pod.priority <= 0 and not self.args.get("preemptZeroPriority", False):
            return None, Status.unschedulable("preemption: pod has no priority", plugin=self.name)
        if not self._eligible(pod):
            return None, Status.unschedulable("preemption: pod is not eligible (preemptionPolicy Never, or victims"
                                              " on its nominated node are still terminating)", plugin=self.name)
        eng, cache = h.engine, h.cache
        from ..ops.native import pod_req
        req = pod_req(eng, pod)
        pdbs = self._pdbs()
        fw = self.framework
        py = self._python_filters(pod)
        if not py and hasattr(eng, "preempt"):
            return self._native(pod, req, pdbs)
        pct = int(self.args.get("minCandidateNodesPercentage", 10))
        absolute = int(self.args.get("minCandidateNodesAbsolute", 100))

        def fits(node: str, idx: int) -> bool:
            return eng.filter_node(req, idx) == 0 and (not py or fw.passes_py_filters(pod, node))

        best = preempt_spec(eng, cache, pod, req, pdbs, pct, absolute, fits=fits, hide=py)
        if best is None:
            return None, Status.unschedulable("preemption: no node can be freed", plugin=self.name)
        node, victims, cards = best
        h.preempt(pod, node, [v.info for v in victims])
        DefaultPreemption.stats["victims"] += len(victims)
        return PostFilterResult(node, cards), Status.ok()


# upstream v1.20 filter order and whether a failure is UnschedulableAndUnresolvable (preemption
# cannot help): the native engine's plugin bits with the reason names each reports
_PREEMPT_ORDER = ("F_NODE_UNSCHEDULABLE", "F_NODE_RESOURCES_FIT", "F_NODE_NAME", "F_NODE_PORTS", "F_NODE_AFFINITY",
                  "F_TAINT_TOLERATION", "F_SPREAD", "F_INTERPOD", "F_YODA")
_UNRESOLVABLE = frozenset({"NodeUnschedulable", "NodeName", "NodeAffinity", "TaintToleration", "VolumeBinding",
                           "VolumeZone", "PodTopologySpreadLabel", "InterPodAffinity", "NoScv", "ScvStale", "NodeGone"})


def preemption_might_help(eng, req, idx: int) -> bool:
    """nodesWherePreemptionMightHelp for one node: the first failing filter in upstream order is
    not UnschedulableAndUnresolvable (a node that passes counts too). The engine evaluates one
    plugin at a time (its ``filters`` mask), so the order here is upstream's, not the engine's."""
    from ..ops.native import core
    C = core()
    saved = eng.filters
    try:
        for name in _PREEMPT_ORDER:
            bit = getattr(C, name)
            if not saved & bit:
                continue
            eng.filters = bit
            r = C.REASONS[eng.filter_node(req, idx)]
            if r != "OK":
                return r not in _UNRESOLVABLE
        return True
    finally:
        eng.filters = saved


def preempt_spec(eng, cache, pod, req, pdbs: list, pct: int = 10, absolute: int = 100, offset: int = -1,
                 fits=None, hide: bool = False, rng=None):
    """Python spec of upstream v1.20 preemption over the engine ledger (``Engine::preempt`` is
    its native twin; tests/test_preemption_native.py pins the two together):

    * potential nodes: ``preemption_might_help``; ``numCandidates`` = max(``pct`` % of them,
      ``absolute``) capped at their count; dry-run from ``offset`` (random when < 0), wrapping,
      until a non-violating candidate exists and the candidates reach ``numCandidates``;
    * selectVictimsOnNode: every lower-priority pod off the node (a what-if); no fit → no
      candidate. Otherwise the pods by MoreImportantPod (priority, then earlier start = earlier
      reservation), PDB budgets consumed in that order, PDB-violating ones reprieved first;
    * pickOneNodeForPreemption: fewest PDB violations, lowest highest victim priority, lowest
      Σ (priority + 2^31), fewest victims, latest earliest start among the top-priority victims,
      then the first (non-violating candidates before violating ones).

    Returns (node, victims [PodState], cards) or None."""
    import random as _random
    fits = fits or (lambda node, idx: eng.filter_node(req, idx) == 0)
    names = {}
    potential = []
    for node in cache.nodes:
        idx = eng.node_index(node)
        if idx >= 0:
            names[idx] = node
    for idx in sorted(names):
        if preemption_might_help(eng, req, idx):
            potential.append(idx)
    if not potential:
        return None
    np_ = len(potential)
    want = min(max(np_ * pct // 100, absolute), np_)
    start = offset % np_ if offset >= 0 else (rng or _random).randrange(np_)
    nonviol, viol = [], []
    for k in range(np_):
        idx = potential[(start + k) % np_]
        node = names[idx]
        lower = []
        for u in cache.node_pods.get(node, ()):
            ps = cache.pods.get(u)
            info = eng.assignment_info(ps.info.num_id) if ps is not None else None
            if info is not None and info[0] == idx and info[4] < pod.priority:
                lower.append((ps, info[3], info[4]))
        if lower:
            for ps, _t, _p in lower:
                eng.detach_pod(ps.info.num_id)
            if hide:
                cache.hide([ps.info.uid for ps, _t, _p in lower])
            try:
                if not fits(node, idx):
                    for ps, _t, _p in lower:
                        eng.attach_pod(ps.info.num_id)
                else:
                    lower.sort(key=lambda x: (-x[2], x[1], x[0].info.num_id))
                    budget = [allowed for _ns, _sel, allowed in pdbs]
                    flagged = []
                    for ps, t, pr in lower:
                        bad = False
                        for q, (ns, sel, _a) in enumerate(pdbs):
                            if ns != ps.info.namespace or sel.empty or not sel.matches(ps.info.labels):
                                continue
                            budget[q] -= 1
                            bad = bad or budget[q] < 0
                        flagged.append((bad, ps, t, pr))
                    victims, violations = [], 0
                    for bad, ps, t, pr in [f for f in flagged if f[0]] + [f for f in flagged if not f[0]]:
                        eng.attach_pod(ps.info.num_id)
                        if hide:
                            cache.unhide([ps])
                        if not fits(node, idx):
                            eng.detach_pod(ps.info.num_id)
                            if hide:
                                cache.hide([ps.info.uid])
                            victims.append((ps, t, pr))
                            violations += bad
                    for ps, _t, _p in victims:
                        eng.attach_pod(ps.info.num_id)
                    if victims:
                        (viol if violations else nonviol).append((node, idx, victims, violations))
            finally:
                if hide:
                    cache.unhide([ps for ps, _t, _p in lower if ps.info.uid not in cache.pods])
        if nonviol and len(nonviol) + len(viol) >= want:
            break
    cands = nonviol + viol
    if not cands:
        return None

    def rank(c):
        _node, _idx, victims, violations = c
        top = max(pr for _ps, _t, pr in victims)
        earliest = min(t for _ps, t, pr in victims if pr == top)
        return (violations, top, sum(pr + (1 << 31) for _ps, _t, pr in victims), len(victims), -earliest)
    node, idx, victims, _v = min(cands, key=rank)     # min keeps the first of equal keys
    for ps, _t, _p in victims:
        eng.detach_pod(ps.info.num_id)
    ok_cards, cards, _q = eng.select_gpus(req, idx)
    for ps, _t, _p in victims:
        eng.attach_pod(ps.info.num_id)
    return node, [ps for ps, _t, _p in victims], (list(cards) if ok_cards else [])


def register_defaults(registry) -> None:
    for cls in (PrioritySort, NodeUnschedulable, NodeName, NodeResourcesFit, NodeAffinity, TaintToleration,
                NodeResourcesLeastAllocated, NodeResourcesMostAllocated, NodeResourcesBalancedAllocation,
                NodePorts, DefaultBinder, DefaultPreemption):
        registry.register(cls.name, cls)
    from .spread_affinity import InterPodAffinity, PodTopologySpread
    registry.register(PodTopologySpread.name, PodTopologySpread)
    registry.register(InterPodAffinity.name, InterPodAffinity)
    from .coscheduling import Coscheduling
    registry.register(Coscheduling.name, Coscheduling)
    from .node_extras import ImageLocality, NodePreferAvoidPods
    from .volumes import VOLUME_PLUGINS
    from .optional import OPTIONAL_PLUGINS
    for cls in (ImageLocality, NodePreferAvoidPods, *VOLUME_PLUGINS, *OPTIONAL_PLUGINS):
        registry.register(cls.name, cls)
    for n in INERT_PLUGINS:
        registry.register(n, _inert(n))
