"""PodTopologySpread with upstream v1.20 semantics: node-affinity-scoped
domains in Filter, ``log(size + 2)``-weighted scoring with ignored nodes, and the
``DefaultPodTopologySpread`` system default constraints for Service / controller pods.

Score vectors are hand-computed from the upstream v1.20 formulas (the reference tree ships
no upstream source, so parity is pinned by these vectors)."""
from types import SimpleNamespace

import pytest

from yoda_scheduler_amd.framework.interfaces import Code, CycleState, NodeScore
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.plugins.spread_affinity import PodTopologySpread

HOST, ZONE = "kubernetes.io/hostname", "topology.kubernetes.io/zone"


def pod(name, labels=None, node="", deleting=False, **spec):
    meta = {"name": name, "namespace": "default", "uid": f"uid-{name}", "labels": dict(labels or {})}
    if deleting:
        meta["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    s = dict(spec)
    if node:
        s["nodeName"] = node
    return PodInfo.from_obj({"metadata": meta, "spec": s})


class FakeHandle:
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


def web_service():
    return {"services": {"default/web": {"metadata": {"name": "web", "namespace": "default"},
                                         "spec": {"selector": {"app": "web"}}}}}


def scores_of(plugin, p, nodes):
    st = CycleState()
    plugin.pre_score(st, p, nodes)
    out = [NodeScore(n, plugin.score(st, p, n)[0]) for n in nodes]
    plugin.normalize_score(st, p, out)
    return {x.name: x.score for x in out}


def three_nodes(extra=None):
    nodes = {"n0": {HOST: "n0", ZONE: "z1"}, "n1": {HOST: "n1", ZONE: "z1"}, "n2": {HOST: "n2", ZONE: "z2"}}
    nodes.update(extra or {})
    return nodes


def test_system_default_constraints_score_service_pods():
    placed = [(pod("a", {"app": "web"}), "n0"), (pod("b", {"app": "web"}), "n0"),
              (pod("c", {"app": "db"}), "n2")]
    h = FakeHandle(three_nodes(), placed, web_service())
    pl = PodTopologySpread({}, h)
    assert pl.defaulting_type == "System"
    newp = pod("new", {"app": "web"})
    assert not pl.is_noop_for(newp)
    # hostname: size 3 → ln 5; zone: 2 domains → ln 4; + (maxSkew − 1) = 2 / 4
    # n0: 2·ln5+2 + 2·ln4+4 = 11.99 → 11; n1: 2 + 6.77 → 8; n2: 2 + 4 = 6
    # normalise 100·(max + min − s)/max with max 11, min 6
    assert scores_of(pl, newp, ["n0", "n1", "n2"]) == {"n0": 54, "n1": 81, "n2": 100}


def test_nodes_missing_a_key_are_ignored_and_score_zero():
    nodes = three_nodes({"n3": {HOST: "n3"}})          # no zone label
    placed = [(pod("a", {"app": "web"}), "n0"), (pod("b", {"app": "web"}), "n0")]
    pl = PodTopologySpread({}, FakeHandle(nodes, placed, web_service()))
    assert scores_of(pl, pod("new", {"app": "web"}), ["n0", "n1", "n2", "n3"]) == \
        {"n0": 54, "n1": 81, "n2": 100, "n3": 0}


def test_pods_without_service_or_controller_are_noop():
    pl = PodTopologySpread({}, FakeHandle(three_nodes(), (), web_service()))
    assert pl.is_noop_for(pod("x", {"app": "other"}))
    pl_list = PodTopologySpread({"defaultingType": "List"}, FakeHandle(three_nodes(), (), web_service()))
    assert pl_list.default_constraints == [] and pl_list.is_noop_for(pod("y", {"app": "web"}))


def test_explicit_soft_constraint_score_and_terminating_pods_skipped():
    spread = [{"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "ScheduleAnyway",
               "labelSelector": {"matchLabels": {"app": "w"}}}]
    placed = [(pod("a", {"app": "w"}), "n0"), (pod("gone", {"app": "w"}, deleting=True), "n2"),
              (pod("other", {"app": "x"}), "n2")]
    pl = PodTopologySpread({}, FakeHandle(three_nodes(), placed))
    # z1 has 1 matching pod (z2's is terminating): n0 = n1 = ln 4 → 1, n2 = 0 → 100·(1+0−s)/1
    assert scores_of(pl, pod("p", {"app": "w"}, topologySpreadConstraints=spread), ["n0", "n1", "n2"]) == \
        {"n0": 0, "n1": 0, "n2": 100}


def test_filter_domains_follow_node_affinity():
    nodes = {"n0": {ZONE: "z1", "pool": "a"}, "n1": {ZONE: "z2", "pool": "a"}, "n2": {ZONE: "z3", "pool": "b"}}
    placed = [(pod("a", {"app": "w"}), "n0"), (pod("b", {"app": "w"}), "n1")]
    spread = [{"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule",
               "labelSelector": {"matchLabels": {"app": "w"}}}]
    pl = PodTopologySpread({}, FakeHandle(nodes, placed))

    def verdict(p, node):
        st = CycleState()
        pl.pre_filter(st, p)
        return pl.filter(st, p, node).code

    # without a node selector z3 (empty) is a domain: min 0 → n0 skew 1+1−0 = 2 > 1
    free = pod("p", {"app": "w"}, topologySpreadConstraints=spread)
    assert verdict(free, "n0") == Code.UNSCHEDULABLE and verdict(free, "n2") == Code.SUCCESS
    # nodeSelector pool=a: z3 is not a domain, min 1 → n0 skew 1 ≤ 1
    pinned = pod("q", {"app": "w"}, nodeSelector={"pool": "a"}, topologySpreadConstraints=spread)
    assert verdict(pinned, "n0") == Code.SUCCESS
    # required node affinity scopes domains the same way
    aff = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
        {"matchExpressions": [{"key": "pool", "operator": "In", "values": ["a"]}]}]}}}
    assert verdict(pod("r", {"app": "w"}, affinity=aff, topologySpreadConstraints=spread), "n0") == Code.SUCCESS


def test_filter_missing_label_is_unresolvable():
    spread = [{"maxSkew": 1, "topologyKey": "rack", "whenUnsatisfiable": "DoNotSchedule",
               "labelSelector": {"matchLabels": {"app": "w"}}}]
    nodes = {"n0": {"rack": "r1"}, "n1": {}}
    pl = PodTopologySpread({}, FakeHandle(nodes))
    p = pod("p", {"app": "w"}, topologySpreadConstraints=spread)
    st = CycleState()
    pl.pre_filter(st, p)
    assert pl.filter(st, p, "n1").code == Code.UNSCHEDULABLE_AND_UNRESOLVABLE
    assert pl.filter(st, p, "n0").is_success()


def test_list_default_constraints_filter_service_pods():
    args = {"defaultingType": "List",
            "defaultConstraints": [{"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule"}]}
    placed = [(pod("a", {"app": "web"}), "n0")]
    pl = PodTopologySpread(args, FakeHandle(three_nodes(), placed, web_service()))
    p = pod("new", {"app": "web"})
    st = CycleState()
    pl.pre_filter(st, p)
    # z1 has 1, z2 has 0: z1 nodes would reach skew 2
    assert [pl.filter(st, p, n).code for n in ("n0", "n1", "n2")] == \
        [Code.UNSCHEDULABLE, Code.UNSCHEDULABLE, Code.SUCCESS]


def test_args_validation():
    with pytest.raises(ValueError):
        PodTopologySpread({"defaultingType": "System", "defaultConstraints": [
            {"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule"}]}, FakeHandle({}))
    with pytest.raises(ValueError):
        PodTopologySpread({"defaultConstraints": [{"maxSkew": 0, "topologyKey": ZONE,
                                                   "whenUnsatisfiable": "DoNotSchedule"}]}, FakeHandle({}))
    with pytest.raises(ValueError):
        PodTopologySpread({"defaultingType": "Cluster"}, FakeHandle({}))
    assert PodTopologySpread({"defaultConstraints": [{"maxSkew": 2, "topologyKey": ZONE,
                                                      "whenUnsatisfiable": "ScheduleAnyway"}]},
                             FakeHandle({})).defaulting_type == "List"
