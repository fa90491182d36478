"""The registered-but-not-default upstream v1.20 plugins: NodeLabel,
ServiceAffinity, SelectorSpread, RequestedToCapacityRatio and CinderLimits.

Score vectors are hand-computed from the upstream v1.20 formulas (the reference tree
ships no upstream source, so parity is pinned by these vectors, not by a run of
kube-scheduler). End-to-end cases go through the scheduler on the fake apiserver.
"""
import asyncio
from types import SimpleNamespace

import pytest

from yoda_scheduler_amd.framework.interfaces import CycleState, NodeScore
from yoda_scheduler_amd.models.pod import PF_CONTROLLER, PodInfo
from yoda_scheduler_amd.plugins.optional import (NodeLabel, RequestedToCapacityRatio, SelectorSpread,
                                                 ServiceAffinity, broken_linear, zone_key)
from yoda_scheduler_amd.testing import FakeCluster, yoda_config


def pod(name, labels=None, ns="default", owner=None, node="", **spec):
    meta = {"name": name, "namespace": ns, "uid": f"uid-{ns}-{name}", "labels": dict(labels or {})}
    if owner:
        meta["ownerReferences"] = [owner]
    s = dict(spec)
    if node:
        s["nodeName"] = node
    return PodInfo.from_obj({"metadata": meta, "spec": s})


class FakeHandle:
    """nodes: name → labels; placed: [(PodInfo, node)]; objs: resource → {key: obj}."""

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


def svc(name, selector, ns="default"):
    return {f"{ns}/{name}": {"metadata": {"name": name, "namespace": ns}, "spec": {"selector": selector}}}


def scores_of(plugin, p, nodes):
    st = CycleState()
    if hasattr(plugin, "pre_score"):
        plugin.pre_score(st, p, nodes)
    out = [NodeScore(n, plugin.score(st, p, n)[0]) for n in nodes]
    plugin.normalize_score(st, p, out)
    return {x.name: x.score for x in out}


# ------------------------------------------------------------------ NodeLabel
def test_node_label_filter_and_score():
    h = FakeHandle({"a": {"gpu": "1", "ssd": "1"}, "b": {"gpu": "1", "spot": "1"}, "c": {}})
    pl = NodeLabel({"presentLabels": ["gpu"], "absentLabels": ["spot"],
                    "presentLabelsPreference": ["ssd"], "absentLabelsPreference": ["spot"]}, h)
    p = pod("p")
    st = CycleState()
    assert pl.filter(st, p, "a").is_success()
    assert not pl.filter(st, p, "b").is_success()           # has an absent label
    assert pl.filter(st, p, "c").message() == "node(s) didn't have the requested labels"
    # a: ssd present (100) + spot absent (100) → 200/2; b: 0 + 0; c: 0 + 100 → 50
    assert [pl.score(st, p, n)[0] for n in "abc"] == [100, 0, 50]
    with pytest.raises(ValueError):
        NodeLabel({"presentLabels": ["x"], "absentLabels": ["x"]}, h)
    assert NodeLabel({}, h).is_noop_for(p) and not pl.is_noop_for(p)


# ------------------------------------------------------------------ SelectorSpread
def test_zone_key():
    assert zone_key({}) == ""
    assert zone_key({"topology.kubernetes.io/zone": "z1"}) == ":\x00:z1"
    assert zone_key({"failure-domain.beta.kubernetes.io/region": "r", "topology.kubernetes.io/zone": "z"}) == \
        "r:\x00:z"


def test_selector_spread_nodes_only():
    nodes = {"a": {}, "b": {}, "c": {}}
    web = {"app": "web"}
    placed = [(pod("w1", web), "a"), (pod("w2", web), "a"), (pod("w3", web), "b"), (pod("x", {"app": "db"}), "c")]
    h = FakeHandle(nodes, placed, {"services": svc("web", web)})
    pl = SelectorSpread({}, h)
    p = pod("new", web)
    assert not pl.is_noop_for(p)
    # counts a=2 b=1 c=0, max 2 → 100·(2−n)/2
    assert scores_of(pl, p, list(nodes)) == {"a": 0, "b": 50, "c": 100}


def test_selector_spread_with_zones_and_replicaset_owner():
    z = "topology.kubernetes.io/zone"
    nodes = {"a": {z: "z1"}, "b": {z: "z1"}, "c": {z: "z2"}, "d": {}}
    lab = {"app": "web", "pod-template-hash": "h"}
    owner = {"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs1", "controller": True, "uid": "rs"}
    placed = [(pod("w1", lab), "a"), (pod("w2", lab), "a"), (pod("w3", lab), "c"),
              (pod("other-ns", lab, ns="kube-system"), "b")]
    rs = {"default/rs1": {"metadata": {"name": "rs1", "namespace": "default"},
                          "spec": {"selector": {"matchLabels": {"app": "web"}}}}}
    h = FakeHandle(nodes, placed, {"replicasets": rs})
    pl = SelectorSpread({}, h)
    p = pod("new", lab, owner=owner)
    assert p.flags & PF_CONTROLLER and not pl.is_noop_for(p)
    got = scores_of(pl, p, list(nodes))
    # node counts a=2 b=0 c=1 d=0 (max 2); zone counts z1=2 z2=1 (max 2)
    # a: node 0, zone 0 → 0;  b: node 100, zone 0 → 100/3 = 33
    # c: node 50, zone 50 → 50;  d: no zone → node score 100
    assert got == {"a": 0, "b": 33, "c": 50, "d": 100}


def test_selector_spread_skips_topology_spread_pods_and_unowned():
    h = FakeHandle({"a": {}}, (), {})
    pl = SelectorSpread({}, h)
    assert pl.is_noop_for(pod("plain", {"app": "x"}))
    assert pl.is_noop_for(pod("tsc", {"app": "x"}, topologySpreadConstraints=[{"maxSkew": 1}]))


# ------------------------------------------------------------------ ServiceAffinity
def test_service_affinity_filter_pins_to_first_service_pod_zone():
    nodes = {"a": {"zone": "z1"}, "b": {"zone": "z1"}, "c": {"zone": "z2"}}
    web = {"app": "web"}
    h = FakeHandle(nodes, [(pod("w1", web), "b")], {"services": svc("web", web)})
    pl = ServiceAffinity({"affinityLabels": ["zone"]}, h)
    p = pod("new", web)
    st = CycleState()
    pl.pre_filter(st, p)
    assert [pl.filter(st, p, n).is_success() for n in "abc"] == [True, True, False]
    assert pl.filter(st, p, "c").message() == "node(s) didn't match service affinity"
    # the pod's own nodeSelector wins over the introspected value
    p2 = pod("new2", web, nodeSelector={"zone": "z2"})
    st2 = CycleState()
    pl.pre_filter(st2, p2)
    assert [pl.filter(st2, p2, n).is_success() for n in "abc"] == [False, False, True]
    # no service → no constraint
    p3 = pod("lonely", {"app": "solo"})
    st3 = CycleState()
    pl.pre_filter(st3, p3)
    assert all(pl.filter(st3, p3, n).is_success() for n in "abc")


def test_service_affinity_anti_affinity_score():
    nodes = {"a": {"zone": "z1"}, "b": {"zone": "z1"}, "c": {"zone": "z2"}, "d": {}}
    web = {"app": "web"}
    placed = [(pod("w1", web), "a"), (pod("w2", web), "a"), (pod("w3", web), "b"), (pod("w4", web), "c")]
    h = FakeHandle(nodes, placed, {"services": svc("web", web)})
    pl = ServiceAffinity({"antiAffinityLabelsPreference": ["zone"]}, h)
    got = scores_of(pl, pod("new", web), list(nodes))
    # service pods per node a=2 b=1 c=1 d=0, total 4; per zone z1=3 z2=1
    # z1 nodes: 100·(4−3)/4 = 25; z2: 100·(4−1)/4 = 75; d has no zone label → 0
    assert got == {"a": 25, "b": 25, "c": 75, "d": 0}


# ------------------------------------------------------------------ RequestedToCapacityRatio
def test_broken_linear_function():
    f = broken_linear([(0, 0), (50, 80), (100, 100)])
    assert [f(0), f(25), f(50), f(75), f(100), f(120)] == [0, 40, 80, 90, 100, 100]
    g = broken_linear([(10, 20)])
    assert g(0) == 20 and g(10) == 20 and g(50) == 20


def test_requested_to_capacity_ratio_score():
    engine = SimpleNamespace(node_index=lambda n: 0, node_usage=lambda i: (0, 0, 3, 0, 2000, 4 << 30))
    node = SimpleNamespace(labels={}, cpu_m=8000, mem=16 << 30, ext_alloc={"amd.com/gpu": 8})
    cache = SimpleNamespace(nodes={"n": node}, engine=engine, node_ext_used={"n": {"amd.com/gpu": 2}})
    h = SimpleNamespace(cache=cache)
    # bin-packing shape: 0% → 0, 100% → 10 (×10 = 100)
    pl = RequestedToCapacityRatio({"shape": [{"utilization": 0, "score": 0}, {"utilization": 100, "score": 10}],
                                   "resources": [{"name": "cpu", "weight": 2}, {"name": "memory", "weight": 1},
                                                 {"name": "amd.com/gpu", "weight": 3}]}, h)
    p = pod("p")
    p.nz_cpu_m, p.nz_mem, p.ext = 2000, 200 * 1024 * 1024, {"amd.com/gpu": 2}
    # cpu (2000+2000)/8000 = 50 → 50; memory (4Gi+200Mi)/16Gi → util 100 − (16Gi−4.2Gi)·100//16Gi = 27 → 27;
    # gpu 4/8 = 50 → 50;  (50·2 + 27·1 + 50·3)/6 = 277/6 = 46.17 → 46
    assert pl.score(CycleState(), p, "n")[0] == 46
    with pytest.raises(ValueError):
        RequestedToCapacityRatio({"shape": [{"utilization": 50, "score": 1}, {"utilization": 40, "score": 2}]}, h)
    with pytest.raises(ValueError):
        RequestedToCapacityRatio({"shape": [{"utilization": 50, "score": 11}]}, h)
    with pytest.raises(ValueError):
        RequestedToCapacityRatio({"shape": [{"utilization": 50, "score": 1}],
                                  "resources": [{"name": "cpu", "weight": 0}]}, h)


# ------------------------------------------------------------------ end to end
def _cfg(filter_plugins=(), score_plugins=(), args=None, yoda_weight=1):
    cfg = yoda_config()
    prof = cfg["profiles"][0]
    prof["plugins"]["filter"]["enabled"] += [{"name": n} for n in filter_plugins]
    prof["plugins"]["score"]["enabled"] = [{"name": "yoda", "weight": yoda_weight}] + \
        [{"name": n, "weight": w} for n, w in score_plugins]
    prof["pluginConfig"] += [{"name": n, "args": a} for n, a in (args or {}).items()]
    return cfg


def run(c):
    return asyncio.run(c)


def test_e2e_selector_spread_spreads_service_pods():
    async def go():
        c = FakeCluster(_cfg(score_plugins=[("SelectorSpread", 1000)]))
        for i in range(4):
            c.add_node(f"n{i}")
        c.server.create("services", {"metadata": {"name": "web", "namespace": "default"},
                                     "spec": {"selector": {"app": "web"}}})
        await c.start()
        for i in range(8):
            c.add_pod(f"w{i}", {"app": "web", "scv/memory": "1000"})
            assert await c.wait_bound(i + 1)
        nodes = [c.node_of(f"w{i}") for i in range(8)]
        await c.stop()
        return nodes
    nodes = run(go())
    assert sorted(nodes.count(f"n{i}") for i in range(4)) == [2, 2, 2, 2]


def test_e2e_node_label_filter_and_cinder_limits():
    async def go():
        c = FakeCluster(_cfg(filter_plugins=["NodeLabel", "CinderLimits"],
                             args={"NodeLabel": {"presentLabels": ["amd.com/mi355x"]}}))
        c.add_node("plain")
        c.add_node("gpu", labels={"amd.com/mi355x": "true"})
        await c.start()
        c.add_pod("p", {"scv/memory": "1000"})
        assert await c.wait_bound(1)
        # Cinder: default limit 256 volumes; a pod with one cinder volume schedules
        c.add_pod("vol", {"scv/memory": "1000"}, volumes=[{"name": "v", "cinder": {"volumeID": "vol-1"}}])
        assert await c.wait_bound(2)
        out = c.node_of("p"), c.node_of("vol")
        await c.stop()
        return out
    assert run(go()) == ("gpu", "gpu")


def test_e2e_requested_to_capacity_ratio_binpacks():
    async def go():
        shape = [{"utilization": 0, "score": 0}, {"utilization": 100, "score": 10}]
        c = FakeCluster(_cfg(score_plugins=[("RequestedToCapacityRatio", 1000)],
                             args={"RequestedToCapacityRatio": {"shape": shape}}))
        for i in range(3):
            c.add_node(f"n{i}")
        await c.start()
        res = {"requests": {"cpu": "8", "memory": "16Gi"}}
        for i in range(4):
            c.add_pod(f"p{i}", {"scv/memory": "1000"}, containers=[{"name": "c", "image": "x", "resources": res}])
            assert await c.wait_bound(i + 1)
        nodes = [c.node_of(f"p{i}") for i in range(4)]
        await c.stop()
        return nodes
    nodes = run(go())
    assert len(set(nodes)) == 1          # most-requested shape packs every pod on one node
