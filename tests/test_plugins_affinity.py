"""PodTopologySpread and InterPodAffinity (upstream default plugins) through the scheduler,
plus the native fast path staying on for pods that do not use them."""
import asyncio

from yoda_scheduler_amd.models.selectors import LabelSelector
from yoda_scheduler_amd.testing import FakeCluster, yoda_config


def run(c):
    return asyncio.run(c)


def default_cfg():
    # the reference's profile shape: yoda on top of the upstream defaults (spread/affinity included)
    cfg = yoda_config()
    return cfg


def test_label_selector_semantics():
    s = LabelSelector({"matchLabels": {"app": "web"}, "matchExpressions": [
        {"key": "tier", "operator": "In", "values": ["fe", "be"]}, {"key": "x", "operator": "DoesNotExist"}]})
    assert s.matches({"app": "web", "tier": "fe"})
    assert not s.matches({"app": "web", "tier": "db"}) and not s.matches({"app": "web", "tier": "fe", "x": "1"})
    assert LabelSelector({}).matches({"a": "b"}) and not LabelSelector(None).matches({"a": "b"})


def test_topology_spread_balances_zones():
    async def go():
        c = FakeCluster(default_cfg())
        for name, zone in (("n0", "z1"), ("n1", "z1"), ("n2", "z2")):
            c.add_node(name, labels={"topology.kubernetes.io/zone": zone})
        await c.start()
        fw = c.sched.frameworks["yoda-scheduler"]
        spread = [{"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule",
                   "labelSelector": {"matchLabels": {"app": "web"}}}]
        for i in range(4):
            c.add_pod(f"w{i}", {"app": "web", "scv/memory": "1000"}, topologySpreadConstraints=spread)
            await c.wait_bound(i + 1)
        zones = [("z1" if c.node_of(f"w{i}") in ("n0", "n1") else "z2") for i in range(4)]
        plain = c.add_pod("plain", {"scv/memory": "1"})
        native_plain = fw.native_for(c.sched.queue._pods.get(plain["metadata"]["uid"]) or
                                     __import__("yoda_scheduler_amd.models.pod", fromlist=["PodInfo"]).PodInfo.from_obj(plain))
        await c.stop()
        return zones, native_plain
    zones, native_plain = run(go())
    assert zones.count("z1") == 2 and zones.count("z2") == 2
    assert native_plain


def test_required_anti_affinity_one_per_node():
    async def go():
        c = FakeCluster(default_cfg())
        for i in range(3):
            c.add_node(f"n{i}")
        await c.start()
        anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"topologyKey": "kubernetes.io/hostname", "labelSelector": {"matchLabels": {"app": "db"}}}]}}
        for i in range(4):
            c.add_pod(f"db{i}", {"app": "db", "scv/memory": "1000"}, affinity=anti)
        await c.wait_bound(3)
        await c.wait(lambda: c.sched.failed >= 1, 2)
        nodes = [c.node_of(f"db{i}") for i in range(4)]
        await c.stop()
        return nodes
    nodes = run(go())
    assert len({n for n in nodes if n}) == 3 and nodes.count("") == 1


def test_required_affinity_and_symmetry():
    async def go():
        c = FakeCluster(default_cfg())
        for i in range(3):
            c.add_node(f"n{i}")
        await c.start()
        c.add_pod("cache", {"app": "cache", "scv/memory": "1000"},
                  affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                      {"topologyKey": "kubernetes.io/hostname", "labelSelector": {"matchLabels": {"app": "noisy"}}}]}})
        await c.wait_bound(1)
        cache_node = c.node_of("cache")
        c.add_pod("client", {"app": "client", "scv/memory": "1000"},
                  affinity={"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                      {"topologyKey": "kubernetes.io/hostname", "labelSelector": {"matchLabels": {"app": "cache"}}}]}})
        for i in range(6):
            c.add_pod(f"noisy{i}", {"app": "noisy", "scv/memory": "1000"})
        await c.wait_bound(8)
        r = cache_node, c.node_of("client"), {c.node_of(f"noisy{i}") for i in range(6)}
        await c.stop()
        return r
    cache_node, client_node, noisy_nodes = run(go())
    assert client_node == cache_node
    assert cache_node not in noisy_nodes


def test_preferred_affinity_and_hard_pod_affinity_weight_scoring():
    """Preferred pod affinity pulls a pod into the zone of matching pods; an existing pod's
    required affinity term that matches the incoming pod scores its domain with
    hardPodAffinityWeight (upstream symmetric scoring)."""
    async def go():
        cfg = default_cfg()
        cfg["profiles"][0]["pluginConfig"].append({"name": "InterPodAffinity", "args": {"hardPodAffinityWeight": 5}})
        # weight the affinity score above yoda's so the test isolates it
        cfg["profiles"][0]["plugins"]["score"]["enabled"].append({"name": "InterPodAffinity", "weight": 1000})
        c = FakeCluster(cfg)
        for i, zone in enumerate(("z1", "z1", "z2", "z2")):
            c.add_node(f"n{i}", labels={"topology.kubernetes.io/zone": zone})
        await c.start()
        c.add_pod("web", {"app": "web", "scv/memory": "1000"}, nodeSelector={"kubernetes.io/hostname": "n3"})
        await c.wait_bound(1)
        pref = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 100, "podAffinityTerm": {"topologyKey": "topology.kubernetes.io/zone",
                                                "labelSelector": {"matchLabels": {"app": "web"}}}}]}}
        c.add_pod("near-web", {"app": "x", "scv/memory": "1000"}, affinity=pref)
        # an existing pod that *requires* affinity to app=db (satisfied by db0 in zone z1):
        # a new db pod is pulled to z1 by hardPodAffinityWeight
        c.add_pod("db0", {"app": "db", "scv/memory": "1000"}, nodeSelector={"kubernetes.io/hostname": "n1"})
        await c.wait_bound(3)
        req = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"topologyKey": "topology.kubernetes.io/zone", "labelSelector": {"matchLabels": {"app": "db"}}}]}}
        c.add_pod("db-client", {"app": "dbc", "scv/memory": "1000"}, affinity=req)
        await c.wait_bound(4)
        # the plugin's own view for a db pod: z1 nodes carry hardPodAffinityWeight (5)
        from yoda_scheduler_amd.framework.interfaces import CycleState
        from yoda_scheduler_amd.models.pod import PodInfo
        ipa = c.sched.frameworks["yoda-scheduler"].plugins["InterPodAffinity"]
        probe = PodInfo.from_obj({"metadata": {"name": "probe", "namespace": "default", "uid": "probe",
                                               "labels": {"app": "db"}}, "spec": {}})
        st = CycleState()
        ipa.pre_score(st, probe, [])
        raw = {n: ipa.score(st, probe, n)[0] for n in ("n0", "n1", "n2", "n3")}
        c.add_pod("db", {"app": "db", "scv/memory": "1000"})
        await c.wait_bound(5)
        out = c.node_of("near-web"), c.node_of("db-client"), c.node_of("db"), raw
        await c.stop()
        return out
    near, dbc, db, raw = run(go())
    assert raw == {"n0": 5, "n1": 5, "n2": 0, "n3": 0}
    assert near in ("n2", "n3")
    assert dbc in ("n0", "n1") and db in ("n0", "n1")


def test_anti_affinity_symmetry_scales():
    """300 bound pods with hostname anti-affinity on a 400-node cluster: the per-cycle
    precomputation keeps scheduling 100 more pods fast (no node × pod rescans)."""
    import time

    async def go():
        c = FakeCluster(default_cfg())
        for i in range(400):
            c.add_node(f"n{i:03d}")
        await c.start()
        anti = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"topologyKey": "kubernetes.io/hostname", "labelSelector": {"matchLabels": {"app": "solo"}}}]}}
        for i in range(300):
            c.add_pod(f"solo{i}", {"app": "solo", "scv/memory": "1000"}, affinity=anti)
        ok1 = await c.wait_bound(300, 60)
        t = time.perf_counter()
        for i in range(100):
            c.add_pod(f"plain{i}", {"app": "plain", "scv/memory": "1000"})
        ok2 = await c.wait_bound(400, 60)
        dt = time.perf_counter() - t
        solo_nodes = {c.node_of(f"solo{i}") for i in range(300)}
        await c.stop()
        return ok1, ok2, dt, len(solo_nodes)
    ok1, ok2, dt, distinct = run(go())
    assert ok1 and ok2 and distinct == 300
    assert dt < 20, dt
