"""Volume plugins' no-op tests for pods whose claims are all bound (plugins/volumes.py).

A pod that mounts a bound PVC is a no-op for VolumeBinding (no PV node affinity),
VolumeZone (no zone labels on the PV), NodeVolumeLimits (no CSI attach limit anywhere) and
the in-tree attach limits (no disk of their kind), so it takes the native cycle. These tests
pin that a "no-op" answer is only given where the plugin's own PreFilter / Filter pass on
every node, that each volume feature moves the pod back to its plugin, and that the answer
follows PVC / PV / CSINode / node changes. Upstream reference: kube-scheduler v1.20's volume
plugins, kept by the reference's profile (/root/reference/deploy/yoda-scheduler.yaml:21-31)."""
import asyncio
import itertools

from yoda_scheduler_amd.framework.interfaces import CycleState
from yoda_scheduler_amd.models.pod import PodInfo
from yoda_scheduler_amd.testing import FakeCluster, yoda_config

VOLUME_PLUGINS = ("VolumeBinding", "VolumeZone", "NodeVolumeLimits", "EBSLimits", "GCEPDLimits", "AzureDiskLimits")


def run(c):
    return asyncio.run(c)


def _pv(name, *, host=None, zone=None, csi=True, ebs=False):
    spec = {"capacity": {"storage": "1Ti"}, "accessModes": ["ReadWriteMany"], "storageClassName": "shared"}
    if csi:
        spec["csi"] = {"driver": "nfs.csi.k8s.io", "volumeHandle": name}
    if ebs:
        spec["awsElasticBlockStore"] = {"volumeID": f"vol-{name}"}
    if host:
        spec["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchExpressions": [
            {"key": "kubernetes.io/hostname", "operator": "In", "values": [host]}]}]}}
    labels = {"topology.kubernetes.io/zone": zone} if zone else {}
    return {"metadata": {"name": name, "labels": labels}, "spec": spec, "status": {"phase": "Bound"}}


def _pvc(name, volume="", sc="shared", deleting=False):
    meta = {"name": name, "namespace": "default"}
    if deleting:
        meta["deletionTimestamp"] = "2026-01-01T00:00:00Z"
    spec = {"accessModes": ["ReadWriteMany"], "resources": {"requests": {"storage": "1Gi"}}, "storageClassName": sc}
    if volume:
        spec["volumeName"] = volume
    return {"metadata": meta, "spec": spec, "status": {"phase": "Bound" if volume else "Pending"}}


def _pod(name, claims=(), inline=()):
    vols = [{"name": f"v{i}", "persistentVolumeClaim": {"claimName": c}} for i, c in enumerate(claims)]
    vols += list(inline)
    return PodInfo.from_obj({"metadata": {"name": name, "namespace": "default", "uid": f"uid-{name}"},
                             "spec": {"schedulerName": "yoda-scheduler", "containers": [{"name": "c", "image": "x"}],
                                      "volumes": vols}})


# claim name → what it is bound to
CLAIMS = {
    "plain": ("pv-plain", {}),                   # CSI, no node affinity, no zone labels
    "pinned": ("pv-pinned", {"host": "n1"}),     # PV node affinity → VolumeBinding
    "zonal": ("pv-zonal", {"zone": "z2"}),       # PV zone label → VolumeZone
    "ebs": ("pv-ebs", {"csi": False, "ebs": True}),   # in-tree EBS source → EBSLimits
}


def _cluster(limits: str = ""):
    c = FakeCluster(yoda_config())
    c.add_node("n0", labels={"topology.kubernetes.io/zone": "z1"})
    c.add_node("n1", labels={"topology.kubernetes.io/zone": "z2"})
    c.server.create("storageclasses", {"metadata": {"name": "shared"}, "provisioner": "nfs.csi.k8s.io",
                                       "volumeBindingMode": "WaitForFirstConsumer"})
    for claim, (pv, kw) in CLAIMS.items():
        c.server.create("persistentvolumes", _pv(pv, **kw))
        c.server.create("persistentvolumeclaims", _pvc(claim, pv))
    c.server.create("persistentvolumeclaims", _pvc("unbound"))                 # WaitForFirstConsumer, unbound
    c.server.create("persistentvolumeclaims", _pvc("lost", "pv-gone"))        # names a PV that does not exist
    c.server.create("persistentvolumes", _pv("pv-del"))
    c.server.create("persistentvolumeclaims", _pvc("deleting", "pv-del", deleting=True))
    if limits == "csinode":
        c.server.create("csinodes", {"metadata": {"name": "n0"}, "spec": {"drivers": [
            {"name": "nfs.csi.k8s.io", "nodeID": "n0", "allocatable": {"count": 8}}]}})
    elif limits == "other":        # a limit for another CSI driver only
        c.server.create("csinodes", {"metadata": {"name": "n0"}, "spec": {"drivers": [
            {"name": "ebs.csi.aws.com", "nodeID": "n0", "allocatable": {"count": 25}}]}})
    elif limits == "node":
        node = c.server.get("nodes", "n1")
        alloc = dict(node["status"]["allocatable"], **{"attachable-volumes-csi-nfs.csi.k8s.io": "8"})
        c.server.patch("nodes", "n1", {"status": {"allocatable": alloc}})
    return c


def _noops(fw, pi) -> set:
    return {n for n in VOLUME_PLUGINS if fw.plugins[n].is_noop_for(pi)}


def test_bound_claim_pods_take_the_native_cycle_and_bind():
    async def go():
        c = _cluster()
        await c.start()
        fw = c.sched.frameworks["yoda-scheduler"]
        native = fw.native_for(_pod("probe", ["plain"]))
        for i in range(4):
            c.add_pod(f"p{i}", {"scv/memory": "1000"}, volumes=[{"name": "d", "persistentVolumeClaim": {
                "claimName": "plain"}}])
        ok = await c.wait_bound(4)
        nodes = {c.node_of(f"p{i}") for i in range(4)}
        await c.stop()
        return native, ok, nodes
    native, ok, nodes = run(go())
    assert native and ok and nodes <= {"n0", "n1"}


def test_each_volume_feature_moves_the_pod_back_to_its_plugin():
    async def go():
        out = {}
        for limits in ("", "csinode", "node", "other"):
            c = _cluster(limits)
            await c.start()
            fw = c.sched.frameworks["yoda-scheduler"]
            for claim in ("plain", "pinned", "zonal", "ebs", "unbound", "lost", "deleting", "absent"):
                pi = _pod(f"p-{claim}", [claim])
                out[(limits, claim)] = (set(VOLUME_PLUGINS) - _noops(fw, pi), fw.native_for(pi))
            pi = _pod("inline-ebs", inline=[{"name": "d", "awsElasticBlockStore": {"volumeID": "v-1"}}])
            out[(limits, "inline")] = (set(VOLUME_PLUGINS) - _noops(fw, pi), fw.native_for(pi))
            await c.stop()
        return out
    out = run(go())
    assert out[("", "plain")] == (set(), True)
    assert out[("", "pinned")] == ({"VolumeBinding"}, False)
    assert out[("", "zonal")] == ({"VolumeZone"}, False)
    assert out[("", "ebs")] == ({"EBSLimits"}, False)
    assert out[("", "inline")][0] == {"EBSLimits"} and not out[("", "inline")][1]
    for claim in ("unbound", "lost", "deleting", "absent"):
        applies, native = out[("", claim)]
        assert {"VolumeBinding", "VolumeZone"} <= applies and not native, claim
    # an attach limit anywhere (a CSINode count, or a node's attachable-volumes-csi-*) makes
    # NodeVolumeLimits count the CSI claim
    for limits in ("csinode", "node"):
        assert out[(limits, "plain")] == ({"NodeVolumeLimits"}, False), limits
        assert "NodeVolumeLimits" not in out[(limits, "ebs")][0]       # not a CSI volume
    # a limit for another driver leaves the NFS claim's pod native (limits are per driver)
    assert out[("other", "plain")] == (set(), True)


def test_noop_answer_is_exact_against_the_plugins_own_prefilter_and_filter():
    """Every pod over every pair of claims (and an inline disk), in clusters without and with
    attach limits: whenever a plugin calls itself a no-op, its PreFilter and its Filter on
    every node pass; and the answer is not vacuous (both kinds of pods occur)."""
    claims = ["plain", "pinned", "zonal", "ebs", "unbound", "lost", "deleting", "absent"]
    combos = [list(x) for k in (1, 2) for x in itertools.combinations(claims, k)]

    async def go():
        seen_noop = seen_applies = 0
        bad = []
        for limits in ("", "csinode", "node", "other"):
            c = _cluster(limits)
            await c.start()
            fw = c.sched.frameworks["yoda-scheduler"]
            for k, combo in enumerate(combos):
                for inline in ((), ({"name": "d", "awsElasticBlockStore": {"volumeID": f"v-{k}"}},)):
                    pi = _pod(f"x{k}-{len(inline)}", combo, inline)
                    for name in VOLUME_PLUGINS:
                        p = fw.plugins[name]
                        if not p.is_noop_for(pi):
                            seen_applies += 1
                            continue
                        seen_noop += 1
                        state = CycleState()
                        if hasattr(p, "pre_filter") and not p.pre_filter(state, pi).is_success():
                            bad.append((limits, combo, inline, name, "pre_filter"))
                            continue
                        for node in ("n0", "n1"):
                            if not p.filter(state, pi, node).is_success():
                                bad.append((limits, combo, inline, name, node))
            await c.stop()
        return seen_noop, seen_applies, bad
    seen_noop, seen_applies, bad = run(go())
    assert not bad, bad[:5]
    assert seen_noop > 100 and seen_applies > 100


def test_noop_answer_follows_pv_csinode_and_node_changes():
    async def go():
        c = _cluster()
        await c.start()
        fw = c.sched.frameworks["yoda-scheduler"]
        pi = _pod("same", ["plain"])            # one PodInfo asked again after each change
        steps = [fw.native_for(pi)]
        c.server.patch("persistentvolumes", "pv-plain", {"metadata": {"labels": {
            "topology.kubernetes.io/zone": "z1"}}})
        await c.wait(lambda: not fw.plugins["VolumeZone"].is_noop_for(pi), 3.0)
        steps.append((fw.plugins["VolumeZone"].is_noop_for(pi), fw.native_for(pi)))
        c.server.patch("persistentvolumes", "pv-plain", {"metadata": {"labels": None}})
        await c.wait(lambda: fw.native_for(pi), 3.0)
        steps.append(fw.native_for(pi))
        c.server.create("csinodes", {"metadata": {"name": "n1"}, "spec": {"drivers": [
            {"name": "nfs.csi.k8s.io", "nodeID": "n1", "allocatable": {"count": 4}}]}})
        await c.wait(lambda: not fw.native_for(pi), 3.0)
        steps.append((fw.plugins["NodeVolumeLimits"].is_noop_for(pi), fw.native_for(pi)))
        c.server.delete("csinodes", "n1")
        await c.wait(lambda: fw.native_for(pi), 3.0)
        steps.append(fw.native_for(pi))
        node = c.server.get("nodes", "n0")
        alloc = dict(node["status"]["allocatable"], **{"attachable-volumes-csi-nfs.csi.k8s.io": "2"})
        c.server.patch("nodes", "n0", {"status": {"allocatable": alloc}})
        await c.wait(lambda: not fw.native_for(pi), 3.0)
        steps.append(fw.native_for(pi))
        c.server.delete("nodes", "n0")
        await c.wait(lambda: fw.native_for(pi), 3.0)
        steps.append(fw.native_for(pi))
        await c.stop()
        return steps
    assert run(go()) == [True, (False, False), True, (False, False), True, False, True]


def test_bench_pvc_workload_mounts_bound_claims():
    """``bench.py --mix-volumes N``: N pods of the burst mount one of the workload's bound
    claims, and the claims and PVs are created with the cluster."""
    from yoda_scheduler_amd.bench.workloads import make_workload
    w = make_workload(3, mix_volumes=100)
    mounts = [v["persistentVolumeClaim"]["claimName"] for s in w.specs.values() for v in s.get("volumes", ())]
    made = {(res, o["metadata"]["name"]) for res, o in w.objects}
    assert len(mounts) == 100 and "PVC pods" in w.name
    assert all(("persistentvolumeclaims", m) in made for m in mounts)
    pvs = {o["metadata"]["name"]: o for res, o in w.objects if res == "persistentvolumes"}
    assert all(o["spec"]["volumeName"] in pvs for res, o in w.objects if res == "persistentvolumeclaims")


def test_incremental_claim_table_equals_a_full_recompute():
    """``LaneClaims`` (per-event updates of the lane's claim table) ≡ ``lane_claims`` recomputed
    over every PVC, after each of a random sequence of PVC / PV / CSINode / node-limit changes."""
    import collections
    import random
    from types import SimpleNamespace

    from yoda_scheduler_amd.plugins.volumes import LaneClaims, claim_volumes, lane_claims

    class H:
        def __init__(self):
            self.objs = {"persistentvolumeclaims": {}, "persistentvolumes": {}, "csinodes": {}, "storageclasses": {
                "shared": {"metadata": {"name": "shared"}, "provisioner": "nfs.csi.k8s.io"}}}
            self.gen = collections.Counter()
            self.cache = SimpleNamespace(csi_limit_drivers={})

        def lister(self, res):
            return self.objs[res]

        def generation(self, res):
            return self.gen[res]

    adds = removes = 0
    for seed in range(40):
        rng = random.Random(seed)
        h = H()
        t = LaneClaims(h)
        for _step in range(60):
            op = rng.random()
            if op < 0.4:
                name = f"c{rng.randrange(6)}"
                key = f"default/{name}"
                if rng.random() < 0.2 and key in h.objs["persistentvolumeclaims"]:
                    obj = h.objs["persistentvolumeclaims"].pop(key)
                else:
                    obj = _pvc(name, rng.choice(["", "pv0", "pv1", "pv2", "pv9"]), deleting=rng.random() < 0.1)
                    h.objs["persistentvolumeclaims"][key] = obj
                t.pvc_event(obj)
            elif op < 0.8:
                name = f"pv{rng.randrange(3)}"
                if rng.random() < 0.2 and name in h.objs["persistentvolumes"]:
                    obj = h.objs["persistentvolumes"].pop(name)
                else:
                    obj = _pv(name, host=rng.choice([None, None, "n1"]), zone=rng.choice([None, None, "z1"]),
                              csi=rng.random() < 0.7, ebs=rng.random() < 0.1)
                    h.objs["persistentvolumes"][name] = obj
                t.pv_event(obj)
            elif op < 0.85:
                prov = rng.choice(["nfs.csi.k8s.io", "kubernetes.io/no-provisioner", "ebs.csi.aws.com"])
                obj = {"metadata": {"name": "shared"}, "provisioner": prov}
                h.objs["storageclasses"]["shared"] = obj
                t.sc_event(obj)
            elif op < 0.9:
                h.gen["csinodes"] += 1
                h.objs["csinodes"] = {} if rng.random() < 0.5 else {"n0": {"metadata": {"name": "n0"}, "spec": {
                    "drivers": [{"name": rng.choice(["nfs.csi.k8s.io", "ebs.csi.aws.com"]),
                                 "allocatable": {"count": 4}}]}}}
            else:
                h.cache.csi_limit_drivers = rng.choice([{}, {}, {"nfs.csi.k8s.io": 1}, {"ebs.csi.aws.com": 2}])
            before, vbefore = dict(t.table), dict(t.vols)
            full, changed, removed, vfull, vchanged, vremoved = t.refresh()
            assert t.table == lane_claims(h), (seed, _step)
            assert t.vols == claim_volumes(h), (seed, _step)
            if full is None:
                assert {**{k: v for k, v in before.items() if k not in removed}, **changed} == t.table
                assert {**{k: v for k, v in vbefore.items() if k not in vremoved}, **vchanged} == t.vols
                assert not (set(changed) & removed) and not (set(vchanged) & vremoved)
            adds, removes = adds + len(changed), removes + len(removed)
    assert adds > 20 and removes > 20             # the sequences move claims both ways
