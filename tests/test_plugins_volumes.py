"""Volume plugins (VolumeBinding, VolumeZone, VolumeRestrictions, NodeVolumeLimits, in-tree
limits), ImageLocality and NodePreferAvoidPods through the scheduler (upstream v1.20
defaults kept by the reference's profile), with the fake PV controller
completing bindings after PreBind."""
import asyncio
import json

from yoda_scheduler_amd.fakeapi.pvcontroller import FakePVController
from yoda_scheduler_amd.models.pod import PodInfo, normalize_image
from yoda_scheduler_amd.models.selectors import NodeSelector
from yoda_scheduler_amd.plugins.volumes import ANN_SELECTED_NODE
from yoda_scheduler_amd.testing import FakeCluster, yoda_config


def run(c):
    return asyncio.run(c)


def pvc(name, sc="", size="10Gi", volume="", modes=("ReadWriteOnce",)):
    spec = {"accessModes": list(modes), "resources": {"requests": {"storage": size}}, "storageClassName": sc}
    if volume:
        spec["volumeName"] = volume
    return {"metadata": {"name": name, "namespace": "default"}, "spec": spec,
            "status": {"phase": "Bound" if volume else "Pending"}}


def pv(name, sc="", size="10Gi", host=None, labels=None, csi=None, claim=None, **src):
    spec = {"capacity": {"storage": size}, "accessModes": ["ReadWriteOnce"], "storageClassName": sc, **src}
    if host:
        spec["nodeAffinity"] = {"required": {"nodeSelectorTerms": [{"matchExpressions": [
            {"key": "kubernetes.io/hostname", "operator": "In", "values": [host]}]}]}}
    if csi:
        spec["csi"] = csi
    if claim:
        spec["claimRef"] = {"namespace": "default", "name": claim}
    return {"metadata": {"name": name, "labels": dict(labels or {})}, "spec": spec,
            "status": {"phase": "Bound" if claim else "Available"}}


def sc(name, provisioner="kubernetes.io/no-provisioner", wffc=True, topo=None):
    o = {"metadata": {"name": name}, "provisioner": provisioner,
         "volumeBindingMode": "WaitForFirstConsumer" if wffc else "Immediate"}
    if topo:
        o["allowedTopologies"] = topo
    return o


def claim_vol(claim, name="data"):
    return {"name": name, "persistentVolumeClaim": {"claimName": claim}}


def condition_msg(c, pod):
    for cond in (c.pod(pod).get("status") or {}).get("conditions") or []:
        if cond.get("type") == "PodScheduled":
            return cond.get("message", "")
    return ""


def test_node_selector_semantics():
    s = NodeSelector({"nodeSelectorTerms": [
        {"matchExpressions": [{"key": "zone", "operator": "In", "values": ["a"]},
                              {"key": "gen", "operator": "Gt", "values": ["3"]}]},
        {"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["special"]}]}]})
    assert s.matches("n", {"zone": "a", "gen": "4"})
    assert not s.matches("n", {"zone": "a", "gen": "3"}) and not s.matches("n", {"zone": "b", "gen": "9"})
    assert s.matches("special", {})
    assert not NodeSelector({"nodeSelectorTerms": [{}]}).matches("n", {"a": "b"})
    assert normalize_image("rocm/pytorch") == "rocm/pytorch:latest"
    assert normalize_image("reg:5000/img") == "reg:5000/img:latest"
    assert normalize_image("img:v1") == "img:v1" and normalize_image("img@sha256:ab") == "img@sha256:ab"


def test_static_pv_binding_follows_pv_node_affinity():
    async def go():
        c = FakeCluster(yoda_config())
        for n in ("n0", "n1", "n2"):
            c.add_node(n)
        c.server.create("storageclasses", sc("local"))
        c.server.create("persistentvolumes", pv("pv-small", "local", "5Gi", host="n1"))
        c.server.create("persistentvolumes", pv("pv-big", "local", "100Gi", host="n1"))
        c.server.create("persistentvolumes", pv("pv-fit", "local", "20Gi", host="n1"))
        c.server.create("persistentvolumes", pv("pv-other", "slow", "20Gi", host="n2"))
        c.server.create("persistentvolumeclaims", pvc("data", "local", "10Gi"))
        ctl = FakePVController(c.server)
        await c.start()
        ctl.start()
        c.add_pod("p", {"scv/memory": "1000"}, volumes=[claim_vol("data")])
        ok = await c.wait_bound(1)
        claim = c.server.get("persistentvolumeclaims", "data", "default")
        await ctl.stop()
        await c.stop()
        return ok, c.node_of("p"), claim
    ok, node, claim = run(go())
    assert ok
    assert node == "n1"                                  # the only node with a matching PV
    # ... and of n1's PVs the smallest one that fits was chosen
    assert claim["spec"]["volumeName"] == "pv-fit" and claim["status"]["phase"] == "Bound"


def test_dynamic_provisioning_respects_allowed_topologies():
    async def go():
        c = FakeCluster(yoda_config())
        c.add_node("n0", labels={"topology.kubernetes.io/zone": "z1"})
        c.add_node("n1", labels={"topology.kubernetes.io/zone": "z2"})
        c.server.create("storageclasses", sc("fast", "csi.example.com", topo=[{"matchLabelExpressions": [
            {"key": "topology.kubernetes.io/zone", "values": ["z2"]}]}]))
        c.server.create("persistentvolumeclaims", pvc("scratch", "fast", "50Gi"))
        ctl = FakePVController(c.server)
        await c.start()
        ctl.start()
        c.add_pod("p", {"scv/memory": "1000"}, volumes=[claim_vol("scratch")])
        ok = await c.wait_bound(1)
        claim = c.server.get("persistentvolumeclaims", "scratch", "default")
        await ctl.stop()
        await c.stop()
        return ok, c.node_of("p"), claim, ctl.provisioned
    ok, node, claim, provisioned = run(go())
    assert ok and node == "n1"
    assert claim["metadata"]["annotations"][ANN_SELECTED_NODE] == "n1"
    assert provisioned == 1 and claim["status"]["phase"] == "Bound"


def test_missing_and_unbound_immediate_claims_are_unschedulable():
    async def go():
        c = FakeCluster(yoda_config())
        c.add_node("n0")
        c.server.create("storageclasses", sc("imm", "csi.example.com", wffc=False))
        c.server.create("persistentvolumeclaims", pvc("later", "imm"))
        await c.start()
        c.add_pod("a", {"scv/memory": "1"}, volumes=[claim_vol("nope")])
        c.add_pod("b", {"scv/memory": "1"}, volumes=[claim_vol("later")])
        await c.wait(lambda: condition_msg(c, "a") and condition_msg(c, "b"), 3.0)
        ma, mb = condition_msg(c, "a"), condition_msg(c, "b")
        # once the claim is bound (by someone else), the pod schedules
        c.server.create("persistentvolumes", pv("pv-l", "imm", claim="later"))
        c.server.patch("persistentvolumeclaims", "later", {"spec": {"volumeName": "pv-l"}, "status": {"phase": "Bound"}},
                       namespace="default")
        ok = await c.wait(lambda: c.node_of("b") == "n0", 5.0)
        await c.stop()
        return ma, mb, ok
    ma, mb, ok = run(go())
    assert 'persistentvolumeclaim "nope" not found' in ma
    assert "unbound immediate PersistentVolumeClaims" in mb
    assert ok


def test_volume_zone_and_bound_pv_affinity():
    async def go():
        c = FakeCluster(yoda_config())
        c.add_node("n0", labels={"topology.kubernetes.io/zone": "z1"})
        c.add_node("n1", labels={"topology.kubernetes.io/zone": "z2"})
        c.server.create("persistentvolumes", pv("pv-z2", labels={"topology.kubernetes.io/zone": "z2__z3"},
                                                claim="zonal"))
        c.server.create("persistentvolumeclaims", pvc("zonal", volume="pv-z2"))
        await c.start()
        for i in range(3):
            c.add_pod(f"p{i}", {"scv/memory": "1000"}, volumes=[claim_vol("zonal")])
        ok = await c.wait_bound(3)
        nodes = {c.node_of(f"p{i}") for i in range(3)}
        await c.stop()
        return ok, nodes
    ok, nodes = run(go())
    assert ok and nodes == {"n1"}


def test_volume_restrictions_gce_pd_conflict():
    async def go():
        c = FakeCluster(yoda_config())
        c.add_node("n0")
        c.add_node("n1")
        await c.start()
        vol = [{"name": "d", "gcePersistentDisk": {"pdName": "disk-1"}}]
        ro = [{"name": "d", "gcePersistentDisk": {"pdName": "disk-2", "readOnly": True}}]
        c.add_pod("a", {"scv/memory": "1"}, volumes=vol)
        await c.wait_bound(1)
        c.add_pod("b", {"scv/memory": "1"}, volumes=vol)
        await c.wait_bound(2)
        c.add_pod("c", {"scv/memory": "1"}, volumes=vol)      # both nodes hold disk-1 read-write
        for i in range(4):                                     # read-only mounts share freely
            c.add_pod(f"r{i}", {"scv/memory": "1"}, volumes=ro)
        await c.wait_bound(6)
        await c.wait(lambda: condition_msg(c, "c"), 3.0)
        out = (c.node_of("a"), c.node_of("b"), c.node_of("c"), condition_msg(c, "c"))
        await c.stop()
        return out
    a, b, cc, msg = run(go())
    assert {a, b} == {"n0", "n1"} and cc == ""
    assert "no available disk" in msg


def test_csi_and_in_tree_attach_limits():
    async def go():
        c = FakeCluster(yoda_config())
        c.add_node("n0")
        c.add_node("n1")
        # n0: CSI driver limit 1, EBS limit 1; n1 unlimited CSI, default EBS
        c.server.create("csinodes", {"metadata": {"name": "n0"}, "spec": {"drivers": [
            {"name": "csi.example.com", "nodeID": "n0", "allocatable": {"count": 1}}]}})
        node = c.server.get("nodes", "n0")
        alloc = dict(node["status"]["allocatable"], **{"attachable-volumes-aws-ebs": "1"})
        c.server.patch("nodes", "n0", {"status": {"allocatable": alloc}})
        for i in range(2):
            c.server.create("persistentvolumes", pv(f"csi-{i}", csi={"driver": "csi.example.com",
                                                                      "volumeHandle": f"h{i}"}, claim=f"c{i}"))
            c.server.create("persistentvolumeclaims", pvc(f"c{i}", volume=f"csi-{i}"))
        await c.start()
        c.add_pod("x0", {"scv/memory": "1"}, volumes=[claim_vol("c0")])
        await c.wait_bound(1)
        first = c.node_of("x0")
        c.add_pod("x1", {"scv/memory": "1"}, volumes=[claim_vol("c1")])
        await c.wait_bound(2)
        e = [{"name": "e", "awsElasticBlockStore": {"volumeID": f"vol-{i}"}} for i in range(2)]
        c.add_pod("e0", {"scv/memory": "1"}, volumes=[e[0]])
        await c.wait_bound(3)
        c.add_pod("e1", {"scv/memory": "1"}, volumes=[e[1]])
        await c.wait_bound(4)
        out = first, c.node_of("x1"), c.node_of("e0"), c.node_of("e1")
        await c.stop()
        return out
    first, second, e0, e1 = run(go())
    # whichever node the first CSI pod took, a second distinct CSI volume may not exceed n0's limit of 1
    assert not (first == "n0" and second == "n0")
    assert not (e0 == "n0" and e1 == "n0")


def test_image_locality_and_prefer_avoid_pods():
    async def go():
        c = FakeCluster(yoda_config())
        for n in ("n0", "n1", "n2"):
            c.add_node(n)
        c.server.patch("nodes", "n2", {"status": {"images": [
            {"names": ["rocm/vllm:v1", "docker.io/rocm/vllm:v1"], "sizeBytes": 900 * 1024 * 1024}]}})
        avoid = {"preferAvoidPods": [{"podSignature": {"podController": {
            "kind": "ReplicaSet", "uid": "rs-1", "apiVersion": "apps/v1", "name": "web"}}}]}
        for n in ("n0", "n2"):
            c.server.patch("nodes", n, {"metadata": {"annotations": {
                "scheduler.alpha.kubernetes.io/preferAvoidPods": json.dumps(avoid)}}})
        await c.start()
        fw = c.sched.frameworks["yoda-scheduler"]
        c.add_pod("img", {"scv/memory": "1000"}, containers=[{"name": "c", "image": "rocm/vllm:v1"}])
        await c.wait_bound(1)
        owned = c.server.create("pods", {
            "metadata": {"name": "rs-pod", "namespace": "default", "labels": {"scv/memory": "1000"},
                         "ownerReferences": [{"kind": "ReplicaSet", "uid": "rs-1", "name": "web", "controller": True}]},
            "spec": {"schedulerName": "yoda-scheduler", "containers": [{"name": "c", "image": "x"}]}})
        await c.wait_bound(2)
        plain = PodInfo.from_obj(c.server.create("pods", {
            "metadata": {"name": "plain", "namespace": "default", "labels": {"scv/memory": "1"}},
            "spec": {"schedulerName": "yoda-scheduler", "containers": [{"name": "c", "image": "x"}]}}))
        native_plain = fw.native_for(plain)
        native_owned = fw.native_for(PodInfo.from_obj(owned))
        out = c.node_of("img"), c.node_of("rs-pod"), native_plain, native_owned
        await c.stop()
        return out
    img, rs, native_plain, native_owned = run(go())
    assert img == "n2"                 # the only node holding the image
    assert rs == "n1"                  # the only node not avoiding the ReplicaSet
    # both score natively now (engine S_IMAGE_LOCALITY / S_PREFER_AVOID): neither the image on
    # n2 nor the ReplicaSet owner moves a pod off the native cycle
    assert native_plain and native_owned


def test_volume_plugins_keep_plain_pods_native():
    async def go():
        c = FakeCluster(yoda_config())
        c.add_node("n0")
        await c.start()
        fw = c.sched.frameworks["yoda-scheduler"]
        names = {p.name for p in fw.conditional}
        plain = PodInfo.from_obj({"metadata": {"name": "p", "namespace": "default", "uid": "u"},
                                  "spec": {"schedulerName": "yoda-scheduler"}})
        with_pvc = PodInfo.from_obj({"metadata": {"name": "q", "namespace": "default", "uid": "v"},
                                     "spec": {"schedulerName": "yoda-scheduler", "volumes": [claim_vol("x")]}})
        informers = set(c.sched.informers)
        await c.stop()
        return names, fw.native_for(plain), fw.native_for(with_pvc), informers
    names, plain, with_pvc, informers = run(go())
    assert {"VolumeBinding", "VolumeZone", "VolumeRestrictions", "NodeVolumeLimits"} <= names
    assert "ImageLocality" not in names and "PodTopologySpread" not in names   # native score terms now
    assert plain and not with_pvc
    assert {"persistentvolumeclaims", "persistentvolumes", "storageclasses", "csinodes"} <= informers


def test_flag_fast_path_agrees_with_plugins():
    """The one-mask native_for fast path must give the same answer as asking every
    conditional plugin, for plain pods and for each optional feature."""
    specs = [
        {},
        {"volumes": [{"name": "t", "projected": {"sources": []}}, {"name": "c", "configMap": {"name": "x"}}]},
        {"volumes": [claim_vol("x")]},
        {"volumes": [{"name": "e", "ephemeral": {"volumeClaimTemplate": {}}}]},
        {"volumes": [{"name": "d", "gcePersistentDisk": {"pdName": "a"}}]},
        {"volumes": [{"name": "d", "azureDisk": {"diskName": "a"}}]},
        {"containers": [{"name": "c", "image": "x", "ports": [{"containerPort": 80, "hostPort": 8080}]}]},
        {"topologySpreadConstraints": [{"maxSkew": 1, "topologyKey": "z", "labelSelector": {}}]},
        {"affinity": {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": []}}},
        {"affinity": {"nodeAffinity": {}}},
    ]

    async def go():
        c = FakeCluster(yoda_config())
        c.add_node("n0")
        await c.start()
        fw = c.sched.frameworks["yoda-scheduler"]
        out = []
        for i, sp in enumerate(specs):
            for owner in (None, {"kind": "ReplicaSet", "uid": "r", "controller": True}):
                meta = {"name": f"p{i}", "namespace": "default", "uid": f"u{i}"}
                if owner:
                    meta["ownerReferences"] = [owner]
                pi = PodInfo.from_obj({"metadata": meta, "spec": {"schedulerName": "yoda-scheduler", **sp}})
                out.append((i, bool(owner), fw.native_for(pi), all(p.is_noop_for(pi) for p in fw.conditional)))
        await c.stop()
        return out
    rows = run(go())
    assert all(fast == slow for _, _, fast, slow in rows), rows
    assert rows[0][2] and rows[2][2] and not rows[4][2] and not rows[6][2]
