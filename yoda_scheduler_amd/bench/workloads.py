"""The five BASELINE.json burst configurations as synthetic, seeded workloads.

| # | BASELINE config                                                         | cluster                        |
|---|-------------------------------------------------------------------------|--------------------------------|
| 1 | 1 pod, scv/memory=1000, 1-node cluster with fake-GPU CRD                | 1 node × 8 MI355X              |
| 2 | 100-pod burst, scv/memory, single 1×MI355X node                         | 1 node × 1 MI355X              |
| 3 | 1000-pod burst, mixed scv/memory + scv/number, single 8×MI355X node     | 1 node × 8 MI355X (headline)   |
| 4 | 1000-pod burst, scv/clock high-perf labels, 4 nodes × 8×MI355X          | 2×MI355X(2400) + 2×MI350X(2200)|
| 5 | 5000-pod burst, mixed + multi-GPU pods, 4 nodes × 8×MI355X              | 4 nodes × 8 MI355X             |

Config 4 mixes MI355X (2400 MHz max sclk) and MI350X (2200 MHz) nodes so the exact-match
``scv/clock`` selector has something to select. Demand is sized
so every pod fits with per-GPU HBM reservation (≈60-75 % of HBM), i.e. the burst
measures scheduling, not capacity exhaustion.

``cluster="kind"`` (``bench.py --cluster kind``) makes any config look like the cluster
BASELINE config 1 names — a kind cluster — instead of the bare synthetic one: every node
reports 50 preloaded images in ``status.images`` and allocatable ``ephemeral-storage`` /
hugepages, the cluster has the ``default/kubernetes`` and ``kube-system/kube-dns`` Services,
30 % of the burst is owned by a ReplicaSet that a Service selects (so the System default
topology-spread constraints apply to them), 20 % request ``ephemeral-storage`` and 10 % run an
image the nodes already hold (ImageLocality has something to score). Each of these alone used
to move pods — or the whole profile — off the native lane.

``cluster="cloud"`` (``bench.py --cluster cloud``) is the kind burst on a zoned pool: every node
carries a zone label (3 zones) and the hot image sits on 30 % of the nodes at varying sizes, so
default spreading and ImageLocality differ per node (``cloudify_node``).
"""
from __future__ import annotations

import random
import re
import time
from dataclasses import dataclass, field
from typing import Optional

from ..models.device import MI350X, MI355X, GpuSpec, make_node, make_scv
from ..models.scv import Card, Scv


@dataclass
class Workload:
    id: int
    name: str
    nodes: list[tuple[str, GpuSpec, int]]            # (name, spec, gpus)
    pods: list[dict] = field(default_factory=list)   # label dicts
    scheduler_name: str = "yoda-scheduler"
    specs: dict = field(default_factory=dict)        # pod index → extra spec fields (e.g. affinity)
    metas: dict = field(default_factory=dict)        # pod index → extra metadata fields (ownerReferences)
    objects: list = field(default_factory=list)      # (resource, object) created with the cluster (PVCs, PVs)
    cluster: str = "synthetic"                       # "kind": realistic node/cluster objects (populate)
    wait_bound: bool = False                         # a burst ends when every pod is bound (preemptors
                                                     # park in backoff while their victims go)

    @property
    def n_pods(self) -> int:
        return len(self.pods)


def _mixed_labels(rng: random.Random) -> dict:
    r = rng.random()
    if r < 0.60:
        return {"scv/memory": str(rng.choice([256, 512, 1024, 2048]))}
    if r < 0.70:
        return {"scv/number": "1"}
    if r < 0.88:
        return {"scv/number": "2", "scv/memory": str(rng.choice([512, 1024]))}
    if r < 0.97:
        return {"scv/number": "4", "scv/memory": "1024"}
    return {"scv/number": "8", "scv/memory": "1024"}


def make_workload(cfg: int, seed: int = 0, template: Optional[Card] = None,
                  node_gpus: Optional[int] = None, nodes: Optional[int] = None, mix_anti: int = 0,
                  cluster: str = "synthetic", mix_spread: int = 0, mix_volumes: int = 0,
                  mix_hostports: int = 0, mix_preempt: int = 0, prefill: float = 0.0) -> Workload:
    """``node_gpus`` overrides the GPUs per node (BASELINE.md protocol item 5: every
    config at 1, 2, 4 and 8 GPUs per node); pods keep their labels, so e.g. ``scv/number: 8``
    pods are unschedulable on smaller nodes and are reported as such. ``nodes`` resizes
    config 6's cluster (beyond BASELINE: the CPU/device crossover end to end). ``cluster``
    "kind" makes the cluster and the burst realistic (module docstring)."""
    w = _make_workload(cfg, seed, template)
    if cluster == "kind":
        _kindify(w, seed)
    elif cluster == "cloud":
        _kindify(w, seed)
        w.cluster = "cloud"
        w.name = w.name.replace("[kind cluster]", "[cloud cluster: 3 zones, images on 30% of nodes]")
    elif cluster != "synthetic":
        raise ValueError(f"unknown cluster kind {cluster!r}")
    if mix_anti:
        # beyond BASELINE: interleave pods with required pod anti-affinity (Python-path plugins
        # that read other pods, lane pods included) — what such pods cost the native lane
        n = len(w.pods)
        for j in range(mix_anti):
            i = (j + 1) * n // (mix_anti + 1)
            w.pods[i] = {"app": f"anti-{j}", "scv/memory": "1024"}
            w.specs[i] = {"affinity": {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchLabels": {"app": f"anti-{j}"}}, "topologyKey": "kubernetes.io/hostname"}]}}}
        w.name += f" + {mix_anti} required-anti-affinity pods"
    if mix_spread:
        # beyond BASELINE: pods with a hostname DoNotSchedule spread constraint over their own group
        n = len(w.pods)
        for j in range(min(mix_spread, n)):
            i = j * n // min(mix_spread, n)
            w.pods[i] = dict(w.pods[i], group=f"g{i % 8}")
            w.specs[i] = dict(w.specs.get(i) or {}, topologySpreadConstraints=[{
                "maxSkew": 1, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "DoNotSchedule",
                "labelSelector": {"matchLabels": {"group": f"g{i % 8}"}}}])
        w.name += f" + {min(mix_spread, n)} hostname-spread pods"
    if mix_volumes:
        _add_volume_pods(w, mix_volumes)
    if mix_hostports:
        # beyond BASELINE: pods with a host port each (distinct ports: all fit on one node), as
        # hostNetwork training pods carry — native NodePorts since round 5
        n = len(w.pods)
        count = min(mix_hostports, n)
        for j in range(count):
            i = j * n // count
            spec = dict(w.specs.get(i) or {})
            c = dict((spec.get("containers") or [{"name": "main", "image": "rocm/pytorch:latest",
                                                   "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}}}])[0])
            c["ports"] = [{"containerPort": 29500, "hostPort": 20000 + j, "protocol": "TCP"}]
            spec["containers"] = [c]
            w.specs[i] = spec
        w.name += f" + {count} host-port pods"
    if mix_preempt:
        _preempt_burst(w, mix_preempt, seed)
    elif prefill > 0:
        _prefill(w, prefill, seed)
    if nodes is not None:
        if cfg != 6 or nodes < 1:
            raise ValueError("nodes: config 6 only, >= 1")
        spec = w.nodes[0][1]
        w.nodes = [(f"node-{i}", spec, 8) for i in range(nodes)]
        w.name = w.name.replace("4096 nodes", f"{nodes} nodes")
    if node_gpus is not None:
        if node_gpus < 1:
            raise ValueError("node_gpus must be >= 1")
        w.nodes = [(name, spec, node_gpus) for name, spec, _g in w.nodes]
        w.name = re.sub(r"x \d+ (MI3\d\dX|GPUs)", rf"x {node_gpus} \1", w.name)
    return w


def _make_workload(cfg: int, seed: int = 0, template: Optional[Card] = None) -> Workload:
    rng = random.Random(seed * 7919 + cfg)
    if cfg == 1:
        w = Workload(1, "1 pod scv/memory=1000, 1 node x 8 MI355X (fake CRD)", [("node-0", MI355X, 8)])
        w.pods = [{"scv/memory": "1000"}]
    elif cfg == 2:
        w = Workload(2, "100-pod burst scv/memory, 1 node x 1 MI355X", [("node-0", MI355X, 1)])
        w.pods = [{"scv/memory": str(rng.choice([512, 1024, 2048]))} for _ in range(100)]
    elif cfg == 3:
        w = Workload(3, "1000-pod burst mixed scv/memory+scv/number, 1 node x 8 MI355X", [("node-0", MI355X, 8)])
        w.pods = [_mixed_labels(rng) for _ in range(1000)]
    elif cfg == 4:
        w = Workload(4, "1000-pod burst scv/clock, 4 nodes x 8 GPUs (2x MI355X@2400, 2x MI350X@2200)",
                     [("node-0", MI355X, 8), ("node-1", MI355X, 8), ("node-2", MI350X, 8), ("node-3", MI350X, 8)])
        w.pods = []
        for _ in range(1000):
            lab = {"scv/clock": "2400" if rng.random() < 0.7 else "2200",
                   "scv/memory": str(rng.choice([1024, 2048, 4096]))}
            if rng.random() < 0.1:
                lab["scv/number"] = "2"
            w.pods.append(lab)
    elif cfg == 5:
        w = Workload(5, "5000-pod burst mixed + multi-GPU, 4 nodes x 8 MI355X (xGMI gang scoring)",
                     [(f"node-{i}", MI355X, 8) for i in range(4)])
        w.pods = [_mixed_labels(rng) for _ in range(5000)]
    elif cfg == 6:
        # beyond BASELINE: a large cluster where the gfx950 device scorer takes the cycle
        w = Workload(6, "1000-pod burst mixed + multi-GPU, 4096 nodes x 8 MI355X (device scorer)",
                     [(f"node-{i}", MI355X, 8) for i in range(4096)])
        w.pods = [_mixed_labels(rng) for _ in range(1000)]
    else:
        raise ValueError(f"unknown config {cfg}")
    return w


# ---------------------------------------------------------------- populated cluster (--prefill)
def _filler(w: Workload, k: int, node: str, g: int, mb: int, prio: int) -> tuple:
    """A bound pod holding card ``g`` of ``node`` whole (its GPU annotation, as the scheduler
    writes it at bind time), of one of 17 jobs."""
    return ("pods", {
        "apiVersion": "v1", "kind": "Pod",
        "metadata": {"name": f"filler-{k}", "namespace": "default",
                     "labels": {"app": f"job-{k % 17}", "scv/memory": str(mb)},
                     "annotations": {"scv.amd.com/gpus": str(g), "scv.amd.com/reserved-mb": str(mb)}},
        "spec": {"schedulerName": w.scheduler_name, "nodeName": node, "priority": prio,
                 "containers": [{"name": "main", "image": "rocm/pytorch:latest",
                                 "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}}}]},
        "status": {"phase": "Running"}})


def _prefill(w: Workload, frac: float, seed: int) -> None:
    """Beyond BASELINE: the burst lands on a populated cluster — a fraction
    ``frac`` of all cards (a seeded choice) is held whole by bound pods, so the ledger, the label
    index and the device rows start full of other pods, and the burst's pods fit only on the
    free cards (the 8-GPU ones on wholly free nodes)."""
    rng = random.Random(seed * 7717 + int(frac * 1000))
    k = 0
    for name, spec, gpus in w.nodes:
        for g in range(gpus):
            if rng.random() < frac:
                w.objects.append(_filler(w, k, name, g, spec.hbm_mb, 0))
                k += 1
    w.name += f" + {k} pods already bound ({frac:.0%} of the cards)"


# ---------------------------------------------------------------- preemption (--mix-preempt)
def _preempt_burst(w: Workload, count: int, seed: int) -> None:
    """Beyond BASELINE: a full cluster — every GPU of every node held by a
    bound low-priority pod (priorities 0-5, one full card each, as ``scripts/preempt_bench.py``) —
    and a burst of ``count`` priority-100 pods that each need one whole card. Each of them fails
    the filters, DefaultPreemption (the native search, upstream v1.20 candidate pruning) picks a
    node and victims, the victims are deleted through the API, and the pod binds once they are
    gone. The fillers are cluster objects (``w.objects``): with ``--transport inproc`` every step
    runs on a freshly populated shard, so every step preempts."""
    rng = random.Random(seed * 104729 + count)
    fillers = []
    k = 0
    for name, spec, gpus in w.nodes:
        for g in range(gpus):
            fillers.append(_filler(w, k, name, g, spec.hbm_mb, rng.randint(0, 5)))
            k += 1
    count = min(count, k)
    # three quarters of a card: the card's Scv telemetry (jittered, or a real amd-smi sample with
    # the driver's own use) never reports it entirely free, so a whole-card request would fit
    # only the few cards that happen to report full; any evicted filler's card fits this
    mb = w.nodes[0][1].hbm_mb * 3 // 4
    w.objects.extend(fillers)
    w.pods = [{"scv/memory": str(mb)} for _ in range(count)]
    w.specs = {i: {"priority": 100} for i in range(count)}
    w.wait_bound = True
    w.metas = {}
    w.name += f" + full cluster ({k} low-priority pods), burst of {count} preemptors"


# ---------------------------------------------------------------- PVC pods (--mix-volumes)
VOLUME_CLAIMS = 4           # ReadWriteMany claims the volume pods share (a dataset / checkpoint share)


def volume_objects() -> list:
    """Bound CSI PersistentVolumes and their claims, as a PV controller leaves them."""
    out = []
    for j in range(VOLUME_CLAIMS):
        claim, pv = f"data-{j}", f"pv-data-{j}"
        out.append(("persistentvolumes", {
            "apiVersion": "v1", "kind": "PersistentVolume", "metadata": {"name": pv},
            "spec": {"capacity": {"storage": "10Ti"}, "accessModes": ["ReadWriteMany"], "storageClassName": "shared",
                     "csi": {"driver": "nfs.csi.k8s.io", "volumeHandle": f"share-{j}"},
                     "claimRef": {"kind": "PersistentVolumeClaim", "namespace": "default", "name": claim}},
            "status": {"phase": "Bound"}}))
        out.append(("persistentvolumeclaims", {
            "apiVersion": "v1", "kind": "PersistentVolumeClaim", "metadata": {"name": claim, "namespace": "default"},
            "spec": {"accessModes": ["ReadWriteMany"], "resources": {"requests": {"storage": "10Ti"}},
                     "storageClassName": "shared", "volumeName": pv},
            "status": {"phase": "Bound"}}))
    return out


def _add_volume_pods(w: Workload, count: int) -> None:
    """Beyond BASELINE: ``count`` pods of the burst mount a bound PVC, so the volume plugins
    (VolumeBinding, VolumeZone, NodeVolumeLimits, the in-tree attach limits) apply to them and
    they take the Python cycle beside the native lane — what a pod that genuinely needs a
    Python plugin costs."""
    n = len(w.pods)
    count = min(count, n)
    for j in range(count):
        i = j * n // count
        w.specs[i] = dict(w.specs.get(i) or {}, volumes=[
            {"name": "data", "persistentVolumeClaim": {"claimName": f"data-{j % VOLUME_CLAIMS}"}}])
    w.objects.extend(volume_objects())
    w.name += f" + {count} PVC pods"


# ---------------------------------------------------------------- kind cluster (--cluster kind)
KIND_IMAGES = (
    # what a kind v1.2x node image preloads, then the usual ROCm / platform images of a GPU pool
    "registry.k8s.io/pause:3.9", "registry.k8s.io/kube-proxy:v1.29.2", "registry.k8s.io/kube-apiserver:v1.29.2",
    "registry.k8s.io/kube-controller-manager:v1.29.2", "registry.k8s.io/kube-scheduler:v1.29.2",
    "registry.k8s.io/etcd:3.5.10-0", "registry.k8s.io/coredns/coredns:v1.11.1",
    "docker.io/kindest/kindnetd:v20240202-8f1494ea", "docker.io/kindest/local-path-provisioner:v20240202-8f1494ea",
    "docker.io/kindest/local-path-helper:v20230510-486859a6",
)
KIND_HOT_IMAGE = "docker.io/rocm/vllm:v0.6.4"     # preloaded on every node; 10 % of the burst runs it
KIND_TRAINER = {"app": "trainer"}                 # Service + ReplicaSet selector of 30 % of the burst


def kind_node_images(i_node: int) -> list:
    extra = [f"docker.io/rocm/tool-{k}:v{(i_node + k) % 7}" for k in range(39)]
    names = list(KIND_IMAGES) + [KIND_HOT_IMAGE] + extra
    return [{"names": [n, n.split("/", 1)[1] if n.count("/") > 1 else n], "sizeBytes": (40 + 37 * k % 900) << 20}
            for k, n in enumerate(names)]


def _kindify(w: Workload, seed: int) -> None:
    rng = random.Random(seed * 104729 + w.id)
    w.cluster = "kind"
    w.name += " [kind cluster]"
    for i in range(len(w.pods)):
        r = rng.random()
        if r < 0.30:                                   # a ReplicaSet's pods, selected by a Service
            w.pods[i] = dict(w.pods[i], **KIND_TRAINER)
            w.metas[i] = {"ownerReferences": [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "trainer-rs",
                                               "uid": "rs-trainer-0001", "controller": True,
                                               "blockOwnerDeletion": True}]}
        req = {"cpu": "100m", "memory": "128Mi"}
        if rng.random() < 0.20:
            req["ephemeral-storage"] = "1Gi"
        image = KIND_HOT_IMAGE if rng.random() < 0.10 else "rocm/pytorch:latest"
        w.specs[i] = dict(w.specs.get(i) or {}, containers=[{"name": "main", "image": image,
                                                             "resources": {"requests": req}}])


def kind_objects() -> list:
    """The cluster objects of a kind cluster that the scheduler's plugins watch."""
    return [
        ("services", {"apiVersion": "v1", "kind": "Service",
                      "metadata": {"name": "kubernetes", "namespace": "default"},
                      "spec": {"clusterIP": "10.96.0.1", "ports": [{"port": 443, "protocol": "TCP"}]}}),
        ("services", {"apiVersion": "v1", "kind": "Service",
                      "metadata": {"name": "kube-dns", "namespace": "kube-system"},
                      "spec": {"selector": {"k8s-app": "kube-dns"}, "clusterIP": "10.96.0.10",
                               "ports": [{"port": 53, "protocol": "UDP"}]}}),
        ("services", {"apiVersion": "v1", "kind": "Service",
                      "metadata": {"name": "trainer", "namespace": "default"},
                      "spec": {"selector": dict(KIND_TRAINER), "ports": [{"port": 29500, "protocol": "TCP"}]}}),
        ("replicasets", {"apiVersion": "apps/v1", "kind": "ReplicaSet",
                         "metadata": {"name": "trainer-rs", "namespace": "default", "uid": "rs-trainer-0001"},
                         "spec": {"replicas": 300, "selector": {"matchLabels": dict(KIND_TRAINER)},
                                  "template": {"metadata": {"labels": dict(KIND_TRAINER)}}}}),
    ]


def kindify_node(obj: dict, i_node: int) -> dict:
    st = obj["status"]
    for k in ("allocatable", "capacity"):
        st[k] = dict(st[k], **{"ephemeral-storage": "1800Gi", "hugepages-1Gi": "0", "hugepages-2Mi": "0"})
    st["images"] = kind_node_images(i_node)
    obj["metadata"]["labels"].update({"kubernetes.io/arch": "amd64", "beta.kubernetes.io/arch": "amd64",
                                      "beta.kubernetes.io/os": "linux"})
    return obj


# ---------------------------------------------------------------- cloud pool (--cluster cloud)
CLOUD_ZONES = ("zone-a", "zone-b", "zone-c")


def cloudify_node(obj: dict, i_node: int) -> dict:
    """A managed-cloud GPU pool node (EKS / GKE / AKS shape): the kind node's images and
    resources, plus ``topology.kubernetes.io/zone`` / ``region`` labels (3 zones, round robin),
    and the hot ROCm image present on a pseudo-random 30 % of the nodes at one of several sizes
    (layers differ by node image version). So for the ReplicaSet pods the System default spreading
    (zone maxSkew 5) and for the hot-image pods ImageLocality are real per-node terms, not
    constants."""
    obj = kindify_node(obj, i_node)
    obj["metadata"]["labels"].update({"topology.kubernetes.io/zone": CLOUD_ZONES[i_node % len(CLOUD_ZONES)],
                                      "topology.kubernetes.io/region": "us-central"})
    h = (i_node * 2654435761) & 0xFFFFFFFF
    images = [im for im in obj["status"]["images"] if KIND_HOT_IMAGE not in im["names"]]
    if h % 100 < 30:
        images.append({"names": [KIND_HOT_IMAGE, KIND_HOT_IMAGE.split("/", 1)[1]],
                       "sizeBytes": (2000 + 250 * (h >> 8) % 5) << 20})
    obj["status"]["images"] = images
    return obj


def pod_object(i: int, labels: dict, scheduler_name: str, namespace: str = "default",
               prefix: str = "burst", spec: Optional[dict] = None, meta: Optional[dict] = None) -> dict:
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": f"{prefix}-{i}", "namespace": namespace, "labels": dict(labels), **(meta or {})},
            "spec": {"schedulerName": scheduler_name,
                     "containers": [{"name": "main", "image": "rocm/pytorch:latest",
                                     "resources": {"requests": {"cpu": "100m", "memory": "128Mi"}}}],
                     **(spec or {})}}


def populate(server, w: Workload, template: Optional[dict] = None, link_load: float = 0.0,
             seed: int = 0) -> None:
    """Create the workload's nodes and their Scv telemetry in a fake apiserver.
    ``template`` (from a real amd-smi sample of the local MI355X) overrides the per-card
    static fields of the MI355X nodes."""
    rng = random.Random(seed)
    if w.cluster in ("kind", "cloud"):
        for res, obj in kind_objects():
            server.create(res, obj)
    for res, obj in w.objects:
        server.create(res, obj)
    for k, (name, spec, gpus) in enumerate(w.nodes):
        # kubelet --max-pods 2048: config 5 packs 5000 HBM-sharing pods onto 4 nodes
        node = make_node(name, pods=2048)
        if w.cluster == "kind":
            node = kindify_node(node, k)
        elif w.cluster == "cloud":
            node = cloudify_node(node, k)
        server.create("nodes", node)
        scv = make_scv(name, spec, gpus, update_time=time.time(), link_load=link_load, rng=rng,
                       jitter=link_load > 0)
        scv.update_interval_ms = 60_000     # one sample stays fresh for the whole burst
        if template and spec is MI355X:     # the template is a real MI355X; MI350X nodes keep their spec
            for c in scv.status.card_list:
                for k, v in template.items():
                    setattr(c, k, v)
                c.free_memory = min(c.free_memory, c.total_memory)
            scv.status.recompute_sums()
        server.create("scvs", scv.to_json())
