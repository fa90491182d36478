"""Parsed views of v1.Pod / v1.Node objects (dict-shaped, as the apiserver returns them).

A ``PodInfo`` parses everything the scheduling cycle needs exactly once per pod
(labels → ``GpuRequest``, resource requests, selectors, tolerations) so the per-node
loops — native or Python — never touch the raw JSON again.
"""
from __future__ import annotations

import itertools
import json
import time
from dataclasses import dataclass, field
from typing import Any, Optional

from ..utils.quantity import bytes_of, cpu_millis
from .labels import GpuRequest, parse_gpu_request
from .scv import parse_rfc3339

_ids = itertools.count(1)
_num_ids: dict[str, int] = {}


def pod_num_id(uid: str) -> int:
    """Process-stable 64-bit id of a pod uid (the native ledger key)."""
    v = _num_ids.get(uid)
    if v is None:
        v = _num_ids[uid] = next(_ids)
    return v


def forget_num_id(uid: str) -> None:
    _num_ids.pop(uid, None)


def pod_key(obj: dict) -> str:
    m = obj.get("metadata") or {}
    return f"{m.get('namespace', 'default')}/{m.get('name', '')}"


DEFAULT_MILLI_CPU_REQUEST = 100                 # upstream schedutil non-zero defaults
DEFAULT_MEMORY_REQUEST = 200 * 1024 * 1024


def _requests(spec: dict) -> tuple[int, int, int, int]:
    """(cpu_m, mem, non-zero cpu_m, non-zero mem): Σ containers, max with each init
    container, + overhead. The non-zero pair substitutes upstream's defaults (100m,
    200 MiB) per container whose request is *absent* (``GetNonzeroRequests``); it feeds
    the Least/Most/Balanced allocation scores, the plain pair the resource fit."""
    cpu = mem = nzc = nzm = 0
    for c in spec.get("containers") or ():
        r = ((c.get("resources") or _EMPTY).get("requests")) or _EMPTY
        if "cpu" in r:
            v = cpu_millis(r["cpu"])
            cpu += v
            nzc += v
        else:
            nzc += DEFAULT_MILLI_CPU_REQUEST
        if "memory" in r:
            v = bytes_of(r["memory"])
            mem += v
            nzm += v
        else:
            nzm += DEFAULT_MEMORY_REQUEST
    for c in spec.get("initContainers") or ():
        r = ((c.get("resources") or _EMPTY).get("requests")) or _EMPTY
        v = cpu_millis(r["cpu"]) if "cpu" in r else 0
        cpu, nzc = max(cpu, v), max(nzc, v if "cpu" in r else DEFAULT_MILLI_CPU_REQUEST)
        v = bytes_of(r["memory"]) if "memory" in r else 0
        mem, nzm = max(mem, v), max(nzm, v if "memory" in r else DEFAULT_MEMORY_REQUEST)
    ov = spec.get("overhead")
    if ov:
        v = cpu_millis(ov["cpu"]) if "cpu" in ov else 0
        cpu += v
        nzc += v
        v = bytes_of(ov["memory"]) if "memory" in ov else 0
        mem += v
        nzm += v
    return cpu, mem, nzc, nzm


_BASIC = ("cpu", "memory")


def _has_ext(spec: dict) -> bool:
    """Cheap pre-check: does any container request something besides cpu/memory?"""
    for key in ("containers", "initContainers"):
        for c in spec.get(key) or ():
            r = (c.get("resources") or _EMPTY).get("requests")
            if r and any(k not in _BASIC for k in r):
                return True
    ov = spec.get("overhead")
    return bool(ov) and any(k not in _BASIC for k in ov)


def ext_requests(spec: dict) -> dict:
    """Requests other than cpu/memory (``amd.com/gpu``, ``ephemeral-storage``, hugepages,
    any extended resource) as integer units: max(Σ containers, max init container) +
    overhead, upstream ``computePodResourceRequest`` semantics. Empty for most pods."""
    out: dict = {}
    for c in spec.get("containers") or ():
        for k, v in (((c.get("resources") or _EMPTY).get("requests")) or _EMPTY).items():
            if k not in _BASIC:
                out[k] = out.get(k, 0) + quantity_int(v)
    for c in spec.get("initContainers") or ():
        for k, v in (((c.get("resources") or _EMPTY).get("requests")) or _EMPTY).items():
            if k not in _BASIC:
                out[k] = max(out.get(k, 0), quantity_int(v))
    for k, v in (spec.get("overhead") or _EMPTY).items():
        if k not in _BASIC:
            out[k] = out.get(k, 0) + quantity_int(v)
    return {k: v for k, v in out.items() if v}


def quantity_int(q) -> int:
    """Integer value of a quantity (bytes for storage, count for devices), rounded up."""
    return bytes_of(q)


FIELD_NODE_NAME = "@metadata.name"   # engine key of a matchFields metadata.name requirement


def _terms(terms: list | None) -> list[list[tuple[str, str, list[str]]]]:
    out = []
    for t in terms or []:
        reqs = [(e.get("key", ""), e.get("operator", "In"), [str(v) for v in e.get("values") or []])
                for e in (t.get("matchExpressions") or [])]
        # matchFields → '@'-prefixed engine keys: In / NotIn with one value on metadata.name (the
        # node name); other fields read as "" and other shapes fail the term (upstream
        # NodeSelectorRequirementsAsFieldSelector)
        for f in t.get("matchFields") or []:
            reqs.append(("@" + str(f.get("key", "")), f.get("operator", "In"),
                         [str(v) for v in f.get("values") or []]))
        out.append(reqs)
    return out


# Pod feature flags: which optional scheduling features a pod uses. Conditional Python
# plugins declare the flags that make them relevant, so the framework can decide "fully
# native cycle" for a plain pod with one mask test instead of asking every plugin.
PF_HOST_PORTS = 1
PF_SPREAD = 2          # topologySpreadConstraints
PF_POD_AFFINITY = 4    # podAffinity / podAntiAffinity
PF_CLAIMS = 8          # persistentVolumeClaim / ephemeral volumes
PF_DISKS = 16          # in-tree attachable disks (GCE PD, EBS, Azure disk, Cinder, iSCSI, RBD)
PF_CONTROLLER = 32     # controlled by a ReplicationController / ReplicaSet / StatefulSet
PF_EXTENDED = 64       # requests resources beyond cpu/memory (amd.com/gpu, ephemeral-storage, ...)
PF_POD_GROUP = 128     # member of a co-scheduled pod group (Coscheduling)
PF_REQ_ANTI = 256      # required pod anti-affinity (other pods' symmetry check)
PF_SPREAD_HARD = 512   # a DoNotSchedule topologySpreadConstraint
LABEL_POD_GROUP = "pod-group.scheduling.sigs.k8s.io"
LABEL_POD_GROUP_MIN = "pod-group.scheduling.sigs.k8s.io/min-available"

_DISK_KINDS = ("gcePersistentDisk", "awsElasticBlockStore", "azureDisk", "cinder", "iscsi", "rbd")


def pod_flags(meta: dict, spec: dict, host_ports, ext: Optional[dict] = None) -> int:
    f = PF_HOST_PORTS if host_ports else 0
    if ext:
        f |= PF_EXTENDED
    tsc = spec.get("topologySpreadConstraints")
    if tsc:
        f |= PF_SPREAD
        if any(isinstance(c, dict) and c.get("whenUnsatisfiable", "DoNotSchedule") == "DoNotSchedule" for c in tsc):
            f |= PF_SPREAD_HARD
    aff = spec.get("affinity")
    if aff and (aff.get("podAffinity") or aff.get("podAntiAffinity")):
        f |= PF_POD_AFFINITY
        anti = aff.get("podAntiAffinity")
        if isinstance(anti, dict) and anti.get("requiredDuringSchedulingIgnoredDuringExecution"):
            f |= PF_REQ_ANTI
    for v in spec.get("volumes") or ():
        if "persistentVolumeClaim" in v or "ephemeral" in v:
            f |= PF_CLAIMS
        elif any(k in v for k in _DISK_KINDS):
            f |= PF_DISKS
    if LABEL_POD_GROUP in (meta.get("labels") or _EMPTY):
        f |= PF_POD_GROUP
    for r in meta.get("ownerReferences") or ():
        if r.get("controller") and r.get("kind") in ("ReplicationController", "ReplicaSet", "StatefulSet"):
            f |= PF_CONTROLLER
    return f


class PodInfo:
    """Parsed pod. ``__slots__`` + a hand-written constructor: one of these is built per
    pod per informer event on the scheduling hot path.

    ``obj`` (the full pod dict) is lazy for pods that arrive through the native transport:
    the C++ projection already holds every field the cycle reads, so the JSON is decoded
    only if something (an extender, a Python plugin, an event) asks for the object."""

    __slots__ = ("_obj", "_src", "uid", "namespace", "name", "num_id", "labels", "gpu", "scheduler_name", "node_name",
                 "cpu_m", "mem", "priority", "node_selector", "required_terms", "preferred_terms", "tolerations",
                 "annotations", "host_ports", "attempts", "initial_attempt", "enqueued", "native_req",
                 "native_owner", "assigned_cards", "_creation", "flags", "ext", "nz_cpu_m", "nz_mem", "applies_memo",
                 "images", "containers", "owner", "avoid", "spread", "deleting", "pod_aff", "vol_memo")

    def __init__(self, obj: dict, uid: str, namespace: str, name: str, num_id: int, labels: dict, gpu: GpuRequest,
                 scheduler_name: str = "default-scheduler", node_name: str = "", cpu_m: int = 0, mem: int = 0,
                 priority: int = 0, node_selector: Optional[dict] = None, required_terms: Optional[list] = None,
                 preferred_terms: Optional[list] = None, tolerations: Optional[list] = None,
                 annotations: Optional[dict] = None, host_ports: Optional[list] = None, flags: int = 0,
                 ext: Optional[dict] = None, nz_cpu_m: int = -1, nz_mem: int = -1,
                 images: Optional[list] = None, containers: int = 0, owner: Optional[tuple] = None,
                 avoid: Optional[tuple] = None, spread: Optional[list] = None, deleting: bool = False,
                 pod_aff: Optional[tuple] = None) -> None:
        self._obj = obj
        # default-plugin inputs the native engine reads (ops/native.py::pod_req): normalized
        # images of spec.containers + their count (ImageLocality), the first controller
        # ownerReference (apiVersion, kind, name, uid) (DefaultSelector), the first RC / RS
        # controller (kind, uid) (NodePreferAvoidPods), the topology spread constraints as
        # (topologyKey, maxSkew, whenUnsatisfiable, LabelSelector.native() | None), and whether
        # the pod is terminating (other pods' spread counts skip it)
        self.images = images if images is not None else _NOLIST
        self.containers = containers
        self.owner = owner
        self.avoid = avoid
        self.spread = spread
        self.deleting = deleting
        # (required affinity, required anti-affinity, preferred affinity, preferred anti-affinity),
        # each [(topologyKey, namespaces | None, LabelSelector.native() | None, weight)]
        self.pod_aff = pod_aff
        self.vol_memo: Optional[tuple] = None   # volume plugins' no-op answers (plugins/volumes.py)
        self._src = None
        # -1: a single container's non-zero request derived from cpu_m / mem
        self.nz_cpu_m = nz_cpu_m if nz_cpu_m >= 0 else (cpu_m or DEFAULT_MILLI_CPU_REQUEST)
        self.nz_mem = nz_mem if nz_mem >= 0 else (mem or DEFAULT_MEMORY_REQUEST)
        self.flags = flags
        self.ext = ext if ext is not None else _EMPTY
        self.uid = uid
        self.namespace = namespace
        self.name = name
        self.num_id = num_id
        self.labels = labels
        self.gpu = gpu
        self.scheduler_name = scheduler_name
        self.node_name = node_name
        self.cpu_m = cpu_m
        self.mem = mem
        self.priority = priority
        self.node_selector = node_selector if node_selector is not None else {}
        self.required_terms = required_terms if required_terms is not None else []
        self.preferred_terms = preferred_terms if preferred_terms is not None else []
        self.tolerations = tolerations if tolerations is not None else []
        self.annotations = annotations if annotations is not None else {}
        self.host_ports = host_ports if host_ports is not None else []
        self.attempts = 0
        self.initial_attempt = 0.0
        self.enqueued = 0.0
        self.native_req: Any = None          # engine-specific PodReq cache
        self.native_owner: Any = None
        self.applies_memo: Optional[dict] = None   # plugin id → applies (one cycle; Framework.memo_cycle)
        self.assigned_cards: Optional[list] = None
        self._creation: Optional[float] = None

    @property
    def obj(self) -> dict:
        o = self._obj
        if o is None:
            src = self._src
            o = self._obj = json.loads(src.raw()) if src is not None else {}
            self._src = None
        return o

    @obj.setter
    def obj(self, value: dict) -> None:
        self._obj, self._src = value, None

    def set_source(self, ev) -> None:
        """Point the lazy ``obj`` at a newer native watch event of the same pod."""
        self._obj, self._src = None, ev

    @property
    def key(self) -> str:
        return f"{self.namespace}/{self.name}"

    @property
    def creation(self) -> float:
        """creationTimestamp (parsed lazily: the hot path never needs it)."""
        if self._creation is None:
            self._creation = parse_rfc3339((self.obj.get("metadata") or {}).get("creationTimestamp")) or time.time()
        return self._creation

    @classmethod
    def from_native(cls, ev) -> "PodInfo":
        """Build from a native transport ``PodEvent`` (C++ projection of the same fields
        ``from_obj`` reads); pods the projection does not cover go through ``from_obj``."""
        a = ev.info_args()
        if a is None:
            pi = cls.from_obj(json.loads(ev.raw()))
            return pi
        (uid, ns, name, labels, ann, sched, node, cpu, mem, nzc, nzm, prio, nsel, req, pref, tols, ports,
         flags, _creation, ext, images, containers, owner, avoid, spread, deleting, pod_aff) = a
        pi = cls(None, uid, ns, name, pod_num_id(uid), labels, parse_gpu_request(labels), sched, node, cpu, mem,
                 prio, nsel, req, pref, tols, ann, ports, flags, ext, nzc, nzm, images, containers, owner, avoid,
                 spread, deleting, pod_aff)
        pi._src = ev
        return pi

    def __repr__(self) -> str:
        return f"PodInfo({self.key}, gpu={self.gpu}, node={self.node_name!r})"

    @classmethod
    def from_obj(cls, obj: dict) -> "PodInfo":
        meta = obj.get("metadata") or _EMPTY
        spec = obj.get("spec") or _EMPTY
        labels = meta.get("labels") or {}
        uid = meta.get("uid") or pod_key(obj)
        containers = spec.get("containers") or ()
        # one pass over the containers: requests, extended requests, host ports, images
        cpu = mem = nzc = nzm = 0
        ext = ports = None
        images = []
        for c in containers:
            img = c.get("image")
            if img:
                images.append(normalize_image(img))
            res = c.get("resources")
            r = res.get("requests") if res else None
            if r:
                if "cpu" in r:
                    v = cpu_millis(r["cpu"])
                    cpu += v
                    nzc += v
                else:
                    nzc += DEFAULT_MILLI_CPU_REQUEST
                if "memory" in r:
                    v = bytes_of(r["memory"])
                    mem += v
                    nzm += v
                else:
                    nzm += DEFAULT_MEMORY_REQUEST
                if len(r) > ("cpu" in r) + ("memory" in r):
                    ext = ext if ext is not None else {}
                    for k, q in r.items():
                        if k not in _BASIC:
                            ext[k] = ext.get(k, 0) + quantity_int(q)
            else:
                nzc += DEFAULT_MILLI_CPU_REQUEST
                nzm += DEFAULT_MEMORY_REQUEST
            cp = c.get("ports")
            if cp:
                for p in cp:
                    if p.get("hostPort"):
                        (ports := ports or []).append((p.get("hostPort"), p.get("protocol", "TCP"),
                                                       p.get("hostIP", "")))
        req = pref = tols = ns = spread = pod_aff = None
        if not _RARE_SPEC.isdisjoint(spec):
            if "initContainers" in spec or "overhead" in spec:
                cpu, mem, nzc, nzm = _requests(spec)
                ext = ext_requests(spec) if _has_ext(spec) else None
            aff = spec.get("affinity")
            if aff:
                na = aff.get("nodeAffinity") or _EMPTY
                req = _terms((na.get("requiredDuringSchedulingIgnoredDuringExecution") or _EMPTY)
                             .get("nodeSelectorTerms"))
                pref = [(int(p.get("weight", 0)), _terms([p.get("preference") or {}])[0])
                        for p in na.get("preferredDuringSchedulingIgnoredDuringExecution") or ()]
                if aff.get("podAffinity") or aff.get("podAntiAffinity"):
                    pod_aff = _pod_aff(aff)
            tols = spec.get("tolerations")
            if tols:
                tols = [(t.get("key") or None, str(t.get("value", "") or ""), t.get("operator", "Equal") or "Equal",
                         t.get("effect", "") or "") for t in tols]
            ns = spec.get("nodeSelector")
            tsc = spec.get("topologySpreadConstraints")
            if tsc:
                from .selectors import LabelSelector
                spread = [(c.get("topologyKey", ""), int(c.get("maxSkew", 1)),
                           c.get("whenUnsatisfiable", "DoNotSchedule"),
                           None if c.get("labelSelector") is None else LabelSelector(c.get("labelSelector")).native())
                          for c in tsc]
        if ext:
            ext = {k: v for k, v in ext.items() if v} or None
        owner = avoid = None
        refs = meta.get("ownerReferences")
        if refs:
            for r in refs:
                if not r.get("controller"):
                    continue
                if owner is None:
                    owner = (r.get("apiVersion", "") or "", r.get("kind", "") or "", r.get("name", "") or "",
                             r.get("uid", "") or "")
                if avoid is None and r.get("kind") in ("ReplicationController", "ReplicaSet"):
                    avoid = (r.get("kind"), r.get("uid", "") or "")
        ann = meta.get("annotations")
        return cls(obj, uid, meta.get("namespace", "default"), meta.get("name", ""), pod_num_id(uid), labels,
                   parse_gpu_request(labels), spec.get("schedulerName") or "default-scheduler",
                   spec.get("nodeName") or "", cpu, mem, int(spec.get("priority") or 0),
                   dict(ns) if ns else None, req, pref, tols or None, dict(ann) if ann else None, ports,
                   pod_flags(meta, spec, ports, ext), ext, nzc, nzm, images, len(containers), owner, avoid, spread,
                   bool(meta.get("deletionTimestamp")), pod_aff)


# spec fields a plain pod does not carry (from_obj parses them only when one is present)
_RARE_SPEC = frozenset(("initContainers", "overhead", "affinity", "tolerations", "nodeSelector",
                        "topologySpreadConstraints"))
_EMPTY: dict = {}
_NOLIST: list = []


def _pod_aff(aff: dict) -> tuple:
    """spec.affinity's pod (anti-)affinity terms as the engine takes them (plugins/spread_affinity.py
    ``_terms``: a required term has weight 1, a preferred one its weight and podAffinityTerm)."""
    from .selectors import LabelSelector

    def term(t, w):
        t = t or {}
        sel = t.get("labelSelector")
        return (t.get("topologyKey", "") or "", tuple(t.get("namespaces") or ()) or None,
                None if sel is None else LabelSelector(sel).native(), w)
    out = []
    for kind in ("podAffinity", "podAntiAffinity"):
        k = aff.get(kind) or {}
        out.append([term(t, 1) for t in k.get("requiredDuringSchedulingIgnoredDuringExecution") or ()])
    for kind in ("podAffinity", "podAntiAffinity"):
        k = aff.get(kind) or {}
        out.append([term(w.get("podAffinityTerm"), int(w.get("weight", 1)))
                    for w in k.get("preferredDuringSchedulingIgnoredDuringExecution") or ()])
    return tuple(out)


@dataclass
class NodeInfo:
    """k8s facts of a node (the GPU side lives in the Scv / native engine)."""
    name: str
    obj: dict
    labels: dict
    taints: list
    unschedulable: bool
    cpu_m: int
    mem: int
    pods: int
    images: dict = field(default_factory=dict)       # normalized image name → size bytes
    ext_alloc: dict = field(default_factory=dict)    # allocatable beyond cpu/memory/pods
    avoid: Optional[str] = None                      # preferAvoidPods annotation (raw JSON)

    @classmethod
    def from_obj(cls, obj: dict) -> "NodeInfo":
        meta = obj.get("metadata") or {}
        spec = obj.get("spec") or {}
        alloc = (obj.get("status") or {}).get("allocatable") or {}
        taints = [(t.get("key", ""), str(t.get("value", "") or ""), t.get("effect", "NoSchedule"))
                  for t in spec.get("taints") or []]
        return cls(name=meta.get("name", ""), obj=obj, labels=dict(meta.get("labels") or {}), taints=taints,
                   unschedulable=bool(spec.get("unschedulable", False)),
                   cpu_m=cpu_millis(alloc.get("cpu", "0")), mem=bytes_of(alloc.get("memory", "0")),
                   pods=int(alloc.get("pods", 110)), images=_node_images(obj),
                   ext_alloc={k: quantity_int(v) for k, v in alloc.items() if k not in ("cpu", "memory", "pods")},
                   avoid=(meta.get("annotations") or _EMPTY).get(ANNOTATION_PREFER_AVOID_PODS))


ANNOTATION_PREFER_AVOID_PODS = "scheduler.alpha.kubernetes.io/preferAvoidPods"


def normalize_image(name: str) -> str:
    """Upstream ``normalizedImageName``: an image without a tag or digest means ``:latest``."""
    if name.rfind(":") <= name.rfind("/") and "@" not in name:
        return name + ":latest"
    return name


def _node_images(obj: dict) -> dict:
    imgs = (obj.get("status") or _EMPTY).get("images")
    if not imgs:
        return {}
    out = {}
    for im in imgs:
        size = int(im.get("sizeBytes") or 0)
        for n in im.get("names") or ():
            out[normalize_image(n)] = size
    return out
