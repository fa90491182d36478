"""Parsed views of v1.Pod / v1.Node objects (dict-shaped, as the apiserver returns them).

A ``PodInfo`` parses everything the scheduling cycle needs exactly once per pod
(labels → ``GpuRequest``, resource requests, selectors, tolerations) so the per-node
loops — native or Python — never touch the raw JSON again.
"""
from __future__ import annotations

import itertools
import time
from dataclasses import dataclass, field
from typing import Any

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


def _requests(spec: dict) -> tuple[int, int]:
    cpu = mem = 0
    for c in spec.get("containers") or []:
        r = ((c.get("resources") or {}).get("requests")) or {}
        cpu += cpu_millis(r.get("cpu")) if "cpu" in r else 0
        mem += bytes_of(r.get("memory")) if "memory" in r else 0
    for c in spec.get("initContainers") or []:
        r = ((c.get("resources") or {}).get("requests")) or {}
        cpu = max(cpu, cpu_millis(r.get("cpu")) if "cpu" in r else 0)
        mem = max(mem, bytes_of(r.get("memory")) if "memory" in r else 0)
    ov = spec.get("overhead") or {}
    cpu += cpu_millis(ov["cpu"]) if "cpu" in ov else 0
    mem += bytes_of(ov["memory"]) if "memory" in ov else 0
    return cpu, mem


def _terms(terms: list | None) -> list[list[tuple[str, str, list[str]]]]:
    out = []
    for t in terms or []:
        reqs = [(e.get("key", ""), e.get("operator", "In"), [str(v) for v in e.get("values") or []])
                for e in (t.get("matchExpressions") or [])]
        # matchFields metadata.name → expressed on the hostname label the fake nodes carry
        for f in t.get("matchFields") or []:
            if f.get("key") == "metadata.name":
                reqs.append(("kubernetes.io/hostname", f.get("operator", "In"),
                             [str(v) for v in f.get("values") or []]))
        out.append(reqs)
    return out


@dataclass
class PodInfo:
    obj: dict
    uid: str
    namespace: str
    name: str
    num_id: int
    labels: dict
    gpu: GpuRequest
    scheduler_name: str
    node_name: str
    cpu_m: int
    mem: int
    priority: int
    node_selector: dict
    required_terms: list
    preferred_terms: list
    tolerations: list
    creation: float
    annotations: dict
    host_ports: list = field(default_factory=list)
    # cycle bookkeeping (queue)
    attempts: int = 0
    initial_attempt: float = 0.0
    enqueued: float = 0.0
    native_req: Any = None          # engine-specific PodReq cache
    native_owner: Any = None

    @property
    def key(self) -> str:
        return f"{self.namespace}/{self.name}"

    @classmethod
    def from_obj(cls, obj: dict) -> "PodInfo":
        meta = obj.get("metadata") or {}
        spec = obj.get("spec") or {}
        labels = meta.get("labels") or {}
        cpu, mem = _requests(spec)
        aff = (spec.get("affinity") or {}).get("nodeAffinity") or {}
        req = (aff.get("requiredDuringSchedulingIgnoredDuringExecution") or {}).get("nodeSelectorTerms")
        pref = [(int(p.get("weight", 0)), _terms([p.get("preference") or {}])[0])
                for p in aff.get("preferredDuringSchedulingIgnoredDuringExecution") or []]
        tols = [(t.get("key") or None, str(t.get("value", "") or ""), t.get("operator", "Equal") or "Equal",
                 t.get("effect", "") or "") for t in spec.get("tolerations") or []]
        ports = [(p.get("hostPort"), p.get("protocol", "TCP"), p.get("hostIP", ""))
                 for c in spec.get("containers") or [] for p in c.get("ports") or [] if p.get("hostPort")]
        created = parse_rfc3339(meta.get("creationTimestamp")) or time.time()
        return cls(
            obj=obj, uid=meta.get("uid") or pod_key(obj), namespace=meta.get("namespace", "default"),
            name=meta.get("name", ""), num_id=pod_num_id(meta.get("uid") or pod_key(obj)), labels=labels, gpu=parse_gpu_request(labels),
            scheduler_name=spec.get("schedulerName") or "default-scheduler",
            node_name=spec.get("nodeName") or "", cpu_m=cpu, mem=mem,
            priority=int(spec.get("priority") or 0),
            node_selector=dict(spec.get("nodeSelector") or {}),
            required_terms=_terms(req), preferred_terms=pref, tolerations=tols, creation=created,
            annotations=dict(meta.get("annotations") or {}), host_ports=ports,
        )


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
                   pods=int(alloc.get("pods", 110)))
