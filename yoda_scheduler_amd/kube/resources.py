"""REST paths of the resources the scheduler and sniffer touch (RBAC
``deploy/yoda-scheduler.yaml:71-216``)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional


@dataclass(frozen=True)
class Resource:
    name: str
    group: str
    version: str
    kind: str
    namespaced: bool

    @property
    def api_version(self) -> str:
        return self.version if not self.group else f"{self.group}/{self.version}"

    def path(self, namespace: Optional[str] = None, name: Optional[str] = None, sub: Optional[str] = None) -> str:
        base = "/api/" + self.version if not self.group else f"/apis/{self.group}/{self.version}"
        p = base
        if self.namespaced and namespace:
            p += f"/namespaces/{namespace}"
        p += f"/{self.name}"
        if name:
            p += f"/{name}"
        if sub:
            p += f"/{sub}"
        return p


RESOURCES = {
    "pods": Resource("pods", "", "v1", "Pod", True),
    "nodes": Resource("nodes", "", "v1", "Node", False),
    "events": Resource("events", "", "v1", "Event", True),
    # upstream v1.20's scheduler records through the events.k8s.io/v1 API (EventBroadcasterAdapter)
    "events.k8s.io": Resource("events", "events.k8s.io", "v1", "Event", True),
    "leases": Resource("leases", "coordination.k8s.io", "v1", "Lease", True),
    "scvs": Resource("scvs", "core.run-linux.com", "v1", "Scv", False),
    "configmaps": Resource("configmaps", "", "v1", "ConfigMap", True),
    "endpoints": Resource("endpoints", "", "v1", "Endpoints", True),      # legacy leader-election lock
    # volume plugins (VolumeBinding / VolumeZone / NodeVolumeLimits)
    "persistentvolumeclaims": Resource("persistentvolumeclaims", "", "v1", "PersistentVolumeClaim", True),
    "persistentvolumes": Resource("persistentvolumes", "", "v1", "PersistentVolume", False),
    "storageclasses": Resource("storageclasses", "storage.k8s.io", "v1", "StorageClass", False),
    "csinodes": Resource("csinodes", "storage.k8s.io", "v1", "CSINode", False),
    # DefaultPreemption honours PodDisruptionBudgets
    "poddisruptionbudgets": Resource("poddisruptionbudgets", "policy", "v1", "PodDisruptionBudget", True),
    # SelectorSpread / ServiceAffinity (DefaultSelector: services + the pod's controller)
    "services": Resource("services", "", "v1", "Service", True),
    "replicationcontrollers": Resource("replicationcontrollers", "", "v1", "ReplicationController", True),
    "replicasets": Resource("replicasets", "apps", "v1", "ReplicaSet", True),
    "statefulsets": Resource("statefulsets", "apps", "v1", "StatefulSet", True),
}


BY_PATH = {(r.group, r.name): key for key, r in RESOURCES.items()}


def resource(name: str) -> Resource:
    try:
        return RESOURCES[name]
    except KeyError:
        raise ValueError(f"unknown resource {name!r}") from None


def obj_key(res: Resource, obj: dict) -> str:
    m = obj.get("metadata") or {}
    if res.namespaced:
        return f"{m.get('namespace') or 'default'}/{m.get('name', '')}"
    return m.get("name", "")
