"""What kube-controller-manager's PV controller and an external provisioner do after the
scheduler's VolumeBinding PreBind, for the in-process fake apiserver:

* a PV whose ``spec.claimRef`` names an unbound PVC → the PVC gets ``spec.volumeName``
  and both become ``Bound``;
* a PVC annotated ``volume.kubernetes.io/selected-node`` by the scheduler → a PV of the
  requested size is provisioned with node affinity to that node's hostname, then bound.

Without it (a real cluster) this file is unused; with it, volume scheduling can be tested
end to end, including PreBind's wait for the binding to complete.
"""
from __future__ import annotations

import asyncio
from typing import Optional

from ..plugins.volumes import ANN_SELECTED_NODE
from .server import FakeApiServer


class FakePVController:
    def __init__(self, server: FakeApiServer, interval: float = 0.005) -> None:
        self.server = server
        self.interval = interval
        self.provisioned = 0
        self.bound = 0
        self._task: Optional[asyncio.Task] = None

    def _bind(self, pvc: dict, pv: dict) -> None:
        srv = self.server
        m = pvc["metadata"]
        ref = {"kind": "PersistentVolumeClaim", "apiVersion": "v1", "namespace": m.get("namespace", "default"),
               "name": m["name"], "uid": m.get("uid", "")}
        srv.patch("persistentvolumes", pv["metadata"]["name"], {"spec": {"claimRef": ref}, "status": {"phase": "Bound"}})
        srv.patch("persistentvolumeclaims", m["name"], {"spec": {"volumeName": pv["metadata"]["name"]},
                                                        "status": {"phase": "Bound"}},
                  namespace=m.get("namespace", "default"))
        self.bound += 1

    def reconcile(self) -> None:
        srv = self.server
        pvcs, _ = srv.list("persistentvolumeclaims")
        by_key = {f"{p['metadata'].get('namespace', 'default')}/{p['metadata']['name']}": p for p in pvcs}
        pvs, _ = srv.list("persistentvolumes")
        for pv in pvs:
            ref = (pv.get("spec") or {}).get("claimRef")
            if not ref or (pv.get("status") or {}).get("phase") == "Bound":
                continue
            pvc = by_key.get(f"{ref.get('namespace', 'default')}/{ref.get('name')}")
            if pvc is not None and not (pvc.get("spec") or {}).get("volumeName"):
                self._bind(pvc, pv)
        for key, pvc in by_key.items():
            ann = (pvc.get("metadata") or {}).get("annotations") or {}
            node = ann.get(ANN_SELECTED_NODE)
            if not node or (pvc.get("spec") or {}).get("volumeName"):
                continue
            spec = pvc.get("spec") or {}
            try:
                host = (srv.get("nodes", node).get("metadata") or {}).get("labels", {}).get("kubernetes.io/hostname",
                                                                                             node)
            except Exception:  # noqa: BLE001 - node gone: leave the claim pending
                continue
            pv = srv.create("persistentvolumes", {
                "metadata": {"name": f"pvc-{pvc['metadata'].get('uid', key.replace('/', '-'))}"},
                "spec": {"capacity": {"storage": ((spec.get("resources") or {}).get("requests") or {}).get("storage",
                                                                                                          "1Gi")},
                         "accessModes": spec.get("accessModes") or ["ReadWriteOnce"],
                         "storageClassName": spec.get("storageClassName", ""),
                         "nodeAffinity": {"required": {"nodeSelectorTerms": [{"matchExpressions": [
                             {"key": "kubernetes.io/hostname", "operator": "In", "values": [host]}]}]}}},
                "status": {"phase": "Available"}})
            self.provisioned += 1
            self._bind(pvc, pv)

    async def run(self) -> None:
        while True:
            self.reconcile()
            await asyncio.sleep(self.interval)

    def start(self) -> None:
        self._task = asyncio.get_event_loop().create_task(self.run())

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            await asyncio.gather(self._task, return_exceptions=True)
