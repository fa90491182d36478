"""Node-side pod executor ("kubelet-lite") that turns a binding into a real GPU workload —
the last hop of SURVEY §7.2's minimum end-to-end slice: scheduler decision →
``scv.amd.com/visible-devices`` annotation (ROCr UUIDs) → a ROCm process pinned with
``ROCR_VISIBLE_DEVICES`` that
allocates the pod's ``scv/memory`` MB of HBM on those GPUs → the next amd-smi sample shows
the HBM drop, closing the telemetry loop the reference never closes (its burst pods are
invisible to the sniffer).

Used for validation and demos against the fake apiserver; in a real cluster the kubelet +
a device plugin reading the annotation play this role.
"""
from __future__ import annotations

import asyncio
import os
import subprocess
import sys
from dataclasses import dataclass, field
from typing import Optional

from ..models.labels import ANNOTATION_GPUS, ANNOTATION_VISIBLE, LABEL_MEMORY

HOLD_SCRIPT = r"""
import os, sys, time, torch
mb = int(sys.argv[1]); secs = float(sys.argv[2])
bufs = [torch.empty(mb * (1 << 20), dtype=torch.uint8, device=f"cuda:{i}") for i in range(torch.cuda.device_count())]
for b in bufs:
    b.fill_(1)
torch.cuda.synchronize()
buses = [torch.cuda.get_device_properties(i).pci_bus_id for i in range(torch.cuda.device_count())]
print("allocated", mb, "MB on", len(bufs), "GPU(s) ROCR_VISIBLE_DEVICES=", os.environ.get("ROCR_VISIBLE_DEVICES"),
      "pci_bus_ids=", ",".join(str(b) for b in buses), flush=True)
time.sleep(secs)
"""


def _field(pod: dict, path: str) -> str:
    """Downward-API ``fieldRef.fieldPath``: ``metadata.annotations['k']`` /
    ``metadata.labels['k']`` and plain dotted paths (``metadata.name``, ``spec.nodeName``)."""
    for kind in ("annotations", "labels"):
        pre = f"metadata.{kind}['"
        if path.startswith(pre) and path.endswith("']"):
            return str(((pod.get("metadata") or {}).get(kind) or {}).get(path[len(pre):-2], ""))
    v = pod
    for k in path.split("."):
        v = v.get(k) if isinstance(v, dict) else None
        if v is None:
            return ""
    return str(v)


def resolve_env(pod: dict, container: dict) -> dict:
    """A container's environment as the kubelet builds it (``value`` and downward-API
    ``fieldRef`` entries; later entries win)."""
    out = {}
    for e in container.get("env") or ():
        name = e.get("name")
        if not name:
            continue
        if "value" in e:
            out[name] = str(e["value"])
        else:
            ref = (e.get("valueFrom") or {}).get("fieldRef") or {}
            if ref.get("fieldPath"):
                out[name] = _field(pod, ref["fieldPath"])
    return out


@dataclass
class Running:
    key: str
    gpus: list[int]
    mb: int
    proc: subprocess.Popen
    log: list[str] = field(default_factory=list)


class PodExecutor:
    def __init__(self, client, node: str, hold_seconds: float = 30.0) -> None:
        self.client = client
        self.node = node
        self.hold_seconds = hold_seconds
        self.running: dict[str, Running] = {}
        self.env_log: dict[str, dict] = {}

    def launch(self, pod: dict) -> Optional[Running]:
        meta = pod.get("metadata") or {}
        key = f"{meta.get('namespace', 'default')}/{meta.get('name')}"
        if key in self.running or (pod.get("spec") or {}).get("nodeName") != self.node:
            return None
        ann = meta.get("annotations") or {}
        gpus = [int(x) for x in (ann.get(ANNOTATION_GPUS) or "").split(",") if x.strip()]
        mb = int((meta.get("labels") or {}).get(LABEL_MEMORY, "0") or 0)
        containers = (pod.get("spec") or {}).get("containers") or [{}]
        spec_env = resolve_env(pod, containers[0])
        env = dict(os.environ)
        for k in ("CUDA_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
            env.pop(k, None)
        if "HIP_VISIBLE_DEVICES" in spec_env or "ROCR_VISIBLE_DEVICES" in spec_env:
            # pinned by the pod spec (yoda-webhook's downward-API injection)
            env.update(spec_env)
        else:
            vis = ann.get(ANNOTATION_VISIBLE) or ",".join(map(str, gpus))
            env.update(spec_env, ROCR_VISIBLE_DEVICES=vis)
        self.env_log[key] = {k: env.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES")}
        proc = subprocess.Popen([sys.executable, "-c", HOLD_SCRIPT, str(mb), str(self.hold_seconds)], env=env,
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        r = Running(key, gpus, mb, proc)
        self.running[key] = r
        return r

    async def wait_allocated(self, r: Running, timeout: float = 180.0) -> bool:
        """Wait for the workload's 'allocated' line (first torch import can be slow)."""
        loop = asyncio.get_event_loop()

        def read():
            for line in r.proc.stdout:   # type: ignore[union-attr]
                r.log.append(line.rstrip())
                if line.startswith("allocated"):
                    return True
            return False

        try:
            return await asyncio.wait_for(loop.run_in_executor(None, read), timeout)
        except asyncio.TimeoutError:
            return False

    def stop_all(self) -> None:
        for r in self.running.values():
            if r.proc.poll() is None:
                r.proc.terminate()
                try:
                    r.proc.wait(10)
                except subprocess.TimeoutExpired:
                    r.proc.kill()
        self.running.clear()
