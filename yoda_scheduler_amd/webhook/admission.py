"""``admission.k8s.io/v1`` AdmissionReview handling for pods using the scv label API.

Validation (``/validate``): every ``scv/*`` and ``scv.amd.com/*`` request label must be a
plain non-negative decimal integer (Go ``Atoi`` syntax, no sign); ``scv/number`` must be
1..``maxGpusPerPod``, ``scv/memory`` at most ``maxMemoryMB`` per GPU (default: one
MI355X's HBM), ``scv/priority`` may be negative. Unknown ``scv/*`` keys are admitted with
a warning (typos such as ``scv/memroy`` would otherwise be ignored silently).

Mutation (``/mutate``, optional): pods that carry scv labels but left
``spec.schedulerName`` at the default are pointed at ``schedulerName`` (the yoda profile),
so users cannot forget the profile name (quirk Q6 made that easy in the reference).
Their containers also get ``ROCR_VISIBLE_DEVICES`` from the downward API
(``metadata.annotations['scv.amd.com/visible-devices']``): the Binding copies the
scheduler's GPU assignment onto the pod before any container starts, so the process sees
exactly the GPUs whose HBM the scheduler reserved (the reference only picked a node, Q10).
The value names each GPU by its ROCr UUID (``GPU-…``, from amd-smi's enumeration info),
so the pinning is right whatever order HIP/KFD enumerate devices in and with CPX/DPX
partitions; ``HIP_VISIBLE_DEVICES`` is *not* set: it indexes the devices ROCr already
filtered, so the same list in both variables would hide GPUs.
Containers that set either variable themselves, pods that request ``amd.com/gpu`` through
the device plugin, and pods annotated ``scv.amd.com/inject-visible-devices: "false"`` are
left alone.
"""
from __future__ import annotations

import base64
import json
from dataclasses import dataclass
from typing import Optional

from ..models.labels import LABEL_CLOCK, LABEL_CLOCK_MIN, LABEL_MEMORY, LABEL_NUMBER, LABEL_PRIORITY

MI355X_HBM_MB = 288 * 1024
_UNSIGNED = (LABEL_NUMBER, LABEL_MEMORY, LABEL_CLOCK, LABEL_CLOCK_MIN)
KNOWN = set(_UNSIGNED) | {LABEL_PRIORITY, "scv.amd.com/gang"}
GANG_VALUES = ("xgmi", "any", "numa")


ANNOTATION_VISIBLE = "scv.amd.com/visible-devices"
ANNOTATION_NO_INJECT = "scv.amd.com/inject-visible-devices"
VISIBLE_ENV = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
INJECT_ENV = "ROCR_VISIBLE_DEVICES"


@dataclass
class AdmissionPolicy:
    max_gpus_per_pod: int = 64            # 8 GPUs × CPX partitions
    max_memory_mb: int = MI355X_HBM_MB
    scheduler_name: str = "yoda-scheduler"
    mutate_scheduler_name: bool = True
    inject_visible_devices: bool = True
    yoda_profiles: tuple = ("yoda-scheduler", "yoda-scheduler2")   # deploy/yoda-scheduler.yaml


def _is_decimal(v: str, signed: bool) -> bool:
    body = v[1:] if signed and v[:1] in ("-", "+") else v
    return bool(body) and body.isascii() and body.isdigit() and len(body) <= 19


def validate_labels(labels: Optional[dict], policy: AdmissionPolicy = AdmissionPolicy()) -> tuple[list, list]:
    """Returns (errors, warnings) for a pod's labels."""
    errors, warnings = [], []
    labels = labels or {}
    for k, v in sorted(labels.items()):
        if not (k.startswith("scv/") or k.startswith("scv.amd.com/")):
            continue
        if k not in KNOWN:
            warnings.append(f"unknown scv label {k!r} is ignored by the scheduler")
            continue
        v = str(v)
        if k == "scv.amd.com/gang":
            if v not in GANG_VALUES:
                errors.append(f"label {k}={v!r}: must be one of {', '.join(GANG_VALUES)}")
            continue
        if not _is_decimal(v, signed=(k == LABEL_PRIORITY)):
            errors.append(f"label {k}={v!r}: must be a {'' if k == LABEL_PRIORITY else 'non-negative '}"
                          f"decimal integer (the scheduler would read it as 0)")
            continue
        n = int(v)
        if k == LABEL_NUMBER and not 1 <= n <= policy.max_gpus_per_pod:
            errors.append(f"label {k}={v!r}: must be between 1 and {policy.max_gpus_per_pod}")
        elif k == LABEL_MEMORY and n > policy.max_memory_mb:
            errors.append(f"label {k}={v!r}: exceeds the {policy.max_memory_mb} MB of HBM of one GPU")
        elif k == LABEL_PRIORITY and not -(1 << 31) <= n < (1 << 31):
            errors.append(f"label {k}={v!r}: out of the int32 range")
    return errors, warnings


def _uses_scv(labels: dict) -> bool:
    return any(k in KNOWN for k in labels)


def _requests_device_plugin_gpus(c: dict) -> bool:
    res = c.get("resources") or {}
    return any(k.startswith("amd.com/") for part in ("limits", "requests") for k in (res.get(part) or {}))


def _visible_devices_ops(pod: dict) -> list:
    spec = pod.get("spec") or {}
    ann = (pod.get("metadata") or {}).get("annotations") or {}
    if str(ann.get(ANNOTATION_NO_INJECT, "")).lower() == "false":
        return []
    ops = []
    for key in ("initContainers", "containers"):
        cs = spec.get(key) or []
        if any(_requests_device_plugin_gpus(c) for c in cs):
            return []          # the device plugin owns GPU visibility for this pod
        for i, c in enumerate(cs):
            env = c.get("env")
            names = {e.get("name") for e in env or ()}
            if names & set(VISIBLE_ENV):
                continue
            vals = [{"name": INJECT_ENV,
                     "valueFrom": {"fieldRef": {"fieldPath": f"metadata.annotations['{ANNOTATION_VISIBLE}']"}}}]
            if env is None:
                ops.append({"op": "add", "path": f"/spec/{key}/{i}/env", "value": vals})
            else:
                ops.extend({"op": "add", "path": f"/spec/{key}/{i}/env/-", "value": v} for v in vals)
    return ops


def _patch(pod: dict, policy: AdmissionPolicy) -> list:
    spec = pod.get("spec") or {}
    labels = (pod.get("metadata") or {}).get("labels") or {}
    if not _uses_scv(labels):
        return []
    ops = []
    target = spec.get("schedulerName")
    if policy.mutate_scheduler_name and target in (None, "", "default-scheduler"):
        ops.append({"op": "replace" if "schedulerName" in spec else "add", "path": "/spec/schedulerName",
                    "value": policy.scheduler_name})
        target = policy.scheduler_name
    # only pods the yoda profile schedules get an assignment annotation to read
    if policy.inject_visible_devices and (target == policy.scheduler_name or target in policy.yoda_profiles):
        ops.extend(_visible_devices_ops(pod))
    return ops


def review(body: dict, mutate: bool, policy: AdmissionPolicy = AdmissionPolicy()) -> dict:
    """One AdmissionReview request → AdmissionReview response."""
    req = body.get("request") or {}
    uid = req.get("uid", "")
    resp: dict = {"uid": uid, "allowed": True}
    kind = (req.get("kind") or {}).get("kind", "Pod")
    pod = req.get("object") or {}
    if kind == "Pod" and req.get("operation", "CREATE") in ("CREATE", "UPDATE"):
        errors, warnings = validate_labels((pod.get("metadata") or {}).get("labels"), policy)
        if warnings:
            resp["warnings"] = warnings
        if errors and not mutate:
            resp["allowed"] = False
            resp["status"] = {"code": 422, "reason": "Invalid", "message": "; ".join(errors)}
        if mutate and req.get("operation", "CREATE") == "CREATE":
            ops = _patch(pod, policy)
            if ops:
                resp["patchType"] = "JSONPatch"
                resp["patch"] = base64.b64encode(json.dumps(ops).encode()).decode()
    return {"apiVersion": body.get("apiVersion", "admission.k8s.io/v1"), "kind": "AdmissionReview",
            "response": resp}


def apply_add_ops(doc: dict, ops: list) -> dict:
    """Apply the RFC 6902 ``add``/``replace`` operations this webhook emits (what the
    apiserver does with the response patch) — for tests and the local demo path."""
    import copy
    doc = copy.deepcopy(doc)
    for o in ops:
        parts = o["path"].strip("/").split("/")
        tgt = doc
        for k in parts[:-1]:
            tgt = tgt[int(k)] if isinstance(tgt, list) else tgt.setdefault(k, {})
        last = parts[-1]
        if isinstance(tgt, list):
            if last == "-":
                tgt.append(o["value"])
            elif o["op"] == "replace":
                tgt[int(last)] = o["value"]
            else:
                tgt.insert(int(last), o["value"])
        else:
            tgt[last] = o["value"]
    return doc
