"""``admission.k8s.io/v1`` AdmissionReview handling for pods using the scv label API.

Validation (``/validate``): every ``scv/*`` and ``scv.amd.com/*`` request label must be a
plain non-negative decimal integer (Go ``Atoi`` syntax, no sign); ``scv/number`` must be
1..``maxGpusPerPod``, ``scv/memory`` at most ``maxMemoryMB`` per GPU (default: one
MI355X's HBM), ``scv/priority`` may be negative. Unknown ``scv/*`` keys are admitted with
a warning (typos such as ``scv/memroy`` would otherwise be ignored silently).

Mutation (``/mutate``, optional): pods that carry scv labels but left
``spec.schedulerName`` at the default are pointed at ``schedulerName`` (the yoda profile),
so users cannot forget the profile name (quirk Q6 made that easy in the reference).
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


@dataclass
class AdmissionPolicy:
    max_gpus_per_pod: int = 64            # 8 GPUs × CPX partitions
    max_memory_mb: int = MI355X_HBM_MB
    scheduler_name: str = "yoda-scheduler"
    mutate_scheduler_name: bool = True


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


def _patch(pod: dict, policy: AdmissionPolicy) -> list:
    spec = pod.get("spec") or {}
    labels = (pod.get("metadata") or {}).get("labels") or {}
    if not policy.mutate_scheduler_name or not _uses_scv(labels):
        return []
    if spec.get("schedulerName") not in (None, "", "default-scheduler"):
        return []
    op = "replace" if "schedulerName" in spec else "add"
    return [{"op": op, "path": "/spec/schedulerName", "value": policy.scheduler_name}]


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
