"""The ``scv/*`` pod-label API (drop-in contract).

Label keys are the ones the reference reads:
  * ``scv/number``   GPU count             (``pkg/yoda/filter/filter.go:12``)
  * ``scv/memory``   free MB per GPU       (``filter.go:19``, ``score/algorithm.go:77``)
  * ``scv/clock``    exact card clock MHz  (``filter.go:36``)
  * ``scv/priority`` queue order, higher first (``pkg/yoda/sort/sort.go:13``)

Values are parsed with Go ``Atoi`` semantics (invalid → 0, negatives wrap, Q5).
MI355X-native additions are namespaced ``scv.amd.com/*`` so the reference keys keep
their exact meaning.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Mapping

from ..utils.gonum import atoi_or_zero, str_to_uint

LABEL_NUMBER = "scv/number"
LABEL_MEMORY = "scv/memory"
LABEL_CLOCK = "scv/clock"
LABEL_PRIORITY = "scv/priority"

# additive AMD extensions (not in the reference)
LABEL_CLOCK_MIN = "scv.amd.com/clock-min"        # card clock >= value (MHz)
LABEL_GANG_POLICY = "scv.amd.com/gang"           # "xgmi" (default) | "any" | "numa"
ANNOTATION_GPUS = "scv.amd.com/gpus"             # assigned GPU indices (amd-smi, BDF order), e.g. "0,3"
# what the pod's ROCr runtime must see, per assigned GPU: the ROCr/HIP UUID ("GPU-…") when
# the sniffer reported it, else the HIP ordinal, else the amd-smi index — always present on
# a yoda binding, so a downward-API env var built from it is never empty
ANNOTATION_VISIBLE = "scv.amd.com/visible-devices"
ANNOTATION_GPU_UUIDS = "scv.amd.com/gpu-uuids"   # amd-smi device UUIDs of the assigned GPUs
ANNOTATION_RESERVED = "scv.amd.com/reserved-mb"  # HBM MB reserved per assigned GPU
ANNOTATION_NODE = "scv.amd.com/node"


@dataclass(frozen=True)
class GpuRequest:
    """Parsed scv labels of one pod. ``has_*`` mirror the ``ok`` of the Go map lookups."""

    has_number: bool
    number: int          # uint64 (wrapped) as in filter.go:13; 1 when absent
    has_memory: bool
    memory: int          # MB per card, uint64
    has_clock: bool
    clock: int           # MHz, uint64
    priority: int        # int64 (Atoi), 0 when absent
    clock_min: int = 0

    @property
    def gpu_count(self) -> int:
        """GPUs actually assigned: the label value, clamped to a sane range for gang
        selection (the reference never assigns GPUs; a wrapped negative is huge and
        can never fit anyway)."""
        return self.number

    @property
    def wants_gpu(self) -> bool:
        return True


_GPU_REQ_CACHE: dict = {}


def parse_gpu_request(labels: Mapping[str, str] | None) -> GpuRequest:
    labels = labels or {}
    n_raw = labels.get(LABEL_NUMBER)
    m_raw = labels.get(LABEL_MEMORY)
    c_raw = labels.get(LABEL_CLOCK)
    p_raw = labels.get(LABEL_PRIORITY)
    cm_raw = labels.get(LABEL_CLOCK_MIN)
    # GpuRequest is immutable and a burst repeats a handful of label combinations
    key = (n_raw, m_raw, c_raw, p_raw, cm_raw)
    r = _GPU_REQ_CACHE.get(key)
    if r is None:
        if len(_GPU_REQ_CACHE) > 4096:
            _GPU_REQ_CACHE.clear()
        r = _GPU_REQ_CACHE[key] = _parse_gpu_request(n_raw, m_raw, c_raw, p_raw, cm_raw)
    return r


def _parse_gpu_request(n_raw, m_raw, c_raw, p_raw, cm_raw) -> GpuRequest:
    return GpuRequest(
        has_number=n_raw is not None,
        number=str_to_uint(n_raw) if n_raw is not None else 1,
        has_memory=m_raw is not None,
        memory=str_to_uint(m_raw) if m_raw is not None else 0,
        has_clock=c_raw is not None,
        clock=str_to_uint(c_raw) if c_raw is not None else 0,
        priority=atoi_or_zero(p_raw) if p_raw is not None else 0,
        clock_min=str_to_uint(cm_raw) if cm_raw is not None else 0,
    )


def pod_priority(labels: Mapping[str, str] | None) -> int:
    """``sort.GetPodPriority`` (sort.go:12-18)."""
    if not labels:
        return 0
    p = labels.get(LABEL_PRIORITY)
    return atoi_or_zero(p) if p is not None else 0
