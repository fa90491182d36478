"""The ``yoda`` plugin (``pkg/yoda/scheduler.go``), MI355X-native.

Extension points, as in the reference (``scheduler.go:27-32``): QueueSort (``scv/priority``,
``sort.go``), Filter (``filter.go``), PostFilter (``collection.go``), Score +
NormalizeScore (``algorithm.go``, ``scheduler.go:132-157``). Filter/Score/Normalize and
the GPU-set Reserve run natively inside the engine cycle (``native/core/engine.cpp``);
this class carries the configuration and the Python-visible pieces.

Plugin args (``pluginConfig[].args`` for ``yoda``):
  compat: false        reproduce the reference bit-exactly (quirks Q2/Q3, no HBM ledger)
  staleFactor: 3.0     Scv older than factor × updateInterval → node unschedulable
  gpuStrategy: spread|binpack     GPU choice inside a node (worst-fit vs best-fit)
  gangWeights: {link: 4, numa: 2, fit: 1, occupancy: 1, score: 3, enumLimit: 5000}

Unlike the reference there is one shared Scv informer per process (Q8), scheduling is
gated on informer sync (Q9), and the cluster maxima are computed in PreScore so
multi-node clusters actually schedule (Q1).
"""
from __future__ import annotations

from typing import Optional

from ..framework.interfaces import (CycleState, FilterPlugin, NativeBinding, PostFilterPlugin, PostFilterResult,
                                    QueueSortPlugin, ScorePlugin, Status)
from ..ops.native import core

NAME = "yoda"


class Yoda(QueueSortPlugin, FilterPlugin, PostFilterPlugin, ScorePlugin):
    name = NAME

    def __init__(self, args: Optional[dict] = None, handle=None) -> None:
        super().__init__(args, handle)
        a = self.args
        self.compat = bool(a.get("compat", False))
        self.stale_factor = float(a.get("staleFactor", 3.0))
        # a reservation counts against the sniffed free HBM until a sample taken this long
        # after it (container start + allocation) is expected to show its usage
        self.settle_seconds = float(a.get("sampleSettleSeconds", 30.0))
        # "spread" (default) fills a node's GPUs evenly (worst-fit): with HBM-sharing pods
        # it keeps the per-GPU free HBM level, so multi-GPU gangs stay placeable until the
        # node is nearly full. "binpack" (best-fit) keeps whole GPUs empty instead — the
        # better choice when most pods want dedicated GPUs.
        self.gpu_strategy = str(a.get("gpuStrategy", "spread")).lower()
        if self.gpu_strategy not in ("binpack", "spread"):
            raise ValueError(f"yoda: gpuStrategy must be binpack|spread, got {self.gpu_strategy!r}")
        gw = a.get("gangWeights") or {}
        self.gang = dict(link=int(gw.get("link", 4)), numa=int(gw.get("numa", 2)), fit=int(gw.get("fit", 1)),
                         occ=int(gw.get("occupancy", 1)), gang_score=int(gw.get("score", 3)),
                         enum_limit=int(gw.get("enumLimit", 5000)), minlink=int(gw.get("minLink", 2)))

    def native(self):
        c = core()
        return NativeBinding(filter_bit=c.F_YODA, score_index=c.S_YODA)

    def configure_engine(self, engine) -> None:
        engine.set_gang_weights(binpack=self.gpu_strategy == "binpack", **self.gang)
        engine.settle_seconds = self.settle_seconds

    # QueueSort: sort.Less (sort.go:8-10) + FIFO tie-break (Q7)
    def sort_key(self, pi) -> tuple:
        return (-pi.gpu.priority,)

    # PostFilter: the reference writes the cluster maxima here (collection.go:30-57).
    # The native engine computes them in PreScore (Q1), so nothing is left to do.
    def post_filter(self, state: CycleState, pod, statuses: dict):
        return PostFilterResult(), Status.unschedulable("yoda: no node has enough healthy GPUs", plugin=NAME)


def new(args, handle):
    """Plugin factory with the reference's signature (``yoda.New``, scheduler.go:46)."""
    return Yoda(args, handle)
