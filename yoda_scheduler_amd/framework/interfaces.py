"""Scheduling-framework extension points, Status and CycleState.

Mirrors the upstream kube-scheduler framework the reference plugs into
(``pkg/yoda/scheduler.go:27-32`` asserts QueueSort, Filter, PostFilter, Score and
ScoreExtensions; the factory signature is ``New(args, handle)`` at ``:46``). Plugins
written against this module look like upstream plugins; the yoda plugin and the
hot default plugins additionally declare a *native* binding so the whole cycle can
run inside the C++ engine.
"""
from __future__ import annotations

import copy
import enum
import threading
from dataclasses import dataclass, field
from typing import Any, Optional

MAX_NODE_SCORE = 100
MIN_NODE_SCORE = 0


class Code(enum.IntEnum):
    SUCCESS = 0
    ERROR = 1
    UNSCHEDULABLE = 2
    UNSCHEDULABLE_AND_UNRESOLVABLE = 3
    WAIT = 4
    SKIP = 5


@dataclass
class Status:
    code: Code = Code.SUCCESS
    reasons: list[str] = field(default_factory=list)
    plugin: str = ""

    @classmethod
    def ok(cls) -> "Status":
        return _OK

    @classmethod
    def unschedulable(cls, *reasons: str, plugin: str = "") -> "Status":
        return cls(Code.UNSCHEDULABLE, list(reasons), plugin)

    @classmethod
    def unresolvable(cls, *reasons: str, plugin: str = "") -> "Status":
        """``UnschedulableAndUnresolvable``: preemption cannot help on this node."""
        return cls(Code.UNSCHEDULABLE_AND_UNRESOLVABLE, list(reasons), plugin)

    @classmethod
    def error(cls, *reasons: str, plugin: str = "") -> "Status":
        return cls(Code.ERROR, list(reasons), plugin)

    def is_success(self) -> bool:
        return self.code == Code.SUCCESS

    def is_unschedulable(self) -> bool:
        return self.code in (Code.UNSCHEDULABLE, Code.UNSCHEDULABLE_AND_UNRESOLVABLE)

    def message(self) -> str:
        return ", ".join(self.reasons)


_OK = Status()


class StateData:
    def clone(self) -> "StateData":
        return copy.copy(self)


class CycleState:
    """Per-cycle scratch map. ``write`` under ``lock`` like upstream v1.20 (the
    reference takes the lock explicitly, ``pkg/yoda/collection/collection.go:53-55``)."""

    __slots__ = ("_data", "_lock", "record_metrics")

    def __init__(self) -> None:
        self._data: dict[str, StateData] = {}
        self._lock = None        # created on first use: most cycles never lock
        self.record_metrics = False

    def read(self, key: str) -> StateData:
        try:
            return self._data[key]
        except KeyError:
            raise KeyError(f"{key!r} not found") from None

    def write(self, key: str, val: StateData) -> None:
        self._data[key] = val

    def delete(self, key: str) -> None:
        self._data.pop(key, None)

    def lock(self):
        if self._lock is None:
            self._lock = threading.RLock()
        return self._lock

    def clone(self) -> "CycleState":
        c = CycleState()
        c._data = {k: v.clone() for k, v in self._data.items()}
        return c


@dataclass
class NodeScore:
    name: str
    score: int


# ----------------------------------------------------------------------------- plugins
class Plugin:
    name: str = ""

    def __init__(self, args: Optional[dict] = None, handle: Any = None) -> None:
        self.args = args or {}
        self.handle = handle

    # a plugin with a native implementation returns its engine binding descriptor
    def native(self) -> Optional["NativeBinding"]:
        return None


@dataclass(frozen=True)
class NativeBinding:
    filter_bit: int = 0            # engine filter bit (0 = none)
    score_index: int = -1          # engine score slot (-1 = none)


class QueueSortPlugin(Plugin):
    def less(self, a, b) -> bool:
        return self.sort_key(a) < self.sort_key(b)

    def sort_key(self, pi) -> tuple:
        raise NotImplementedError


class PreFilterPlugin(Plugin):
    def pre_filter(self, state: CycleState, pod) -> Status:
        raise NotImplementedError


class FilterPlugin(Plugin):
    def filter(self, state: CycleState, pod, node_name: str) -> Status:
        raise NotImplementedError


class PostFilterResult:
    def __init__(self, nominated_node: str = "", cards: Optional[list] = None) -> None:
        self.nominated_node = nominated_node
        self.cards = cards          # GPUs the preemptor will use there (nominated reservation)


class PostFilterPlugin(Plugin):
    def post_filter(self, state: CycleState, pod, statuses: dict) -> tuple[Optional[PostFilterResult], Status]:
        raise NotImplementedError


class PreScorePlugin(Plugin):
    def pre_score(self, state: CycleState, pod, nodes: list[str]) -> Status:
        raise NotImplementedError


class ScorePlugin(Plugin):
    def score(self, state: CycleState, pod, node_name: str) -> tuple[int, Status]:
        raise NotImplementedError

    def normalize_score(self, state: CycleState, pod, scores: list[NodeScore]) -> Status:
        return Status.ok()

    def has_normalize(self) -> bool:
        return type(self).normalize_score is not ScorePlugin.normalize_score


class ReservePlugin(Plugin):
    def reserve(self, state: CycleState, pod, node_name: str) -> Status:
        return Status.ok()

    def unreserve(self, state: CycleState, pod, node_name: str) -> None:
        return None


class PermitPlugin(Plugin):
    def permit(self, state: CycleState, pod, node_name: str) -> tuple[Status, float]:
        """Success, an error/unschedulable status, or ``Status(Code.WAIT)`` with a timeout in
        seconds: the pod is then held (assumed, not bound) until every waiting plugin calls
        ``allow`` on its :class:`WaitingPod` or one calls ``reject``, or the timeout hits."""
        return Status.ok(), 0.0


class WaitingPod:
    """A pod whose Permit returned Wait (upstream ``framework.WaitingPod``)."""

    def __init__(self, pod, node: str, plugins: set, timeout: float) -> None:
        import asyncio
        self.pod = pod
        self.node = node
        self.pending = set(plugins)
        self.timeout = timeout
        self._fut = asyncio.get_event_loop().create_future()

    def allow(self, plugin: str) -> None:
        self.pending.discard(plugin)
        if not self.pending and not self._fut.done():
            self._fut.set_result(_OK)

    def reject(self, plugin: str, msg: str = "") -> None:
        if not self._fut.done():
            self._fut.set_result(Status(Code.UNSCHEDULABLE, [msg or f"rejected by {plugin}"], plugin))

    async def wait(self) -> "Status":
        import asyncio
        try:
            return await asyncio.wait_for(asyncio.shield(self._fut), self.timeout)
        except asyncio.TimeoutError:
            return Status(Code.UNSCHEDULABLE, ["rejected due to timeout after waiting at permit"], "")


class PreBindPlugin(Plugin):
    async def pre_bind(self, state: CycleState, pod, node_name: str) -> Status:
        return Status.ok()


class BindPlugin(Plugin):
    async def bind(self, state: CycleState, pod, node_name: str) -> Status:
        raise NotImplementedError


class PostBindPlugin(Plugin):
    def post_bind(self, state: CycleState, pod, node_name: str) -> None:
        return None


EXTENSION_POINTS = ("queueSort", "preFilter", "filter", "postFilter", "preScore", "score",
                    "reserve", "permit", "preBind", "bind", "postBind")

POINT_TYPES = {
    "queueSort": QueueSortPlugin, "preFilter": PreFilterPlugin, "filter": FilterPlugin,
    "postFilter": PostFilterPlugin, "preScore": PreScorePlugin, "score": ScorePlugin,
    "reserve": ReservePlugin, "permit": PermitPlugin, "preBind": PreBindPlugin,
    "bind": BindPlugin, "postBind": PostBindPlugin,
}
