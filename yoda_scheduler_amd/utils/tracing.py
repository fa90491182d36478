"""Scheduling-cycle tracer → Chrome trace JSON (``chrome://tracing`` / Perfetto).

SURVEY §5 tracing row: upstream only offers pprof; this records one span per scheduling
cycle / native batch / bind (bounded ring buffer, ~1 µs per span) and serves them at
``/debug/trace`` of the status server. Enable with ``yodaRuntime.trace: true`` or
``yoda-scheduler --trace``.
"""
from __future__ import annotations

import collections
import os
import threading
import time
from typing import Optional


class Tracer:
    def __init__(self, capacity: int = 200_000) -> None:
        self._ev: collections.deque = collections.deque(maxlen=capacity)
        self._t0 = time.perf_counter()
        self._pid = os.getpid()

    def now_us(self) -> float:
        return (time.perf_counter() - self._t0) * 1e6

    def span(self, name: str, start_us: float, end_us: Optional[float] = None, cat: str = "sched",
             tid: int = 0, **args) -> None:
        end = self.now_us() if end_us is None else end_us
        self._ev.append({"name": name, "cat": cat, "ph": "X", "ts": round(start_us, 3),
                         "dur": round(max(end - start_us, 0.0), 3), "pid": self._pid,
                         "tid": tid or threading.get_ident() % 100000, "args": args})

    def instant(self, name: str, cat: str = "sched", **args) -> None:
        self._ev.append({"name": name, "cat": cat, "ph": "i", "s": "t", "ts": round(self.now_us(), 3),
                         "pid": self._pid, "tid": threading.get_ident() % 100000, "args": args})

    def __len__(self) -> int:
        return len(self._ev)

    def chrome_trace(self) -> dict:
        return {"traceEvents": list(self._ev), "displayTimeUnit": "ms"}

    def dump(self, path: str) -> None:
        import json
        with open(path, "w") as f:
            json.dump(self.chrome_trace(), f)
