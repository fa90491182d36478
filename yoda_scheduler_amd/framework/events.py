"""Event recorder: ``Scheduled`` / ``FailedScheduling`` / ``Preempted`` pod events
(upstream behaviour the reference's RBAC grants, ``deploy/yoda-scheduler.yaml:76-84``
for core/v1 and ``:197-204`` for events.k8s.io).

Like upstream v1.20 (``EventBroadcasterAdapter``) events go through ``events.k8s.io/v1``
by default: ``reportingController`` is the profile's scheduler name, ``action`` is
``Binding`` / ``Scheduling`` / ``Preempting``, the preemptor is the ``related`` object of a
``Preempted`` event, and repeats of an isomorphic event update its ``series``
(count, lastObservedTime). ``api="v1"`` keeps the core/v1 shape (count/lastTimestamp).

Events are buffered and written by a background task with their own rate limiter and
a per-(object, reason, message) de-duplication counter, so recording never blocks the
scheduling loop. Like client-go's broadcaster (``maxQueuedEvents = 1000``,
``DropIfChannelFull``) the buffer is bounded and a full buffer drops the *incoming*
event: a burst of thousands of pods produces more ``Scheduled`` events than the event
QPS can write, and those must not pile up in memory.
"""
from __future__ import annotations

import asyncio
import collections
import itertools
import logging
import socket
import time
import uuid
from datetime import datetime, timezone
from typing import Optional

from ..models.scv import rfc3339
from ..utils.ratelimit import TokenBucket

log = logging.getLogger("yoda.events")


ACTIONS = {"Scheduled": "Binding", "FailedScheduling": "Scheduling", "Preempted": "Preempting"}
API_EVENTS_V1 = "events.k8s.io/v1"


_SEC_CACHE = [-1, ""]


def micro_time(ts: float) -> str:
    """metav1.MicroTime: RFC 3339 with microseconds (the per-second prefix is cached: a burst
    records hundreds of events within the same second)."""
    sec = int(ts)
    us = round((ts - sec) * 1e6)
    if us >= 1_000_000:
        sec, us = sec + 1, us - 1_000_000
    if sec != _SEC_CACHE[0]:
        _SEC_CACHE[0], _SEC_CACHE[1] = sec, datetime.fromtimestamp(sec, timezone.utc).strftime("%Y-%m-%dT%H:%M:%S")
    return f"{_SEC_CACHE[1]}.{us:06d}Z"


class EventRecorder:
    def __init__(self, client, component: str = "yoda-scheduler", qps: float = 50.0, burst: int = 300,
                 max_buffer: int = 1000, enabled: bool = True, api: str = API_EVENTS_V1) -> None:
        if api not in (API_EVENTS_V1, "v1"):
            raise ValueError(f"events API must be {API_EVENTS_V1} or v1, got {api!r}")
        self.client = client
        self.component = component
        self.api = api
        self.host = socket.gethostname()
        # event names: <object>.<16 hex>; a random per-recorder prefix + counter (uuid4 per
        # event costs more than the rest of recording it)
        self._name_prefix = uuid.uuid4().hex[:8]
        self._name_seq = itertools.count(1)
        self.enabled = enabled
        self.limiter = TokenBucket(qps, burst)
        self.max_buffer = max_buffer
        self._buf: collections.deque = collections.deque()
        self._wake = asyncio.Event()
        self._dedup: dict[tuple, dict] = {}
        self.recorded = collections.Counter()
        self.dropped = 0

    def event(self, pod_obj_meta: dict, kind: str, typ: str, reason: str, message: str,
              controller: str = "", related: Optional[dict] = None) -> None:
        if not self.enabled:
            return
        self.recorded[reason] += 1
        if len(self._buf) >= self.max_buffer:
            self.dropped += 1
            return
        self._buf.append((pod_obj_meta, kind, typ, reason, message, time.time(), controller, related))
        self._wake.set()

    def pod_scheduled(self, pi, node: str) -> None:
        """``Scheduled`` for a bound pod; the message is formatted only if the event is kept
        (a burst fills the buffer and then drops most of them)."""
        if not self.enabled:
            return
        if len(self._buf) >= self.max_buffer:
            self.recorded["Scheduled"] += 1
            self.dropped += 1
            return
        self.pod_event(pi, "Normal", "Scheduled", f"Successfully assigned {pi.namespace}/{pi.name} to {node}")

    def pod_event(self, pi, typ: str, reason: str, message: str, related=None) -> None:
        if self.enabled:
            rel = None if related is None else {"apiVersion": "v1", "kind": "Pod", "name": related.name,
                                                "namespace": related.namespace, "uid": related.uid}
            self.event({"name": pi.name, "namespace": pi.namespace, "uid": pi.uid}, "Pod", typ, reason, message,
                       pi.scheduler_name, rel)

    def _new_v1(self, meta, kind, typ, reason, message, ts, controller, related) -> dict:
        ctl = controller or self.component
        ev = {"apiVersion": API_EVENTS_V1, "kind": "Event",
              "metadata": {"name": f"{meta.get('name')}.{self._name_prefix}{next(self._name_seq):08x}",
                           "namespace": meta.get("namespace") or "default"},
              "eventTime": micro_time(ts), "reportingController": ctl, "reportingInstance": f"{ctl}-{self.host}",
              "action": ACTIONS.get(reason, reason), "reason": reason,
              "regarding": {"apiVersion": "v1", "kind": kind, **meta}, "note": message[:1024], "type": typ}
        if related:
            ev["related"] = related
        return ev

    async def _write_v1(self, key, item) -> None:
        meta, kind, typ, reason, message, ts, controller, related = item
        prev = self._dedup.get(key)
        if prev is not None:      # isomorphic event: bump the series
            series = dict(prev.get("series") or {"count": 1})
            series["count"] = int(series.get("count", 1)) + 1
            series["lastObservedTime"] = micro_time(ts)
            self._dedup[key] = await self.client.patch("events.k8s.io", prev["metadata"]["name"],
                                                       {"series": series}, meta.get("namespace") or "default")
        else:
            # the dedup record needs only what we sent (the name a series bump patches): the
            # created object is not decoded
            ev = self._new_v1(meta, kind, typ, reason, message, ts, controller, related)
            await self.client.create("events.k8s.io", ev, meta.get("namespace"), parse=False)
            self._dedup[key] = ev

    async def run(self) -> None:
        while True:
            if not self._buf:
                self._wake.clear()
                await self._wake.wait()
            item = self._buf.popleft()
            meta, kind, typ, reason, message, ts, controller, related = item
            await self.limiter.acquire()
            key = (meta.get("namespace"), meta.get("name"), reason, message, controller,
                   (related or {}).get("uid"))
            try:
                if self.api == API_EVENTS_V1:
                    await self._write_v1(key, item)
                    if len(self._dedup) > 10_000:
                        self._dedup.clear()
                    continue
                prev = self._dedup.get(key)
                if prev is not None:
                    prev = dict(prev, count=prev.get("count", 1) + 1, lastTimestamp=rfc3339(ts))
                    prev["metadata"] = dict(prev["metadata"])
                    self._dedup[key] = await self.client.update("events", prev, meta.get("namespace"))
                else:
                    ev = {
                        "apiVersion": "v1", "kind": "Event",
                        "metadata": {"name": f"{meta.get('name')}.{self._name_prefix}{next(self._name_seq):08x}",
                                     "namespace": meta.get("namespace") or "default"},
                        "involvedObject": {"kind": kind, **meta},
                        "reason": reason, "message": message, "type": typ,
                        "source": {"component": controller or self.component},
                        "firstTimestamp": rfc3339(ts), "lastTimestamp": rfc3339(ts), "count": 1,
                    }
                    self._dedup[key] = await self.client.create("events", ev, meta.get("namespace"))
                    if len(self._dedup) > 10_000:
                        self._dedup.clear()
            except Exception as e:  # noqa: BLE001 - events are best effort
                log.debug("event write failed: %r", e)
