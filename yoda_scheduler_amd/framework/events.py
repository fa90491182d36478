"""Event recorder: ``Scheduled`` / ``FailedScheduling`` / ``Preempted`` pod events
(upstream behaviour the reference's RBAC grants, ``deploy/yoda-scheduler.yaml:76-84``).

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
import logging
import time
import uuid

from ..models.scv import rfc3339
from ..utils.ratelimit import TokenBucket

log = logging.getLogger("yoda.events")


class EventRecorder:
    def __init__(self, client, component: str = "yoda-scheduler", qps: float = 50.0, burst: int = 300,
                 max_buffer: int = 1000, enabled: bool = True) -> None:
        self.client = client
        self.component = component
        self.enabled = enabled
        self.limiter = TokenBucket(qps, burst)
        self.max_buffer = max_buffer
        self._buf: collections.deque = collections.deque()
        self._wake = asyncio.Event()
        self._dedup: dict[tuple, dict] = {}
        self.recorded = collections.Counter()
        self.dropped = 0

    def event(self, pod_obj_meta: dict, kind: str, typ: str, reason: str, message: str) -> None:
        if not self.enabled:
            return
        self.recorded[reason] += 1
        if len(self._buf) >= self.max_buffer:
            self.dropped += 1
            return
        self._buf.append((pod_obj_meta, kind, typ, reason, message, time.time()))
        self._wake.set()

    def pod_event(self, pi, typ: str, reason: str, message: str) -> None:
        if self.enabled:
            self.event({"name": pi.name, "namespace": pi.namespace, "uid": pi.uid}, "Pod", typ, reason, message)

    async def run(self) -> None:
        while True:
            if not self._buf:
                self._wake.clear()
                await self._wake.wait()
            meta, kind, typ, reason, message, ts = self._buf.popleft()
            await self.limiter.acquire()
            key = (meta.get("namespace"), meta.get("name"), reason, message)
            try:
                prev = self._dedup.get(key)
                if prev is not None:
                    prev = dict(prev, count=prev.get("count", 1) + 1, lastTimestamp=rfc3339(ts))
                    prev["metadata"] = dict(prev["metadata"])
                    self._dedup[key] = await self.client.update("events", prev, meta.get("namespace"))
                else:
                    ev = {
                        "apiVersion": "v1", "kind": "Event",
                        "metadata": {"name": f"{meta.get('name')}.{uuid.uuid4().hex[:16]}",
                                     "namespace": meta.get("namespace") or "default"},
                        "involvedObject": {"kind": kind, **meta},
                        "reason": reason, "message": message, "type": typ,
                        "source": {"component": self.component},
                        "firstTimestamp": rfc3339(ts), "lastTimestamp": rfc3339(ts), "count": 1,
                    }
                    self._dedup[key] = await self.client.create("events", ev, meta.get("namespace"))
                    if len(self._dedup) > 10_000:
                        self._dedup.clear()
            except Exception as e:  # noqa: BLE001 - events are best effort
                log.debug("event write failed: %r", e)
