"""Lease-based leader election (client-go ``leaderelection`` semantics).

The reference runs leader election on Lease ``kube-system/yoda-scheduler`` with
leaseDuration 15 s / renewDeadline 10 s / retryPeriod 2 s (``deploy/yoda-scheduler.yaml:10-17``).
A candidate acquires the lease when it is free or expired (``renewTime + leaseDuration <
now``), renews it every retryPeriod with optimistic concurrency (resourceVersion), and
gives up leadership — ``lost`` is set and the scheduler stops — if it cannot renew within
renewDeadline. ``release()`` clears the holder on clean shutdown so a standby takes over
immediately.
"""
from __future__ import annotations

import asyncio
import logging
import random
import socket
import time
import uuid
from typing import Callable, Optional

from ..kube.errors import ApiError
from ..models.scv import parse_rfc3339, rfc3339

log = logging.getLogger("yoda.leader")


def default_identity() -> str:
    return f"{socket.gethostname()}_{uuid.uuid4()}"


class LeaderElector:
    def __init__(self, client, name: str = "yoda-scheduler", namespace: str = "kube-system",
                 identity: Optional[str] = None, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, clock: Callable[[], float] = time.time) -> None:
        if not (lease_duration > renew_deadline > retry_period > 0):
            raise ValueError("need leaseDuration > renewDeadline > retryPeriod > 0")
        self.client = client
        self.name = name
        self.namespace = namespace
        self.identity = identity or default_identity()
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.clock = clock
        self.is_leader = False
        self.lost = asyncio.Event()
        self.transitions = 0
        self._last_renew = 0.0
        self._task: Optional[asyncio.Task] = None

    def _spec(self, now: float, prev: Optional[dict]) -> dict:
        prev = prev or {}
        same = prev.get("holderIdentity") == self.identity
        trans = int(prev.get("leaseTransitions", 0) or 0) + (0 if same or not prev else 1)
        return {"holderIdentity": self.identity, "leaseDurationSeconds": int(round(self.lease_duration)),
                "acquireTime": prev.get("acquireTime") if same else rfc3339(now),
                "renewTime": rfc3339(now), "leaseTransitions": trans}

    async def try_acquire_or_renew(self) -> bool:
        now = self.clock()
        try:
            lease = await self.client.get("leases", self.name, self.namespace)
        except ApiError as e:
            if e.code != 404:
                log.warning("lease get failed: %s", e)
                return False
            obj = {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                   "metadata": {"name": self.name, "namespace": self.namespace}, "spec": self._spec(now, None)}
            try:
                await self.client.create("leases", obj, self.namespace)
            except ApiError:
                return False
            self._last_renew = now
            return True
        spec = lease.get("spec") or {}
        holder = spec.get("holderIdentity") or ""
        renew = parse_rfc3339(spec.get("renewTime")) or 0.0
        dur = float(spec.get("leaseDurationSeconds") or self.lease_duration)
        if holder and holder != self.identity and renew + dur > now:
            return False                       # someone else holds a valid lease
        new = dict(lease)
        new["spec"] = self._spec(now, spec)
        try:
            await self.client.update("leases", new, self.namespace)
        except ApiError as e:
            if e.code != 409:
                log.warning("lease update failed: %s", e)
            return False
        if holder != self.identity:
            self.transitions = new["spec"]["leaseTransitions"]
        self._last_renew = now
        return True

    async def acquire(self) -> None:
        """Block until this candidate is the leader, then keep renewing in the background."""
        while True:
            if await self.try_acquire_or_renew():
                break
            await asyncio.sleep(self.retry_period * (1.0 + 0.2 * random.random()))
        self.is_leader = True
        self.lost.clear()
        log.info("%s became leader of %s/%s", self.identity, self.namespace, self.name)
        self._task = asyncio.get_event_loop().create_task(self._renew_loop())

    async def _renew_loop(self) -> None:
        while self.is_leader:
            await asyncio.sleep(self.retry_period)
            ok = False
            try:
                ok = await asyncio.wait_for(self.try_acquire_or_renew(), self.renew_deadline)
            except asyncio.TimeoutError:
                ok = False
            if not ok and self.clock() - self._last_renew > self.renew_deadline:
                self.is_leader = False
                self.lost.set()
                log.error("%s lost leadership of %s/%s", self.identity, self.namespace, self.name)
                return

    async def release(self) -> None:
        if self._task is not None:
            self._task.cancel()
            await asyncio.gather(self._task, return_exceptions=True)
        if not self.is_leader:
            return
        self.is_leader = False
        try:
            lease = await self.client.get("leases", self.name, self.namespace)
            spec = dict(lease.get("spec") or {})
            if spec.get("holderIdentity") == self.identity:
                spec["holderIdentity"] = ""
                spec["leaseDurationSeconds"] = 1
                new = dict(lease)
                new["spec"] = spec
                await self.client.update("leases", new, self.namespace)
        except ApiError as e:
            log.warning("lease release failed: %s", e)
