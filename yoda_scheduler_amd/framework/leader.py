"""Leader election (client-go ``leaderelection`` semantics).

The reference runs leader election on Lease ``kube-system/yoda-scheduler`` with
leaseDuration 15 s / renewDeadline 10 s / retryPeriod 2 s (``deploy/yoda-scheduler.yaml:10-17``),
and its RBAC also grants the legacy ``endpoints`` lock (``deploy:85-95``). A candidate
acquires the lock when it is free or expired (``renewTime + leaseDuration < now``), renews
it every retryPeriod with optimistic concurrency (resourceVersion), and gives up
leadership — ``lost`` is set and the scheduler stops — if it cannot renew within
renewDeadline. ``release()`` clears the holder on clean shutdown so a standby takes over
immediately.

Lock types (``leaderElection.resourceLock``, client-go ``resourcelock``): ``leases``;
``endpoints`` / ``configmaps`` (the record as JSON in the
``control-plane.alpha.kubernetes.io/leader`` annotation); ``endpointsleases`` /
``configmapsleases`` (multilock: the legacy object is primary, the Lease is kept in
step, for migrating a running deployment between lock types).
"""
from __future__ import annotations

import asyncio
import json
import logging
import random
import socket
import time
import uuid
from typing import Callable, Optional

from ..kube.errors import ApiError
from ..models.scv import parse_rfc3339, rfc3339
from ..utils import aio

log = logging.getLogger("yoda.leader")

LEADER_ANNOTATION = "control-plane.alpha.kubernetes.io/leader"
LOCK_TYPES = ("leases", "endpoints", "configmaps", "endpointsleases", "configmapsleases")


def default_identity() -> str:
    return f"{socket.gethostname()}_{uuid.uuid4()}"


class LeaseLock:
    """Record ↔ ``coordination.k8s.io/v1`` Lease spec."""
    res = "leases"

    def __init__(self, client, name: str, namespace: str) -> None:
        self.client, self.name, self.namespace = client, name, namespace

    async def get(self) -> tuple[Optional[dict], Optional[dict]]:
        try:
            obj = await self.client.get(self.res, self.name, self.namespace)
        except ApiError as e:
            if e.code == 404:
                return None, None
            raise
        sp = obj.get("spec") or {}
        return {"holderIdentity": sp.get("holderIdentity") or "",
                "leaseDurationSeconds": sp.get("leaseDurationSeconds"), "acquireTime": sp.get("acquireTime"),
                "renewTime": sp.get("renewTime"), "leaderTransitions": int(sp.get("leaseTransitions", 0) or 0)}, obj

    @staticmethod
    def _spec(rec: dict) -> dict:
        return {"holderIdentity": rec["holderIdentity"], "leaseDurationSeconds": rec["leaseDurationSeconds"],
                "acquireTime": rec["acquireTime"], "renewTime": rec["renewTime"],
                "leaseTransitions": rec["leaderTransitions"]}

    async def create(self, rec: dict) -> None:
        await self.client.create(self.res, {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                                            "metadata": {"name": self.name, "namespace": self.namespace},
                                            "spec": self._spec(rec)}, self.namespace)

    async def update(self, rec: dict, obj: dict) -> None:
        new = dict(obj)
        new["spec"] = self._spec(rec)
        await self.client.update(self.res, new, self.namespace)


class AnnotationLock(LeaseLock):
    """Record as JSON in an Endpoints / ConfigMap annotation (client-go EndpointsLock /
    ConfigMapLock)."""

    def __init__(self, client, res: str, name: str, namespace: str) -> None:
        super().__init__(client, name, namespace)
        self.res = res

    async def get(self) -> tuple[Optional[dict], Optional[dict]]:
        try:
            obj = await self.client.get(self.res, self.name, self.namespace)
        except ApiError as e:
            if e.code == 404:
                return None, None
            raise
        raw = ((obj.get("metadata") or {}).get("annotations") or {}).get(LEADER_ANNOTATION)
        rec = json.loads(raw) if raw else {"holderIdentity": "", "leaderTransitions": 0}
        return rec, obj

    async def create(self, rec: dict) -> None:
        kind = "Endpoints" if self.res == "endpoints" else "ConfigMap"
        await self.client.create(self.res, {"apiVersion": "v1", "kind": kind, "metadata": {
            "name": self.name, "namespace": self.namespace, "annotations": {LEADER_ANNOTATION: json.dumps(rec)}}},
            self.namespace)

    async def update(self, rec: dict, obj: dict) -> None:
        new = dict(obj)
        meta = dict(new.get("metadata") or {})
        meta["annotations"] = {**(meta.get("annotations") or {}), LEADER_ANNOTATION: json.dumps(rec)}
        new["metadata"] = meta
        await self.client.update(self.res, new, self.namespace)


class MultiLock:
    """Primary (legacy) lock decides; the secondary Lease is created / updated alongside."""

    def __init__(self, primary: LeaseLock, secondary: LeaseLock) -> None:
        self.primary, self.secondary = primary, secondary
        self._sec_obj: Optional[dict] = None

    async def get(self) -> tuple[Optional[dict], Optional[dict]]:
        rec, obj = await self.primary.get()
        if rec is None:
            return None, None
        _srec, self._sec_obj = await self.secondary.get()
        return rec, obj

    async def create(self, rec: dict) -> None:
        await self.primary.create(rec)
        _srec, sobj = await self.secondary.get()
        await (self.secondary.update(rec, sobj) if sobj is not None else self.secondary.create(rec))

    async def update(self, rec: dict, obj: dict) -> None:
        await self.primary.update(rec, obj)
        if self._sec_obj is None:
            await self.secondary.create(rec)
        else:
            await self.secondary.update(rec, self._sec_obj)


def make_lock(client, kind: str, name: str, namespace: str):
    if kind == "leases":
        return LeaseLock(client, name, namespace)
    if kind in ("endpoints", "configmaps"):
        return AnnotationLock(client, kind, name, namespace)
    if kind in ("endpointsleases", "configmapsleases"):
        return MultiLock(AnnotationLock(client, kind[:-len("leases")], name, namespace),
                         LeaseLock(client, name, namespace))
    raise ValueError(f"leaderElection.resourceLock must be one of {LOCK_TYPES}, got {kind!r}")


class LeaderElector:
    def __init__(self, client, name: str = "yoda-scheduler", namespace: str = "kube-system",
                 identity: Optional[str] = None, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, clock: Callable[[], float] = time.time,
                 resource_lock: str = "leases") -> None:
        if not (lease_duration > renew_deadline > retry_period > 0):
            raise ValueError("need leaseDuration > renewDeadline > retryPeriod > 0")
        self.client = client
        self.lock = make_lock(client, resource_lock, name, namespace)
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

    def _record(self, now: float, prev: Optional[dict]) -> dict:
        prev = prev or {}
        same = prev.get("holderIdentity") == self.identity
        trans = int(prev.get("leaderTransitions", 0) or 0) + (0 if same or not prev else 1)
        return {"holderIdentity": self.identity, "leaseDurationSeconds": int(round(self.lease_duration)),
                "acquireTime": prev.get("acquireTime") if same else rfc3339(now),
                "renewTime": rfc3339(now), "leaderTransitions": trans}

    async def try_acquire_or_renew(self) -> bool:
        now = self.clock()
        try:
            rec, obj = await self.lock.get()
        except ApiError as e:
            log.warning("leader lock get failed: %s", e)
            return False
        if rec is None:
            try:
                await self.lock.create(self._record(now, None))
            except ApiError:
                return False
            self._last_renew = now
            return True
        holder = rec.get("holderIdentity") or ""
        renew = parse_rfc3339(rec.get("renewTime")) or 0.0
        dur = float(rec.get("leaseDurationSeconds") or self.lease_duration)
        if holder and holder != self.identity and renew + dur > now:
            return False                       # someone else holds a valid lock
        new = self._record(now, rec)
        try:
            await self.lock.update(new, obj)
        except ApiError as e:
            if e.code != 409:
                log.warning("leader lock update failed: %s", e)
            return False
        if holder != self.identity:
            self.transitions = new["leaderTransitions"]
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
                ok = await aio.wait_for(self.try_acquire_or_renew(), self.renew_deadline)
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
            rec, obj = await self.lock.get()
            if rec is not None and rec.get("holderIdentity") == self.identity:
                rec = dict(rec, holderIdentity="", leaseDurationSeconds=1)
                await self.lock.update(rec, obj)
        except ApiError as e:
            log.warning("leader lock release failed: %s", e)
