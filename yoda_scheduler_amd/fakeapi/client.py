"""Async client bound directly to an in-process :class:`FakeApiServer`.

Same method surface as :class:`yoda_scheduler_amd.kube.client.KubeClient` (the HTTP
client), so the scheduler, sniffer publisher and leader election run unchanged
against either.
"""
from __future__ import annotations

import asyncio
import json
from typing import AsyncIterator, Optional

from ..kube.errors import ApiError
from .server import FakeApiServer


class DirectBinds:
    """The native transport's binding surface (``bind`` / ``bind_many`` with a
    ``cb(status, body)`` completion) over an in-process apiserver: each Binding is applied
    synchronously and the completions run on the next loop iteration, so the scheduler's
    all-native runs hand their Bindings over in one call instead of one bind-worker task
    switch, rate-limiter check and plugin dispatch per pod. With injected latency the
    batch waits ``latency_s`` first, as one pipelined round trip."""

    def __init__(self, server: FakeApiServer) -> None:
        self.server = server

    def bind(self, namespace: str, name: str, uid: str, node: str, annotations, cb, timeout: float = 0.0) -> None:
        self.bind_many([(namespace, name, uid, node, annotations)], [cb], timeout)

    def bind_many(self, items: list, cbs: list, timeout: float = 0.0) -> None:
        loop = asyncio.get_running_loop()
        lat = self.server.faults.latency_s
        if lat:
            loop.call_later(lat, self._apply, items, cbs)
        else:
            loop.call_soon(self._apply, items, cbs)

    def _apply(self, items: list, cbs: list) -> None:
        bind = self.server.bind
        for (ns, name, uid, node, ann), cb in zip(items, cbs):
            try:
                bind(ns, name, uid, node, dict(ann) if ann else None)
            except ApiError as e:
                cb(e.code, json.dumps(e.status_obj()).encode())
                continue
            except Exception as e:  # noqa: BLE001 - surfaced as a transport failure
                cb(-1, repr(e).encode())
                continue
            cb(201, b"")


class InProcessClient:
    def __init__(self, server: FakeApiServer) -> None:
        self.server = server

    def direct_binds(self) -> DirectBinds:
        return DirectBinds(self.server)

    async def _lat(self) -> None:
        if self.server.faults.latency_s:
            await asyncio.sleep(self.server.faults.latency_s)

    async def list(self, res: str, namespace: Optional[str] = None, resource_version: Optional[str] = None,
                   limit: int = 0, field_selector: Optional[str] = None) -> tuple[list[dict], str]:
        if self.server.faults.latency_s:
            await self._lat()
        if not limit:
            return self.server.list(res, namespace, field_selector)
        items, cont = [], ""
        while True:
            page, rv, cont = self.server.list_page(res, namespace, limit, cont, field_selector)
            items.extend(page)
            if not cont:
                return items, rv

    async def watch(self, res: str, resource_version: str,
                    field_selector: Optional[str] = None) -> AsyncIterator[tuple[str, dict]]:
        w = self.server.watch(res, resource_version, field_selector)
        try:
            async for ev in w:
                yield ev
        finally:
            w.close()

    async def watch_batches(self, res: str, resource_version: str,
                            field_selector: Optional[str] = None) -> AsyncIterator[list]:
        """``watch`` delivering every event queued since the last read as one list (the
        informer dispatches a burst's events without an async-generator hop per event)."""
        w = self.server.watch(res, resource_version, field_selector)
        try:
            while True:
                batch = await w.next_batch()
                if batch is None:
                    return
                yield batch
        finally:
            w.close()

    async def get(self, res: str, name: str, namespace: Optional[str] = None) -> dict:
        if self.server.faults.latency_s:
            await self._lat()
        return self.server.get(res, name, namespace)

    async def create(self, res: str, obj: dict, namespace: Optional[str] = None, parse: bool = True) -> dict:
        if self.server.faults.latency_s:
            await self._lat()
        return self.server.create(res, obj, namespace)

    async def update(self, res: str, obj: dict, namespace: Optional[str] = None) -> dict:
        if self.server.faults.latency_s:
            await self._lat()
        return self.server.update(res, obj, namespace)

    async def update_status(self, res: str, obj: dict, namespace: Optional[str] = None) -> dict:
        if self.server.faults.latency_s:
            await self._lat()
        return self.server.update(res, obj, namespace, status_only=True)

    async def patch(self, res: str, name: str, patch: dict, namespace: Optional[str] = None,
                    strategic: bool = False) -> dict:
        if self.server.faults.latency_s:
            await self._lat()
        return self.server.patch(res, name, patch, namespace, strategic=strategic)

    async def delete(self, res: str, name: str, namespace: Optional[str] = None) -> dict:
        if self.server.faults.latency_s:
            await self._lat()
        return self.server.delete(res, name, namespace)

    async def bind(self, namespace: str, name: str, uid: str, node: str, annotations: Optional[dict] = None) -> None:
        if self.server.faults.latency_s:
            await self._lat()
        self.server.bind(namespace, name, uid, node, annotations)

    async def close(self) -> None:
        return None
