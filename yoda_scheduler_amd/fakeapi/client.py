"""Async client bound directly to an in-process :class:`FakeApiServer`.

Same method surface as :class:`yoda_scheduler_amd.kube.client.KubeClient` (the HTTP
client), so the scheduler, sniffer publisher and leader election run unchanged
against either.
"""
from __future__ import annotations

import asyncio
from typing import AsyncIterator, Optional

from .server import FakeApiServer


class InProcessClient:
    def __init__(self, server: FakeApiServer) -> None:
        self.server = server

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
