"""List/watch reflector with an indexer-free local store (client-go informer analogue).

One informer per resource per process: the reference runs a *second* controller-runtime
manager per profile just to watch ``Scv`` (``pkg/yoda/scheduler.go:53-68``, quirk Q8);
here all profiles share these informers, and ``synced`` gates scheduling (Q9).
"""
from __future__ import annotations

import asyncio
import logging
from typing import Callable, Optional

from .errors import ApiError
from .resources import obj_key, resource

log = logging.getLogger("yoda.informer")

Handler = Callable[[dict], None]


class Informer:
    def __init__(self, client, res: str, on_add: Optional[Handler] = None,
                 on_update: Optional[Callable[[dict, dict], None]] = None,
                 on_delete: Optional[Handler] = None, relist_backoff: float = 0.2,
                 field_selector: Optional[str] = None) -> None:
        self.client = client
        self.field_selector = field_selector
        self.res = res
        self.r = resource(res)
        self.on_add, self.on_update, self.on_delete = on_add, on_update, on_delete
        self.store: dict[str, dict] = {}
        self.synced = asyncio.Event()
        self.resource_version = "0"
        self.relist_backoff = relist_backoff
        self.relists = 0
        self.bookmarks = 0
        self.page_size = 500            # client-go pager default
        self._consistent_relist = False
        self._stop = False

    def _dispatch(self, typ: str, obj: dict) -> None:
        key = obj_key(self.r, obj)
        if typ == "DELETED":
            old = self.store.pop(key, None)
            if self.on_delete:
                self.on_delete(old or obj)
        else:
            old = self.store.get(key)
            self.store[key] = obj
            if old is None:
                if self.on_add:
                    self.on_add(obj)
            elif self.on_update:
                self.on_update(old, obj)
        rv = (obj.get("metadata") or {}).get("resourceVersion")
        if rv:
            self.resource_version = rv

    def _fs(self) -> dict:
        return {"field_selector": self.field_selector} if self.field_selector else {}

    async def _list(self) -> None:
        # client-go reflector: the first list may come from the watch cache (RV "0");
        # after a 410 the relist is a consistent read, paged like client-go's pager
        if self._consistent_relist:
            items, rv = await self.client.list(self.res, resource_version="", limit=self.page_size,
                                               **self._fs())
            self._consistent_relist = False
        else:
            items, rv = await self.client.list(self.res, resource_version="0", **self._fs())
        fresh = {obj_key(self.r, o): o for o in items}
        # deletions that happened while we were not watching
        for key in [k for k in self.store if k not in fresh]:
            old = self.store.pop(key)
            if self.on_delete:
                self.on_delete(old)
        for key, o in fresh.items():
            old = self.store.get(key)
            self.store[key] = o
            if old is None:
                if self.on_add:
                    self.on_add(o)
            elif old.get("metadata", {}).get("resourceVersion") != o.get("metadata", {}).get("resourceVersion"):
                if self.on_update:
                    self.on_update(old, o)
        self.resource_version = rv
        self.relists += 1

    async def run(self) -> None:
        need_list = True
        while not self._stop:
            try:
                if need_list:
                    await self._list()
                    self.synced.set()
                    need_list = False
                async for typ, obj in self.client.watch(self.res, self.resource_version, **self._fs()):
                    if typ == "ERROR":
                        need_list = True
                        break
                    if typ == "BOOKMARK":
                        rv = (obj.get("metadata") or {}).get("resourceVersion")
                        if rv:
                            self.resource_version = rv
                            self.bookmarks += 1
                        continue
                    self._dispatch(typ, obj)
                    if self._stop:
                        return
                # watch closed by the server: resume from the last resourceVersion
            except ApiError as e:
                if e.code == 410:
                    need_list = True
                    self._consistent_relist = True
                else:
                    log.warning("informer %s: %s", self.res, e)
                    await asyncio.sleep(self.relist_backoff)
                    need_list = True
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001 - keep the reflector alive
                log.warning("informer %s error: %r", self.res, e)
                await asyncio.sleep(self.relist_backoff)
                need_list = True

    def stop(self) -> None:
        self._stop = True
