"""List/watch reflector with an indexer-free local store (client-go informer analogue).

One informer per resource per process: the reference runs a *second* controller-runtime
manager per profile just to watch ``Scv`` (``pkg/yoda/scheduler.go:53-68``, quirk Q8);
here all profiles share these informers, and ``synced`` gates scheduling (Q9).

Failure handling follows client-go's reflector (``ListAndWatch`` under
``wait.BackoffUntil``): a 410 Gone relists at once (consistent, paged); any other list or
watch error relists after an exponential backoff with jitter (0.8 s → 30 s, reset after a
quiet period), so an unreachable apiserver sees a bounded request rate. Event-handler
exceptions are logged and counted per handler call and never restart the reflector (a
single bad object must not cause a relist storm).

:class:`NativePodInformer` is the pod reflector on the native transport: events arrive
decoded and projected by C++ (``PodEvent``), are dispatched synchronously from the
transport's eventfd callback, and the store keeps the events, decoding a pod to a dict
only when a lister asks for it.
"""
from __future__ import annotations

import asyncio
import collections.abc
import json
import logging
import random
import time
from typing import Callable, Optional

from .errors import ApiError
from .resources import obj_key, resource

log = logging.getLogger("yoda.informer")

Handler = Callable[[dict], None]


class Backoff:
    """client-go ``wait.Backoff`` as the reflector uses it: ``initial`` doubling up to
    ``cap``, each sleep stretched by up to ``jitter`` × itself, back to ``initial`` after
    ``reset_after`` seconds without a failure."""

    def __init__(self, initial: float = 0.8, cap: float = 30.0, factor: float = 2.0, jitter: float = 1.0,
                 reset_after: float = 120.0, rng: Callable[[], float] = random.random,
                 clock: Callable[[], float] = time.monotonic) -> None:
        self.initial, self.cap, self.factor, self.jitter = initial, cap, factor, jitter
        self.reset_after, self.rng, self.clock = reset_after, rng, clock
        self._cur = initial
        self._last = None

    def next(self) -> float:
        now = self.clock()
        if self._last is not None and now - self._last > self.reset_after:
            self._cur = self.initial
        self._last = now
        d = self._cur
        self._cur = min(self.cap, self._cur * self.factor)
        return d * (1.0 + self.jitter * self.rng()) if self.jitter else d

    def reset(self) -> None:
        self._cur = self.initial


_EMPTY: dict = {}


class Informer:
    def __init__(self, client, res: str, on_add: Optional[Handler] = None,
                 on_update: Optional[Callable[[dict, dict], None]] = None,
                 on_delete: Optional[Handler] = None, relist_backoff: float = 0.8,
                 field_selector: Optional[str] = None, max_backoff: float = 30.0) -> None:
        self.client = client
        self.field_selector = field_selector
        self.res = res
        self.r = resource(res)
        self.on_add, self.on_update, self.on_delete = on_add, on_update, on_delete
        self.store: dict[str, dict] = {}
        self.synced = asyncio.Event()
        self.resource_version = "0"
        self.backoff = Backoff(relist_backoff, max(relist_backoff, max_backoff))
        self.relists = 0
        self.bookmarks = 0
        self.handler_errors = 0
        self.errors = 0
        self.page_size = 500            # client-go pager default
        self._consistent_relist = False
        self._stop = False

    def _call(self, fn, *args) -> None:
        try:
            fn(*args)
        except Exception:  # noqa: BLE001 - isolate handlers: log, count, keep the stream
            self.handler_errors += 1
            log.exception("informer %s: event handler failed", self.res)

    def _dispatch(self, typ: str, obj: dict) -> None:
        m = obj.get("metadata") or _EMPTY
        key = f"{m.get('namespace') or 'default'}/{m.get('name', '')}" if self.r.namespaced else m.get("name", "")
        if typ == "DELETED":
            old = self.store.pop(key, None)
            if self.on_delete:
                self._call(self.on_delete, old or obj)
        else:
            old = self.store.get(key)
            self.store[key] = obj
            if old is None:
                if self.on_add:
                    self._call(self.on_add, obj)
            elif self.on_update:
                self._call(self.on_update, old, obj)
        rv = m.get("resourceVersion")
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
                self._call(self.on_delete, old)
        for key, o in fresh.items():
            old = self.store.get(key)
            self.store[key] = o
            if old is None:
                if self.on_add:
                    self._call(self.on_add, o)
            elif old.get("metadata", {}).get("resourceVersion") != o.get("metadata", {}).get("resourceVersion"):
                if self.on_update:
                    self._call(self.on_update, old, o)
        self.resource_version = rv
        self.relists += 1

    def _event(self, typ: str, obj: dict) -> None:
        if typ == "ERROR":
            raise ApiError(int(obj.get("code", 500)), obj.get("reason", "Error"), obj.get("message", ""))
        if typ == "BOOKMARK":
            rv = (obj.get("metadata") or {}).get("resourceVersion")
            if rv:
                self.resource_version = rv
                self.bookmarks += 1
            return
        self._dispatch(typ, obj)

    async def _watch_once(self) -> None:
        batches = getattr(self.client, "watch_batches", None)
        if batches is not None:           # in-process apiserver: a burst's events per read
            async for batch in batches(self.res, self.resource_version, **self._fs()):
                for typ, obj in batch:
                    self._event(typ, obj)
                    if self._stop:
                        return
            return
        async for typ, obj in self.client.watch(self.res, self.resource_version, **self._fs()):
            self._event(typ, obj)
            if self._stop:
                return

    async def run(self) -> None:
        need_list = True
        while not self._stop:
            try:
                if need_list:
                    await self._list()
                    self.synced.set()
                    need_list = False
                await self._watch_once()
                # watch closed by the server (timeoutSeconds): resume from the last resourceVersion
            except ApiError as e:
                if e.code == 410:
                    need_list = True
                    self._consistent_relist = True
                    continue
                self.errors += 1
                log.warning("informer %s: %s", self.res, e)
                await asyncio.sleep(self.backoff.next())
                need_list = True
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001 - keep the reflector alive
                self.errors += 1
                log.warning("informer %s error: %r", self.res, e)
                await asyncio.sleep(self.backoff.next())
                need_list = True

    def stop(self) -> None:
        self._stop = True


class LazyPodStore(collections.abc.Mapping):
    """``key → pod dict`` view of a :class:`NativePodInformer`: decodes on access."""

    def __init__(self, entries: dict) -> None:
        self._e = entries

    def __getitem__(self, key: str) -> dict:
        return json.loads(self._e[key][0].raw())

    def get(self, key, default=None):
        e = self._e.get(key)
        return json.loads(e[0].raw()) if e is not None else default

    def __contains__(self, key) -> bool:
        return key in self._e

    def __iter__(self):
        return iter(self._e)

    def __len__(self) -> int:
        return len(self._e)


PodNativeHandler = Callable[[str, object, tuple, Optional[tuple]], None]


class NativePodInformer(Informer):
    """Pod reflector over the native transport. ``on_event(type, PodEvent, ident, old)``
    with ``ident = (key, uid, node, scheduler, phase, spec/meta hash)`` and ``old`` the
    previous ``(PodEvent, ident)`` of the key (``None`` for a new pod)."""

    def __init__(self, client, on_event: PodNativeHandler, field_selector: Optional[str] = None,
                 relist_backoff: float = 0.8, max_backoff: float = 30.0, lane=None) -> None:
        """``lane``: a native pod lane (``core.Lane``) attached to the transport as its pod
        sink. It then receives every pod watch event and owns the store; this informer only
        keeps the stream alive (bookmarks, errors, re-watch / relist) and the lane forwards
        to ``on_event`` the events Python must see."""
        super().__init__(client, "pods", relist_backoff=relist_backoff, field_selector=field_selector,
                         max_backoff=max_backoff)
        self.on_event = on_event
        self.lane = lane
        if lane is not None:
            from ..framework.lane import LaneEntries
            self.entries = LaneEntries(lane)        # type: ignore[assignment]
        else:
            self.entries: dict[str, tuple] = {}
        self.store = LazyPodStore(self.entries)      # type: ignore[assignment]

    def ident(self, key: str) -> Optional[tuple]:
        e = self.entries.get(key)
        return e[1] if e is not None else None

    def _dispatch_native(self, typ: str, ev) -> None:
        idt = ev.ident()
        key = idt[0]
        if typ == "DELETED":
            old = self.entries.pop(key, None)
            self._call(self.on_event, "DELETED", ev, idt, old)
        else:
            old = self.entries.get(key)
            self.entries[key] = (ev, idt)
            self._call(self.on_event, "ADDED" if old is None else "MODIFIED", ev, idt, old)

    async def _list(self) -> None:
        fresh: dict[str, tuple] = {}
        rv = "0"
        consistent = self._consistent_relist
        self._consistent_relist = False
        async for evs, rv in self.client.list_pods_native(resource_version="" if consistent else "0",
                                                          limit=self.page_size if consistent else 0,
                                                          field_selector=self.field_selector):
            for ev in evs:
                idt = ev.ident()
                fresh[idt[0]] = (ev, idt)
        for key in ([] if self.lane is not None else [k for k in self.entries if k not in fresh]):
            old = self.entries.pop(key)
            self._call(self.on_event, "DELETED", old[0], old[1], old)
        if self.lane is not None:
            # the lane diffs the list against its store; Python sees what it forwards
            for typ, ev, old in self.lane.relist([e[0] for e in fresh.values()]):
                self._call(self.on_event, typ, ev, ev.ident(), (old, old.ident()) if old is not None else None)
            self.resource_version = rv
            self.relists += 1
            return
        for key, e in fresh.items():
            old = self.entries.get(key)
            self.entries[key] = e
            if old is None:
                self._call(self.on_event, "ADDED", e[0], e[1], None)
            elif old[0].rv != e[0].rv:
                self._call(self.on_event, "MODIFIED", e[0], e[1], old)
        self.resource_version = rv
        self.relists += 1

    async def _watch_once(self) -> None:
        loop = asyncio.get_event_loop()
        done = loop.create_future()
        err: list = []

        def on_events(evs) -> None:
            if err:
                return
            # _dispatch_native + _call inlined: this loop runs three times per scheduled pod
            entries, handler = self.entries, self.on_event
            for typ, rv, payload, idt in evs:
                if typ == "BOOKMARK":
                    if rv:
                        self.resource_version = rv
                        self.bookmarks += 1
                    continue
                if typ == "ERROR":
                    try:
                        st = json.loads(payload) if payload else {}
                    except ValueError:
                        st = {}
                    err.append(ApiError(int(st.get("code", 500)), st.get("reason", "Error"), st.get("message", "")))
                    self.client.native.cancel(wid)
                    if not done.done():
                        done.set_result((0, b""))
                    return
                key = idt[0]
                try:
                    if typ == "DELETED":
                        handler("DELETED", payload, idt, entries.pop(key, None))
                    else:
                        old = entries.get(key)
                        entries[key] = (payload, idt)
                        handler("ADDED" if old is None else "MODIFIED", payload, idt, old)
                except Exception:  # noqa: BLE001 - isolate handlers: log, count, keep the stream
                    self.handler_errors += 1
                    log.exception("informer %s: event handler failed", self.res)
                if rv:
                    self.resource_version = rv

        def on_end(status: int, body: bytes) -> None:
            h = handle[0]
            if h is not None and h.last_rv and self.lane is not None:
                self.resource_version = h.last_rv    # events went to the lane: resume after them
            if not done.done():
                done.set_result((status, body))

        handle: list = [None]
        wid = self.client.watch_native("pods", self.resource_version, on_events, on_end, self.field_selector,
                                       pods=True)
        handle[0] = self.client.native._watches.get(wid)
        try:
            status, body = await done
        except asyncio.CancelledError:
            self.client.native.cancel(wid)
            raise
        if err:
            raise err[0]
        if status in (0, 200):
            return
        from .native import api_error
        if status == 401:
            self.client._refresh_token(force=True)
        raise api_error(status, body)
