"""asyncio front of the native Kubernetes transport (``native/kube``, module ``_yoda_kube``).

The C++ side runs one epoll I/O thread: pipelined keep-alive request connections, one
connection per watch, chunked decoding, JSON parsing and the pod projection. This module
connects it to the event loop: the transport's completion eventfd is registered with
``loop.add_reader`` and every wake-up drains *all* finished requests and decoded watch
events in one call, dispatching them to callbacks (no task or future per bind on the hot
path). Replaces the reference process's two client-go stacks on the hot path
(``/root/reference/pkg/yoda/scheduler.go:53-73``).
"""
from __future__ import annotations

import asyncio
import collections
import json
import logging
import os
from typing import Callable, Optional
from urllib.parse import urlsplit

from .errors import ApiError

log = logging.getLogger("yoda.native")

_mod = None


def module():
    """The compiled ``_yoda_kube`` extension (raises ImportError when it is not built)."""
    global _mod
    if _mod is None:
        from ..ops.native import load_native
        _mod = load_native("kube", "yoda_scheduler_amd._native._yoda_kube")
    return _mod


def available() -> bool:
    try:
        module()
        return True
    except ImportError:
        return False


def api_error(status: int, body: bytes) -> Exception:
    """HTTP status / transport failure → the exception the Python client raises."""
    if status < 0:
        msg = body.decode("utf-8", "replace")
        return asyncio.TimeoutError(msg) if status == -2 else ConnectionError(msg)
    try:
        st = json.loads(body) if body else {}
    except ValueError:
        st = {}
    if not isinstance(st, dict):
        st = {}
    return ApiError(status, st.get("reason", "Error"), st.get("message", body[:300].decode("utf-8", "replace")))


class WatchHandle:
    """One native watch stream: ``on_events(list)`` per decoded batch, ``on_end(status, body)``
    once when the stream ends (server timeout, error status, connection loss)."""

    __slots__ = ("id", "on_events", "on_end", "last_rv")

    def __init__(self, wid: int, on_events: Callable, on_end: Callable) -> None:
        self.id, self.on_events, self.on_end = wid, on_events, on_end
        self.last_rv = ""        # set at the end: the stream's last event version (pod-sink streams)


class NativeTransport:
    def __init__(self, config, conns: int = 8, max_inflight: int = 64, qps: float = 0.0, burst: int = 0) -> None:
        u = urlsplit(config.server)
        tls = u.scheme == "https"
        host = u.hostname or "127.0.0.1"
        port = u.port or (443 if tls else 80)
        self.config = config
        self.t = module().Transport(host, port, tls, (u.path or "").rstrip("/"), config.ca_file or "",
                                    config.cert_file or "", config.key_file or "", bool(config.insecure),
                                    config.token or "", conns, max_inflight, float(qps), int(burst))
        self._cbs: dict[int, Callable] = {}
        self._watches: dict[int, WatchHandle] = {}
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self.callback_errors = 0
        # completions handed over by the C++ thread but not yet dispatched: at most
        # DRAIN_BUDGET watch events run per loop turn, so a 5000-pod burst's ADDED events do
        # not hold the scheduling loop off for tens of ms (it takes a batch between chunks)
        self._backlog: collections.deque = collections.deque()
        self._continue_pending = False

    # ------------------------------------------------------------------ loop wiring
    def _attach(self) -> None:
        loop = asyncio.get_event_loop()
        if self._loop is loop:
            return
        if self._loop is not None and not self._loop.is_closed():
            self._loop.remove_reader(self.t.fileno())
        self._loop = loop
        loop.add_reader(self.t.fileno(), self._drain)

    # YODA_DRAIN_BUDGET: A/B knob for the per-turn event budget
    DRAIN_BUDGET = int(os.environ.get("YODA_DRAIN_BUDGET", "512"))

    def _drain(self) -> None:
        self._backlog.extend(self.t.drain())
        self._run_backlog()

    def _continue(self) -> None:
        self._continue_pending = False
        self._run_backlog()

    def _run_backlog(self) -> None:
        bl, budget = self._backlog, self.DRAIN_BUDGET
        while bl and budget > 0:
            c = bl[0]
            kind = c[0]
            if kind == 1 and len(c[2]) > budget:
                # split a large event batch: this turn's share now, the rest stays first in line
                evs = c[2]
                bl[0] = (1, c[1], evs[budget:])
                c = (1, c[1], evs[:budget])
                budget = 0
            else:
                bl.popleft()
                budget -= len(c[2]) if kind == 1 else 1
            try:
                if kind == 0:
                    cb = self._cbs.pop(c[1], None)
                    if cb is not None:
                        cb(c[2], c[3])
                elif kind == 1:
                    h = self._watches.get(c[1])
                    if h is not None:
                        h.on_events(c[2])
                else:
                    h = self._watches.pop(c[1], None)
                    if h is not None:
                        h.last_rv = c[4] if len(c) > 4 else ""
                        h.on_end(c[2], c[3])
            except Exception:  # noqa: BLE001 - one failing callback must not stall the rest
                self.callback_errors += 1
                log.exception("native transport callback failed")
        if bl and not self._continue_pending and self._loop is not None:
            self._continue_pending = True
            self._loop.call_soon(self._continue)

    # ------------------------------------------------------------------ verbs
    def submit(self, method: str, path: str, body: bytes, cb: Callable[[int, bytes], None],
               content_type: str = "", limited: bool = True, timeout: float = 0.0) -> int:
        self._attach()
        rid = self.t.request(method, path, body, content_type, limited, timeout)
        self._cbs[rid] = cb
        return rid

    async def request(self, method: str, path: str, body: bytes = b"", content_type: str = "",
                      limited: bool = True, timeout: float = 0.0) -> tuple[int, bytes]:
        fut = asyncio.get_event_loop().create_future()

        def done(status: int, data: bytes) -> None:
            if not fut.done():
                fut.set_result((status, data))
        self.submit(method, path, body, done, content_type, limited, timeout)
        return await fut

    def bind(self, namespace: str, name: str, uid: str, node: str, annotations: list,
             cb: Callable[[int, bytes], None], timeout: float = 0.0) -> int:
        """Binding POST (rate-limited by the transport's token bucket); ``cb(status, body)``
        runs on the event loop when the apiserver answers."""
        self._attach()
        rid = self.t.bind(namespace, name, uid, node, annotations, timeout)
        self._cbs[rid] = cb
        return rid

    def bind_many(self, binds: list, cbs: list, timeout: float = 0.0) -> None:
        """A run of Binding POSTs — ``binds[k] = (namespace, name, uid, node, annotations)``,
        answered through ``cbs[k](status, body)`` — handed to the I/O thread in one call (one
        lock and one wake-up for the run instead of one per pod)."""
        if not binds:
            return
        self._attach()
        first = self.t.bind_many(binds, timeout)
        cb_map = self._cbs
        for k, cb in enumerate(cbs):
            cb_map[first + k] = cb

    def watch(self, path: str, pods: bool, on_events: Callable, on_end: Callable, idle_timeout: float = 0.0) -> int:
        """``idle_timeout``: end the stream (status -1) if nothing arrives for that long — a
        black-holed connection never delivers the server's own ``timeoutSeconds`` end.
        ``on_end`` may take a third argument: the resourceVersion of the stream's last event
        (the only way to learn it when a native pod lane consumed the events)."""
        self._attach()
        wid = self.t.watch(path, pods, float(idle_timeout))
        h = WatchHandle(wid, on_events, on_end)
        self._watches[wid] = h
        return wid

    def cancel(self, wid: int) -> None:
        self._watches.pop(wid, None)
        self.t.cancel(wid)

    def set_token(self, token: str) -> None:
        self.t.set_token(token or "")

    def set_rate(self, qps: float, burst: int) -> None:
        self.t.set_rate(float(qps), int(burst))

    def stats(self) -> dict:
        return self.t.stats()

    def close(self) -> None:
        if self._loop is not None and not self._loop.is_closed():
            try:
                self._loop.remove_reader(self.t.fileno())
            except Exception:  # noqa: BLE001
                pass
        self.t.close()
        # anything still pending fails like a dropped connection
        err_cbs, self._cbs = self._cbs, {}
        for cb in err_cbs.values():
            try:
                cb(-1, b"transport closed")
            except Exception:  # noqa: BLE001
                pass
        self._watches.clear()
