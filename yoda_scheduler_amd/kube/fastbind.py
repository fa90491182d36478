"""Lean HTTP/1.1 client for the scheduler's hottest API call: ``POST pods/{name}/binding``.

A 1000-pod burst is 1000 binding POSTs; through aiohttp's general-purpose client each one
costs ≈100 µs of scheduler CPU (request/response objects, yarl URLs, header multidicts),
which caps HTTP-transport throughput long before the apiserver does. Here a small pool of
keep-alive connections (TLS when the apiserver is HTTPS) carries *pipelined* requests: a
bind is one pre-formatted write and one future, and a reader task per connection parses
responses in order (status line, headers, Content-Length or chunked body). Requests on a
connection are answered in order (HTTP/1.1), so the FIFO of futures is the whole protocol.

Everything else (list/watch/get/patch/events/leases) stays on aiohttp.
"""
from __future__ import annotations

import asyncio
import collections
import json
import ssl as _ssl
from typing import Optional
from urllib.parse import urlsplit

from .errors import ApiError


class _Conn:
    def __init__(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        self.r, self.w = reader, writer
        self.pending: collections.deque = collections.deque()
        self.closed = False
        self.task = asyncio.get_event_loop().create_task(self._read_loop())

    async def _read_body(self, headers: dict) -> bytes:
        if "content-length" in headers:
            n = int(headers["content-length"])
            return await self.r.readexactly(n) if n else b""
        if headers.get("transfer-encoding", "").lower() == "chunked":
            out = bytearray()
            while True:
                size = int((await self.r.readline()).split(b";", 1)[0].strip() or b"0", 16)
                if size == 0:
                    while (await self.r.readline()) not in (b"\r\n", b"\n", b""):
                        pass            # trailers
                    return bytes(out)
                out += await self.r.readexactly(size)
                await self.r.readline()
        return b""

    async def _read_loop(self) -> None:
        err: Exception = ConnectionError("connection closed")
        try:
            while True:
                line = await self.r.readline()
                if not line:
                    break
                parts = line.split(None, 2)
                status = int(parts[1])
                headers = {}
                while True:
                    h = await self.r.readline()
                    if h in (b"\r\n", b"\n", b""):
                        break
                    k, _, v = h.decode("latin-1").partition(":")
                    headers[k.strip().lower()] = v.strip()
                body = await self._read_body(headers)
                if self.pending:
                    fut = self.pending.popleft()
                    if not fut.done():
                        fut.set_result((status, body))
                if headers.get("connection", "").lower() == "close":
                    break
        except (asyncio.IncompleteReadError, ConnectionError, OSError, ValueError, IndexError) as e:
            err = e
        except asyncio.CancelledError:
            err = ConnectionError("client closed")
        self.closed = True
        while self.pending:
            fut = self.pending.popleft()
            if not fut.done():
                fut.set_exception(err)
        try:
            self.w.close()
        except Exception:  # noqa: BLE001
            pass


def _expire(fut: asyncio.Future) -> None:
    if not fut.done():
        fut.set_exception(asyncio.TimeoutError("binding request timed out"))


class FastBinder:
    """Pipelined binding POSTs over ``conns`` keep-alive connections (``max_inflight`` per
    connection). Errors surface as :class:`ApiError` (HTTP status) or ``ConnectionError``
    (the scheduler treats both as a failed bind: forget + requeue)."""

    def __init__(self, server: str, token: Optional[str] = None, ssl_context: Optional[_ssl.SSLContext] = None,
                 conns: int = 16, max_inflight: int = 64, timeout: Optional[float] = None) -> None:
        self.timeout = timeout
        u = urlsplit(server)
        self.tls = u.scheme == "https"
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if self.tls else 80)
        self.prefix = (u.path or "").rstrip("/")
        self.ssl = ssl_context if self.tls else None
        self.n = max(1, conns)
        self.max_inflight = max(1, max_inflight)
        host_hdr = self.host if u.port is None else f"{self.host}:{self.port}"
        auth = f"Authorization: Bearer {token}\r\n" if token else ""
        self._head = (f"Host: {host_hdr}\r\nUser-Agent: yoda-scheduler\r\nAccept: application/json\r\n"
                      f"Content-Type: application/json\r\n{auth}")
        self._conns: list[Optional[_Conn]] = [None] * self.n
        self._rr = 0
        self._lock = asyncio.Lock()

    async def _conn(self, i: int) -> _Conn:
        c = self._conns[i]
        if c is not None and not c.closed:
            return c
        async with self._lock:
            c = self._conns[i]
            if c is None or c.closed:
                r, w = await asyncio.open_connection(self.host, self.port, ssl=self.ssl,
                                                     server_hostname=self.host if self.ssl else None)
                c = self._conns[i] = _Conn(r, w)
        return c

    async def post(self, path: str, body: dict) -> tuple[int, bytes]:
        data = json.dumps(body, separators=(",", ":")).encode()
        req = (f"POST {self.prefix}{path} HTTP/1.1\r\n{self._head}Content-Length: {len(data)}\r\n\r\n").encode() + data
        # least-loaded of two round-robin candidates keeps pipelines short under skew
        i = self._rr % self.n
        self._rr += 1
        c = await self._conn(i)
        if len(c.pending) >= self.max_inflight and self.n > 1:
            j = (i + 1) % self.n
            c2 = await self._conn(j)
            if len(c2.pending) < len(c.pending):
                c = c2
        loop = asyncio.get_event_loop()
        fut = loop.create_future()
        c.pending.append(fut)
        c.w.write(req)
        if self.timeout is None:
            return await fut
        # the timer fails the response future itself (it stays queued, so the pipeline's
        # request/response pairing holds when the late answer arrives); no wait_for, whose
        # Python < 3.12 race could swallow the caller's cancellation
        h = loop.call_later(self.timeout, _expire, fut)
        try:
            return await fut
        finally:
            h.cancel()

    async def bind(self, namespace: str, name: str, uid: str, node: str, annotations: Optional[dict] = None) -> None:
        body = {"apiVersion": "v1", "kind": "Binding",
                "metadata": {"name": name, "namespace": namespace, "uid": uid, "annotations": dict(annotations or {})},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        status, raw = await self.post(f"/api/v1/namespaces/{namespace}/pods/{name}/binding", body)
        if status >= 400:
            try:
                st = json.loads(raw)
            except ValueError:
                st = {}
            raise ApiError(status, st.get("reason", "Error"), st.get("message", raw[:300].decode("utf-8", "replace")))

    async def close(self) -> None:
        for c in self._conns:
            if c is not None:
                c.task.cancel()
                try:
                    c.w.close()
                except Exception:  # noqa: BLE001
                    pass
        await asyncio.gather(*(c.task for c in self._conns if c is not None), return_exceptions=True)
        self._conns = [None] * self.n
