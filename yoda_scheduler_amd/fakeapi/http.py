"""HTTP front of the fake apiserver: the subset of the Kubernetes REST API the scheduler,
sniffer and leader election use, served by aiohttp so the real :class:`KubeClient` (and
``kubectl``-style tools) can be exercised end to end without a cluster, including from
other processes (multi-process / HA tests).
"""
from __future__ import annotations

import asyncio
import json
import os
import re
from typing import Optional

from aiohttp import web

from ..kube.errors import ApiError
from ..kube.resources import BY_PATH, RESOURCES
from .server import FakeApiServer

_PATH = re.compile(
    r"^/(?:api/v1|apis/(?P<group>[^/]+)/(?P<version>[^/]+))"
    r"(?:/namespaces/(?P<ns>[^/]+))?/(?P<res>[^/]+)(?:/(?P<name>[^/]+))?(?:/(?P<sub>[^/]+))?$")


def _resolve(path: str):
    m = _PATH.match(path)
    if not m:
        return None
    res = BY_PATH.get((m.group("group") or "", m.group("res")))
    if res is None:
        return None
    return res, m.group("ns"), m.group("name"), m.group("sub")


def _status(e: ApiError) -> web.Response:
    return web.json_response(e.status_obj(), status=e.code)


class FakeApiHttp:
    def __init__(self, server: Optional[FakeApiServer] = None, host: str = "127.0.0.1", port: int = 0,
                 ssl_context=None, token: Optional[str] = None, bench: bool = False) -> None:
        """``ssl_context`` serves HTTPS (as a real apiserver does); ``token`` makes every
        API route require ``Authorization: Bearer <token>`` (401 otherwise)."""
        self.server = server or FakeApiServer()
        self.host = host
        self.port = port
        self.ssl_context = ssl_context
        self.token = token
        self._runner: Optional[web.AppRunner] = None
        self.app = web.Application()
        async def healthz(_r):
            return web.Response(text="ok")

        async def version(_r):
            return web.json_response({"major": "1", "minor": "20", "gitVersion": "v1.20.0-yoda-fake"})

        self.app.router.add_get("/healthz", healthz)
        self.app.router.add_get("/version", version)
        if bench:
            # burst driver for the HTTP transport of bench.py: pods are created and the
            # latencies measured here, on the apiserver's clock, like the in-process harness
            self.app.router.add_post("/debug/bench/burst", self._bench_burst)
            self.app.router.add_get("/debug/bench/status", self._bench_status)
            self.app.router.add_post("/debug/bench/reset", self._bench_reset)
            self.bench_workload = None
            self.bench_keys: list = []
        self.app.router.add_route("*", "/{tail:.*}", self.dispatch)

    @property
    def url(self) -> str:
        return f"{'https' if self.ssl_context else 'http'}://{self.host}:{self.port}"

    async def start(self) -> str:
        self._runner = web.AppRunner(self.app)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port, ssl_context=self.ssl_context)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]   # type: ignore[union-attr]
        return self.url

    async def _bench_burst(self, req: web.Request) -> web.Response:
        from ..bench.workloads import pod_object
        body = await req.json()
        w = self.bench_workload
        tag = body.get("tag", "b")
        self.server.reset_logs()
        for i, lab in enumerate(w.pods):
            o = self.server.create("pods", pod_object(i, lab, w.scheduler_name, prefix=tag))
            self.bench_keys.append((o["metadata"]["name"], o["metadata"].get("namespace", "default")))
            if i % 64 == 63:
                await asyncio.sleep(0)
        return web.json_response({"n": len(w.pods)})

    async def _bench_status(self, req: web.Request) -> web.Response:
        s = self.server
        out = {"created": len(s.create_log), "bound": len(s.bind_log)}
        if req.query.get("full"):
            out["latencies"] = s.latencies()
            t0 = min(s.create_log.values()) if s.create_log else 0.0
            out["elapsed"] = (max(s.bind_log.values()) - t0) if s.bind_log else 0.0
        return web.json_response(out)

    async def _bench_reset(self, _req: web.Request) -> web.Response:
        # the bursts' pods only: pods created through the API (a populated cluster) stay
        n = 0
        for name, ns in self.bench_keys:
            try:
                self.server.delete("pods", name, ns)
                n += 1
            except Exception:  # noqa: BLE001 - already gone (e.g. preempted)
                pass
        self.bench_keys.clear()
        self.server.reset_logs()
        return web.json_response({"deleted": n})

    async def stop(self) -> None:
        self.server.close_watches()
        if self._runner is not None:
            await self._runner.cleanup()

    async def dispatch(self, req: web.Request) -> web.StreamResponse:
        if self.token is not None and req.headers.get("Authorization") != f"Bearer {self.token}":
            return _status(ApiError(401, "Unauthorized", "Unauthorized"))
        r = _resolve(req.path)
        if r is None:
            return _status(ApiError(404, "NotFound", f"no route for {req.path}"))
        res, ns, name, sub = r
        s = self.server
        try:
            if req.method == "GET":
                if name is None:
                    fsel = req.query.get("fieldSelector") or None
                    if req.query.get("watch") in ("1", "true"):
                        return await self._watch(req, res, req.query.get("resourceVersion", "0"), fsel)
                    limit, cont = int(req.query.get("limit", "0") or 0), req.query.get("continue", "")
                    if limit or cont:
                        items, rv, nxt = s.list_page(res, ns, limit, cont, fsel)
                    else:
                        (items, rv), nxt = s.list(res, ns, fsel), ""
                    meta = {"resourceVersion": rv}
                    if nxt:
                        meta["continue"] = nxt
                    return web.json_response({"kind": RESOURCES[res].kind + "List", "apiVersion": RESOURCES[res].api_version,
                                              "metadata": meta, "items": items})
                return web.json_response(s.get(res, name, ns))
            body = await req.json() if req.can_read_body else {}
            if req.method == "POST":
                if sub == "binding" and res == "pods":
                    meta = body.get("metadata") or {}
                    s.bind(ns or "default", name, meta.get("uid", ""), (body.get("target") or {}).get("name", ""),
                           meta.get("annotations"))
                    return web.json_response({"kind": "Status", "status": "Success", "code": 201}, status=201)
                return web.json_response(s.create(res, body, ns), status=201)
            if req.method == "PUT":
                return web.json_response(s.update(res, body, ns, status_only=(sub == "status")))
            if req.method == "PATCH":
                strategic = "strategic-merge-patch" in (req.headers.get("Content-Type") or "")
                return web.json_response(s.patch(res, name, body, ns, strategic=strategic))
            if req.method == "DELETE":
                return web.json_response(s.delete(res, name, ns))
        except ApiError as e:
            return _status(e)
        return _status(ApiError(405, "MethodNotAllowed", req.method))

    async def _watch(self, req: web.Request, res: str, rv: str, fsel: Optional[str] = None) -> web.StreamResponse:
        try:
            w = self.server.watch(res, rv, fsel)
        except ApiError as e:
            resp = web.StreamResponse(status=200, headers={"Content-Type": "application/json"})
            await resp.prepare(req)
            await resp.write((json.dumps({"type": "ERROR", "object": e.status_obj()}) + "\n").encode())
            return resp
        resp = web.StreamResponse(status=200, headers={"Content-Type": "application/json",
                                                       "Transfer-Encoding": "chunked"})
        await resp.prepare(req)
        timeout = float(req.query.get("timeoutSeconds", "300"))
        try:
            while True:
                try:
                    ev = await asyncio.wait_for(w.get(), timeout)
                except asyncio.TimeoutError:
                    break
                if ev is None:
                    break
                typ, obj = ev
                await resp.write((json.dumps({"type": typ, "object": obj}) + "\n").encode())
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            w.close()
        return resp


async def serve_forever(host: str = "127.0.0.1", port: int = 8001, server: Optional[FakeApiServer] = None,
                        workload=None, port_file: str = "") -> None:
    api = FakeApiHttp(server, host, port, bench=workload is not None)
    api.bench_workload = workload
    url = await api.start()
    if port_file:
        with open(port_file + ".tmp", "w") as f:
            f.write(str(api.port))
        os.replace(port_file + ".tmp", port_file)
    print(f"fake apiserver listening on {url}", flush=True)
    while True:
        await asyncio.sleep(3600)
