"""Health / metrics / configz / debug HTTP endpoints of the scheduler process (the
kube-scheduler serving surface the reference inherits)."""
from __future__ import annotations

import json
from typing import Callable, Optional

from aiohttp import web


class StatusServer:
    def __init__(self, host: str, port: int, metrics_render: Callable[[], bytes],
                 healthy: Callable[[], bool] = lambda: True, configz: Optional[Callable[[], dict]] = None,
                 debug: Optional[Callable[[], dict]] = None, trace: Optional[Callable[[], dict]] = None,
                 profiling: bool = False, resources: Optional[Callable[[], bytes]] = None,
                 cache: Optional[Callable[[], dict]] = None, ssl_context=None) -> None:
        self.ssl_context = ssl_context
        self.host, self.port = host, port
        self.app = web.Application()
        self.app.router.add_get("/healthz", self._health(healthy))
        self.app.router.add_get("/livez", self._health(healthy))
        self.app.router.add_get("/readyz", self._health(healthy))
        async def metrics(_r):
            return web.Response(body=metrics_render(), content_type="text/plain", charset="utf-8")

        self.app.router.add_get("/metrics", metrics)
        if resources is not None:
            async def metrics_resources(_r):
                return web.Response(body=resources(), content_type="text/plain", charset="utf-8")

            self.app.router.add_get("/metrics/resources", metrics_resources)
        for path, fn in (("/configz", configz), ("/debug/yoda", debug), ("/debug/trace", trace),
                         ("/debug/cache", cache)):
            if fn is not None:
                self.app.router.add_get(path, self._json(fn))
        if profiling:
            from . import pprof

            async def profile(r):
                q = r.query
                txt = await pprof.profile_text(float(q.get("seconds", 5)), q.get("sort", "cumulative"),
                                               int(q.get("limit", 60)))
                return web.Response(text=txt)

            async def goroutine(_r):
                return web.Response(text=pprof.goroutine_text())

            async def heap(_r):
                return web.json_response(pprof.heap_summary(), dumps=_dumps)

            self.app.router.add_get("/debug/pprof/profile", profile)
            self.app.router.add_get("/debug/pprof/goroutine", goroutine)
            self.app.router.add_get("/debug/pprof/heap", heap)
        self._runner: Optional[web.AppRunner] = None

    @staticmethod
    def _json(fn):
        async def h(_r):
            return web.json_response(fn(), dumps=_dumps)
        return h

    @staticmethod
    def _health(fn):
        async def h(_r):
            return web.Response(text="ok") if fn() else web.Response(text="unhealthy", status=500)
        return h

    async def start(self) -> int:
        self._runner = web.AppRunner(self.app)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port, ssl_context=self.ssl_context)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]   # type: ignore[union-attr]
        return self.port

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()


def _dumps(o) -> str:
    return json.dumps(o, default=lambda x: getattr(x, "__dict__", str(x)))
