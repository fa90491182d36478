"""HTTPS server for the admission webhook: ``POST /validate``, ``POST /mutate``,
``GET /healthz`` (the apiserver only calls webhooks over TLS; tests may run plain HTTP)."""
from __future__ import annotations

import json
import logging
from typing import Optional

from aiohttp import web

from .admission import AdmissionPolicy, review

log = logging.getLogger("yoda.webhook")


class WebhookServer:
    def __init__(self, host: str = "0.0.0.0", port: int = 9443, policy: Optional[AdmissionPolicy] = None,
                 ssl_context=None) -> None:
        self.host, self.port = host, port
        self.policy = policy or AdmissionPolicy()
        self.ssl_context = ssl_context
        self.app = web.Application(client_max_size=8 << 20)
        self.app.router.add_post("/validate", self._handler(mutate=False))
        self.app.router.add_post("/mutate", self._handler(mutate=True))
        self.app.router.add_get("/healthz", self._health)
        self._runner: Optional[web.AppRunner] = None
        self.reviewed = 0
        self.rejected = 0

    @staticmethod
    async def _health(_r: web.Request) -> web.Response:
        return web.Response(text="ok")

    def _handler(self, mutate: bool):
        async def h(request: web.Request) -> web.Response:
            try:
                body = await request.json()
            except (ValueError, json.JSONDecodeError):
                return web.Response(status=400, text="AdmissionReview JSON expected")
            out = review(body, mutate, self.policy)
            self.reviewed += 1
            if not out["response"]["allowed"]:
                self.rejected += 1
                log.info("rejected pod %s: %s", ((body.get("request") or {}).get("name") or ""),
                         out["response"]["status"]["message"])
            return web.json_response(out)
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
