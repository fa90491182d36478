"""Minimal async Kubernetes REST client (aiohttp): list / watch / get / create / update /
status / merge-patch / delete / pods/binding.

Replaces the two client stacks of the reference process (kube-scheduler's informers and
the controller-runtime manager, ``pkg/yoda/scheduler.go:53-73``) with one client shared by
every informer, the binder, the event recorder and leader election. Auth: in-cluster
service-account token + CA (``ctrl.GetConfigOrDie`` equivalent) or a kubeconfig
(token / client certificate / insecure-skip-tls-verify).
"""
from __future__ import annotations

import base64
import asyncio
import json
import os
import ssl
import tempfile
from typing import AsyncIterator, Optional

import aiohttp
import yaml

from .errors import ApiError
from .resources import resource

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class KubeConfig:
    def __init__(self, server: str, token: Optional[str] = None, ca_file: Optional[str] = None,
                 cert_file: Optional[str] = None, key_file: Optional[str] = None, insecure: bool = False) -> None:
        self.server = server.rstrip("/")
        self.token = token
        self.ca_file = ca_file
        self.cert_file = cert_file
        self.key_file = key_file
        self.insecure = insecure

    @classmethod
    def in_cluster(cls) -> "KubeConfig":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if not host or not port:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
        with open(os.path.join(SA_DIR, "token")) as f:
            token = f.read().strip()
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        return cls(f"https://{host}:{port}", token=token, ca_file=os.path.join(SA_DIR, "ca.crt"))

    @classmethod
    def from_kubeconfig(cls, path: str, context: Optional[str] = None) -> "KubeConfig":
        with open(os.path.expanduser(path)) as f:
            doc = yaml.safe_load(f) or {}
        ctx_name = context or doc.get("current-context")
        ctx = next((c["context"] for c in doc.get("contexts") or [] if c.get("name") == ctx_name), None)
        if ctx is None:
            raise ValueError(f"{path}: context {ctx_name!r} not found")
        cl = next(c["cluster"] for c in doc.get("clusters") or [] if c.get("name") == ctx.get("cluster"))
        user = next((u.get("user") or {} for u in doc.get("users") or [] if u.get("name") == ctx.get("user")), {})

        def materialise(data_key: str, file_key: str, obj: dict) -> Optional[str]:
            if obj.get(file_key):
                return obj[file_key]
            if obj.get(data_key):
                fd, p = tempfile.mkstemp(prefix="yoda-kc-")
                with os.fdopen(fd, "wb") as out:
                    out.write(base64.b64decode(obj[data_key]))
                return p
            return None

        return cls(cl["server"], token=user.get("token"),
                   ca_file=materialise("certificate-authority-data", "certificate-authority", cl),
                   cert_file=materialise("client-certificate-data", "client-certificate", user),
                   key_file=materialise("client-key-data", "client-key", user),
                   insecure=bool(cl.get("insecure-skip-tls-verify", False)))

    @classmethod
    def load(cls, kubeconfig: str = "", master: str = "") -> "KubeConfig":
        """--kubeconfig / --master / $KUBECONFIG / in-cluster, like client-go's loader."""
        if master and not kubeconfig:
            return cls(master)
        path = kubeconfig or os.environ.get("KUBECONFIG", "")
        if path:
            kc = cls.from_kubeconfig(path)
            if master:
                kc.server = master.rstrip("/")
            return kc
        return cls.in_cluster()


class KubeClient:
    def __init__(self, config: KubeConfig, timeout: float = 30.0, fast_bind: bool = True) -> None:
        """``fast_bind``: binding POSTs go through the pipelined keep-alive client in
        :mod:`.fastbind` (≈5× less scheduler CPU per bind than aiohttp); every other call
        uses aiohttp."""
        self.config = config
        self.timeout = timeout
        self._session: Optional[aiohttp.ClientSession] = None
        self.fast_bind = fast_bind
        self._binder = None

    def _ssl(self):
        c = self.config
        if not c.server.startswith("https"):
            return None
        if c.insecure:
            return False
        ctx = ssl.create_default_context(cafile=c.ca_file) if c.ca_file else ssl.create_default_context()
        if c.cert_file and c.key_file:
            ctx.load_cert_chain(c.cert_file, c.key_file)
        return ctx

    async def session(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            headers = {"Accept": "application/json", "User-Agent": "yoda-scheduler/0.1 (MI355X)"}
            if self.config.token:
                headers["Authorization"] = f"Bearer {self.config.token}"
            conn = aiohttp.TCPConnector(ssl=self._ssl(), limit=512, keepalive_timeout=60)
            self._session = aiohttp.ClientSession(headers=headers, connector=conn)
        return self._session

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()
        if self._binder is not None:
            await self._binder.close()
            self._binder = None

    def _binder_ssl(self):
        ctx = self._ssl()
        if ctx is False:            # insecure-skip-tls-verify
            ctx = ssl.create_default_context()
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        return ctx

    def _url(self, res: str, namespace: Optional[str] = None, name: Optional[str] = None,
             sub: Optional[str] = None) -> str:
        return self.config.server + resource(res).path(namespace, name, sub)

    async def _req(self, method: str, url: str, body=None, content_type: str = "application/json",
                   params: Optional[dict] = None) -> dict:
        s = await self.session()
        data = None if body is None else json.dumps(body)
        async with s.request(method, url, data=data, params=params, headers={"Content-Type": content_type},
                             timeout=aiohttp.ClientTimeout(total=self.timeout)) as r:
            text = await r.text()
            if r.status >= 400:
                try:
                    st = json.loads(text)
                except ValueError:
                    st = {}
                raise ApiError(r.status, st.get("reason", r.reason or "Error"), st.get("message", text[:300]))
            return json.loads(text) if text else {}

    # ------------------------------------------------------------------ verbs
    async def list(self, res: str, namespace: Optional[str] = None, resource_version: Optional[str] = None,
                   limit: int = 0, field_selector: Optional[str] = None) -> tuple[list[dict], str]:
        """List (client-go pager semantics): ``resource_version="0"`` may be served from the
        apiserver's watch cache (which ignores ``limit``); otherwise a consistent read in
        ``limit``-sized chunks, following ``continue`` tokens. Returns (items, list RV)."""
        params: dict = {}
        if resource_version is not None:
            params["resourceVersion"] = resource_version
        if limit:
            params["limit"] = str(limit)
        if field_selector:
            params["fieldSelector"] = field_selector
        items: list = []
        while True:
            out = await self._req("GET", self._url(res, namespace), params=params or None)
            items.extend(out.get("items") or [])
            meta = out.get("metadata") or {}
            cont = meta.get("continue")
            if not cont:
                return items, meta.get("resourceVersion", "0")
            params = {"limit": str(limit), "continue": cont} if limit else {"continue": cont}
            if field_selector:
                params["fieldSelector"] = field_selector

    async def watch(self, res: str, resource_version: str, field_selector: Optional[str] = None,
                    timeout_s: int = 300) -> AsyncIterator[tuple[str, dict]]:
        s = await self.session()
        params = {"watch": "1", "resourceVersion": resource_version or "0", "allowWatchBookmarks": "true",
                  "timeoutSeconds": str(timeout_s)}
        if field_selector:
            params["fieldSelector"] = field_selector
        async with s.get(self._url(res), params=params,
                         timeout=aiohttp.ClientTimeout(total=None, sock_read=timeout_s + 30)) as r:
            if r.status >= 400:
                text = await r.text()
                raise ApiError(r.status, r.reason or "Error", text[:300])
            buf = b""
            async for chunk in r.content.iter_any():
                buf += chunk
                if b"\n" not in chunk:
                    continue
                *lines, buf = buf.split(b"\n")     # one split per chunk, not per event
                for line in lines:
                    if not line.strip():
                        continue
                    ev = json.loads(line)
                    typ, obj = ev.get("type"), ev.get("object") or {}
                    if typ == "ERROR":
                        raise ApiError(int(obj.get("code", 500)), obj.get("reason", "Error"), obj.get("message", ""))
                    yield typ, obj          # BOOKMARK too: the informer advances its RV

    async def get(self, res: str, name: str, namespace: Optional[str] = None) -> dict:
        return await self._req("GET", self._url(res, namespace, name))

    async def create(self, res: str, obj: dict, namespace: Optional[str] = None) -> dict:
        ns = namespace or (obj.get("metadata") or {}).get("namespace") or ("default" if resource(res).namespaced else None)
        return await self._req("POST", self._url(res, ns), obj)

    async def update(self, res: str, obj: dict, namespace: Optional[str] = None) -> dict:
        m = obj.get("metadata") or {}
        ns = namespace or m.get("namespace")
        return await self._req("PUT", self._url(res, ns, m["name"]), obj)

    async def update_status(self, res: str, obj: dict, namespace: Optional[str] = None) -> dict:
        m = obj.get("metadata") or {}
        ns = namespace or m.get("namespace")
        return await self._req("PUT", self._url(res, ns, m["name"], "status"), obj)

    async def patch(self, res: str, name: str, patch: dict, namespace: Optional[str] = None) -> dict:
        sub = "status" if res == "pods" and set(patch) == {"status"} else None
        return await self._req("PATCH", self._url(res, namespace, name, sub), patch,
                               content_type="application/merge-patch+json")

    async def delete(self, res: str, name: str, namespace: Optional[str] = None) -> dict:
        return await self._req("DELETE", self._url(res, namespace, name))

    async def bind(self, namespace: str, name: str, uid: str, node: str, annotations: Optional[dict] = None) -> None:
        if self.fast_bind:
            if self._binder is None:
                from .fastbind import FastBinder
                self._binder = FastBinder(self.config.server, self.config.token, self._binder_ssl(),
                                          timeout=self.timeout)
            await self._binder.bind(namespace, name, uid, node, annotations)
            return
        body = {"apiVersion": "v1", "kind": "Binding",
                "metadata": {"name": name, "namespace": namespace, "uid": uid, "annotations": dict(annotations or {})},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        await self._req("POST", self._url("pods", namespace, name, "binding"), body)
