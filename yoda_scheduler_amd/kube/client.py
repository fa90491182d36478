"""Async Kubernetes REST client: list / watch / get / create / update / status /
merge-patch / delete / pods/binding.

Replaces the two client stacks of the reference process (kube-scheduler's informers and
the controller-runtime manager, ``pkg/yoda/scheduler.go:53-73``) with one client shared by
every informer, the binder, the event recorder and leader election. Auth: in-cluster
service-account token + CA (``ctrl.GetConfigOrDie`` equivalent) or a kubeconfig
(token / client certificate / insecure-skip-tls-verify).

Two transports behind the same verbs: the native C++ transport (:mod:`.native`: epoll
I/O thread, pipelined keep-alive connections, watch decoding and pod projection off the
event loop) whenever ``_yoda_kube`` is built, else aiohttp. Like client-go's
``transport.NewCachedFileTokenSource`` a service-account token is re-read from its file
(projected tokens rotate; every minute and after any 401, which is retried once).
"""
from __future__ import annotations

import base64
import asyncio
import json
import logging
import os
import ssl
import tempfile
import time
from typing import AsyncIterator, Optional
from urllib.parse import urlencode

import aiohttp
import yaml

from .errors import ApiError
from .resources import resource

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"
# a native watch that delivered nothing (no event, no bookmark, no server-side end) for its
# timeoutSeconds plus this grace is taken as a black-holed connection and re-watched
WATCH_IDLE_GRACE_S = 30.0
TOKEN_REFRESH_S = 60.0          # client-go cachedTokenSource re-reads the file every minute
log = logging.getLogger("yoda.client")


class KubeConfig:
    def __init__(self, server: str, token: Optional[str] = None, ca_file: Optional[str] = None,
                 cert_file: Optional[str] = None, key_file: Optional[str] = None, insecure: bool = False,
                 token_file: Optional[str] = None) -> None:
        self.server = server.rstrip("/")
        self.token = token
        self.ca_file = ca_file
        self.cert_file = cert_file
        self.key_file = key_file
        self.insecure = insecure
        self.token_file = token_file          # re-read periodically (rotating projected tokens)
        self._token_read = time.monotonic()

    def current_token(self, force: bool = False) -> Optional[str]:
        """The bearer token, re-read from ``token_file`` at most every TOKEN_REFRESH_S
        (or now, with ``force``). A failed read keeps the previous token."""
        if self.token_file and (force or time.monotonic() - self._token_read >= TOKEN_REFRESH_S):
            self._token_read = time.monotonic()
            try:
                with open(self.token_file) as f:
                    tok = f.read().strip()
                if tok:
                    self.token = tok
            except OSError as e:
                log.warning("token file %s: %s", self.token_file, e)
        return self.token

    @classmethod
    def in_cluster(cls) -> "KubeConfig":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        if not host or not port:
            raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST unset)")
        token_file = os.path.join(SA_DIR, "token")
        with open(token_file) as f:
            token = f.read().strip()
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        return cls(f"https://{host}:{port}", token=token, ca_file=os.path.join(SA_DIR, "ca.crt"),
                   token_file=token_file)

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

        return cls(cl["server"], token=user.get("token"), token_file=user.get("tokenFile"),
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
    def __init__(self, config: KubeConfig, timeout: float = 30.0, fast_bind: bool = True,
                 native: str | bool = "auto", native_conns: int = 8) -> None:
        """``native``: ``"auto"`` uses the C++ transport when ``_yoda_kube`` is built,
        ``True`` requires it, ``False`` keeps every call on aiohttp (with ``fast_bind``:
        binding POSTs on the pipelined Python client of :mod:`.fastbind`)."""
        self.config = config
        self.timeout = timeout
        self._session: Optional[aiohttp.ClientSession] = None
        self.fast_bind = fast_bind
        self._binder = None
        self.native = None
        if native:
            from . import native as nat
            if native == "auto" and not nat.available():
                self.native = None
            else:
                self.native = nat.NativeTransport(config, conns=native_conns)
        self._token_seen = config.token
        self.retried_401 = 0

    def set_rate(self, qps: float, burst: int) -> None:
        """clientConnection QPS/burst: enforced by the native transport for the calls that
        pass ``limited=True`` (binds, status patches, deletes), like client-go's limiter."""
        if self.native is not None:
            self.native.set_rate(qps, burst)

    def _refresh_token(self, force: bool = False) -> None:
        tok = self.config.current_token(force)
        if tok != self._token_seen:
            self._token_seen = tok
            if self.native is not None:
                self.native.set_token(tok or "")
            if self._session is not None and not self._session.closed:
                # aiohttp bakes the header into the session: rebuild it on rotation
                old, self._session = self._session, None
                asyncio.get_event_loop().create_task(old.close())
            if self._binder is not None:
                old_b, self._binder = self._binder, None
                asyncio.get_event_loop().create_task(old_b.close())

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
        self._refresh_token()
        if self._session is None or self._session.closed:
            headers = {"Accept": "application/json", "User-Agent": "yoda-scheduler/0.2 (MI355X)"}
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
        if self.native is not None:
            self.native.close()
            self.native = None

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

    @staticmethod
    def _path(res: str, namespace: Optional[str] = None, name: Optional[str] = None,
              sub: Optional[str] = None, params: Optional[dict] = None) -> str:
        p = resource(res).path(namespace, name, sub)
        return p + "?" + urlencode(params) if params else p

    async def _req(self, method: str, res: str, namespace: Optional[str] = None, name: Optional[str] = None,
                   sub: Optional[str] = None, body=None, content_type: str = "application/json",
                   params: Optional[dict] = None, limited: bool = False, parse: bool = True) -> dict:
        for attempt in (0, 1):
            if self.native is not None:
                self._refresh_token()
                data = b"" if body is None else json.dumps(body, separators=(",", ":")).encode()
                status, raw = await self.native.request(method, self._path(res, namespace, name, sub, params), data,
                                                        content_type if body is not None else "", limited,
                                                        self.timeout)
                if status < 0:
                    from .native import api_error
                    raise api_error(status, raw)
                text = raw
            else:
                s = await self.session()
                data = None if body is None else json.dumps(body)
                async with s.request(method, self._url(res, namespace, name, sub), data=data, params=params,
                                     headers={"Content-Type": content_type},
                                     timeout=aiohttp.ClientTimeout(total=self.timeout)) as r:
                    text = await r.read()
                    status = r.status
            if status == 401 and attempt == 0 and self.config.token_file:
                self.retried_401 += 1
                self._refresh_token(force=True)      # rotated token: retry once with the new one
                continue
            if status >= 400:
                try:
                    st = json.loads(text)
                except ValueError:
                    st = {}
                if not isinstance(st, dict):
                    st = {}
                raise ApiError(status, st.get("reason", "Error"),
                               st.get("message", text[:300].decode("utf-8", "replace")))
            return json.loads(text) if text and parse else {}
        raise AssertionError("unreachable")

    # ------------------------------------------------------------------ verbs
    async def list(self, res: str, namespace: Optional[str] = None, resource_version: Optional[str] = None,
                   limit: int = 0, field_selector: Optional[str] = None) -> tuple[list[dict], str]:
        """List (client-go pager semantics): ``resource_version="0"`` may be served from the
        apiserver's watch cache (which ignores ``limit``); otherwise a consistent read in
        ``limit``-sized chunks, following ``continue`` tokens. Returns (items, list RV)."""
        items: list = []
        rv = "0"
        async for page, rv in self.list_pages(res, namespace, resource_version, limit, field_selector):
            items.extend(page)
        return items, rv

    def _list_params(self, resource_version, limit, field_selector, cont: str = "") -> dict:
        params: dict = {}
        if resource_version is not None and not cont:
            params["resourceVersion"] = resource_version
        if limit:
            params["limit"] = str(limit)
        if cont:
            params["continue"] = cont
        if field_selector:
            params["fieldSelector"] = field_selector
        return params

    async def list_pages(self, res: str, namespace: Optional[str] = None, resource_version: Optional[str] = None,
                         limit: int = 0, field_selector: Optional[str] = None):
        """Yields (items, list RV) page by page."""
        cont = ""
        while True:
            out = await self._req("GET", res, namespace,
                                  params=self._list_params(resource_version, limit, field_selector, cont) or None)
            meta = out.get("metadata") or {}
            yield out.get("items") or [], meta.get("resourceVersion", "0")
            cont = meta.get("continue") or ""
            if not cont:
                return

    async def list_pods_native(self, resource_version: Optional[str] = None, limit: int = 0,
                               field_selector: Optional[str] = None):
        """Pod list decoded and projected in C++: yields ([PodEvent], list RV) per page."""
        from .native import api_error, module
        cont = ""
        while True:
            self._refresh_token()
            status, raw = await self.native.request(
                "GET", self._path("pods", params=self._list_params(resource_version, limit, field_selector, cont)
                                  or None), b"", "", False, self.timeout)
            if status == 401 and self.config.token_file:
                self._refresh_token(force=True)
                status, raw = await self.native.request(
                    "GET", self._path("pods", params=self._list_params(resource_version, limit, field_selector,
                                                                       cont) or None), b"", "", False, self.timeout)
            if status < 0 or status >= 400:
                raise api_error(status, raw)
            rv, cont, evs = module().project_list(raw)
            yield evs, rv or "0"
            if not cont:
                return

    def _watch_params(self, resource_version: str, field_selector: Optional[str], timeout_s: int) -> dict:
        params = {"watch": "1", "resourceVersion": resource_version or "0", "allowWatchBookmarks": "true",
                  "timeoutSeconds": str(timeout_s)}
        if field_selector:
            params["fieldSelector"] = field_selector
        return params

    def watch_native(self, res: str, resource_version: str, on_events, on_end, field_selector: Optional[str] = None,
                     timeout_s: int = 300, pods: bool = False) -> int:
        """Start a native watch stream; events arrive in batches through ``on_events``."""
        self._refresh_token()
        return self.native.watch(self._path(res, params=self._watch_params(resource_version, field_selector,
                                                                           timeout_s)), pods, on_events, on_end,
                                 idle_timeout=timeout_s + WATCH_IDLE_GRACE_S)

    async def watch(self, res: str, resource_version: str, field_selector: Optional[str] = None,
                    timeout_s: int = 300) -> AsyncIterator[tuple[str, dict]]:
        if self.native is not None:
            async for ev in self._watch_native_iter(res, resource_version, field_selector, timeout_s):
                yield ev
            return
        s = await self.session()
        params = self._watch_params(resource_version, field_selector, timeout_s)
        async with s.get(self._url(res), params=params,
                         timeout=aiohttp.ClientTimeout(total=None, sock_read=timeout_s + 30)) as r:
            if r.status >= 400:
                text = await r.text()
                if r.status == 401:
                    self._refresh_token(force=True)
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

    async def _watch_native_iter(self, res: str, resource_version: str, field_selector: Optional[str],
                                 timeout_s: int):
        import collections
        q: collections.deque = collections.deque()
        end: list = []
        waiter: list = [None]

        def wake() -> None:
            w = waiter[0]
            if w is not None and not w.done():
                w.set_result(None)

        def on_events(evs) -> None:
            q.extend(evs)
            wake()

        def on_end(status: int, body: bytes) -> None:
            end.append((status, body))
            wake()

        wid = self.watch_native(res, resource_version, on_events, on_end, field_selector, timeout_s)
        try:
            while True:
                while q:
                    typ, _rv, payload, _idt = q.popleft()
                    obj = json.loads(payload) if payload else {"metadata": {"resourceVersion": _rv}}
                    if typ == "ERROR":
                        raise ApiError(int(obj.get("code", 500)), obj.get("reason", "Error"), obj.get("message", ""))
                    yield typ, obj
                if end:
                    status, body = end[0]
                    if status == 200 or status == 0:
                        return
                    if status == 401:
                        self._refresh_token(force=True)
                    from .native import api_error
                    raise api_error(status, body)
                waiter[0] = asyncio.get_event_loop().create_future()
                await waiter[0]
        finally:
            if not end and self.native is not None:
                self.native.cancel(wid)

    async def get(self, res: str, name: str, namespace: Optional[str] = None) -> dict:
        return await self._req("GET", res, namespace, name)

    async def create(self, res: str, obj: dict, namespace: Optional[str] = None, parse: bool = True) -> dict:
        """POST ``obj``; the created object as the apiserver returned it (``parse=False``: an
        empty dict — the caller needs only the success)."""
        ns = namespace or (obj.get("metadata") or {}).get("namespace") or ("default" if resource(res).namespaced else None)
        return await self._req("POST", res, ns, body=obj, parse=parse)

    async def update(self, res: str, obj: dict, namespace: Optional[str] = None) -> dict:
        m = obj.get("metadata") or {}
        ns = namespace or m.get("namespace")
        return await self._req("PUT", res, ns, m["name"], body=obj)

    async def update_status(self, res: str, obj: dict, namespace: Optional[str] = None) -> dict:
        m = obj.get("metadata") or {}
        ns = namespace or m.get("namespace")
        return await self._req("PUT", res, ns, m["name"], "status", body=obj)

    async def patch(self, res: str, name: str, patch: dict, namespace: Optional[str] = None,
                    limited: bool = False, strategic: bool = False) -> dict:
        """A JSON merge patch, or with ``strategic`` a strategic merge patch (what upstream's
        scheduler sends for pod status: conditions merge by type instead of replacing the list)."""
        sub = "status" if res == "pods" and set(patch) == {"status"} else None
        return await self._req("PATCH", res, namespace, name, sub, body=patch,
                               content_type="application/strategic-merge-patch+json" if strategic
                               else "application/merge-patch+json", limited=limited)

    async def delete(self, res: str, name: str, namespace: Optional[str] = None, limited: bool = False) -> dict:
        return await self._req("DELETE", res, namespace, name, limited=limited)

    async def bind(self, namespace: str, name: str, uid: str, node: str, annotations: Optional[dict] = None) -> None:
        if self.native is not None:
            self._refresh_token()
            fut = asyncio.get_event_loop().create_future()

            def done(status: int, body: bytes) -> None:
                if not fut.done():
                    fut.set_result((status, body))
            self.native.bind(namespace, name, uid, node, list((annotations or {}).items()), done, self.timeout)
            status, body = await fut
            if status < 0 or status >= 400:
                from .native import api_error
                raise api_error(status, body)
            return
        if self.fast_bind:
            if self._binder is None:
                from .fastbind import FastBinder
                self._binder = FastBinder(self.config.server, self.config.current_token(), self._binder_ssl(),
                                          timeout=self.timeout)
            await self._binder.bind(namespace, name, uid, node, annotations)
            return
        body = {"apiVersion": "v1", "kind": "Binding",
                "metadata": {"name": name, "namespace": namespace, "uid": uid, "annotations": dict(annotations or {})},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node}}
        await self._req("POST", "pods", namespace, name, "binding", body=body)
