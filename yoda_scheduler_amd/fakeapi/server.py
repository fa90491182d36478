"""In-process fake kube-apiserver (SURVEY §4 item 3, §7.3 hard part 1).

Faithful enough that scheduler behaviour transfers to a real cluster:

* global monotonically increasing ``resourceVersion``; optimistic concurrency on
  update (409 Conflict on a stale resourceVersion);
* list + watch with per-resource event history; a watch from a resourceVersion older
  than the retained history fails with 410 Gone (forcing a relist, like etcd
  compaction);
* ``pods/binding`` semantics: 404 for a missing pod, 409 if the pod is already bound
  or the uid does not match, annotations of the Binding are copied onto the pod,
  ``PodScheduled=True`` is set;
* lease objects for leader election, events, the cluster-scoped ``scvs`` CRD;
* fault injection (:class:`Faults`): bind failure ratio, API latency, watch drops;
* latency accounting for benches: ``perf_counter`` at pod create and at bind ack.

Objects handed to watchers/clients are treated as immutable snapshots: every write
produces a new dict, so consumers never need deep copies.
"""
from __future__ import annotations

import asyncio
import base64
import collections
import itertools
import json
import random
import time
import uuid
from dataclasses import dataclass
from typing import Optional

from ..kube.errors import ApiError, already_exists, conflict, gone, not_found
from ..kube.fields import FieldSelector, filter_event
from ..kube.fields import parse as parse_fields
from ..kube.resources import RESOURCES, obj_key, resource
from ..models.scv import rfc3339


@dataclass
class Faults:
    bind_fail_ratio: float = 0.0        # probability a bind returns 500
    bind_conflict_ratio: float = 0.0    # probability a bind returns 409
    latency_s: float = 0.0              # added to every client call
    drop_watch_every: int = 0           # close watches after N events (0 = never)
    seed: int = 0

    def __post_init__(self) -> None:
        self.rng = random.Random(self.seed)


class Watch:
    """One watch stream: events queue in a deque; a reader parks on one future only when
    the deque is empty (an ``asyncio.Queue`` costs a put/get pair of coroutine hops per
    event, which an in-process burst pays twice per pod)."""
    __slots__ = ("resource", "_dq", "_waiter", "closed", "sent", "server", "selector")

    def __init__(self, server: "FakeApiServer", resource: str, selector: Optional[FieldSelector] = None) -> None:
        self.server = server
        self.resource = resource
        self.selector = selector
        self._dq: collections.deque = collections.deque()
        self._waiter: Optional[asyncio.Future] = None
        self.closed = False
        self.sent = 0

    def _wake(self) -> None:
        w = self._waiter
        if w is not None:
            self._waiter = None
            if not w.done():
                w.set_result(None)

    def _put(self, ev) -> None:
        self._dq.append(ev)
        if self._waiter is not None:
            self._wake()

    def push(self, ev: tuple) -> None:
        if self.closed:
            return
        self._put(ev)
        self.sent += 1
        dw = self.server.faults.drop_watch_every
        if dw and self.sent % dw == 0:
            self.close()

    def close(self) -> None:
        if not self.closed:
            self.closed = True
            self._put(None)
            self.server._watchers[self.resource].discard(self)

    async def _wait(self) -> None:
        fut = self._waiter = asyncio.get_running_loop().create_future()
        try:
            await fut
        finally:
            if self._waiter is fut:
                self._waiter = None

    async def get(self):
        """The next event, or None once the watch is closed."""
        dq = self._dq
        while not dq:
            await self._wait()
        ev = dq[0]
        if ev is not None:
            dq.popleft()
        return ev

    async def next_batch(self) -> Optional[list]:
        """Every queued event (at least one), or None once the watch is closed."""
        dq = self._dq
        while not dq:
            await self._wait()
        if dq[-1] is None:
            out = list(dq)[:-1]
            dq.clear()
            dq.append(None)          # the end marker stays for the next call
            return out or None
        out = list(dq)
        dq.clear()
        return out

    def __aiter__(self):
        return self

    async def __anext__(self):
        ev = await self.get()
        if ev is None:
            raise StopAsyncIteration
        return ev


class FakeApiServer:
    def __init__(self, history: int = 200_000, faults: Optional[Faults] = None,
                 clock=time.perf_counter) -> None:
        self._rv = itertools.count(1)
        self._last_rv = 0
        # uids: unique per server (random prefix) and per object (counter) — uuid4 per
        # object costs more than the rest of a create
        self._uid_prefix = uuid.uuid4().hex[:20]
        self._uids = itertools.count(1)
        self._objs: dict[str, dict[str, dict]] = {r: {} for r in RESOURCES}
        self._watchers: dict[str, set[Watch]] = {r: set() for r in RESOURCES}
        self._history: dict[str, collections.deque] = {r: collections.deque(maxlen=history) for r in RESOURCES}
        self._oldest_rv: dict[str, int] = {r: 0 for r in RESOURCES}
        self.faults = faults or Faults()
        self.clock = clock
        self.create_log: dict[str, float] = {}
        self.bind_log: dict[str, float] = {}
        self.bind_node: dict[str, str] = {}
        self.calls = collections.Counter()
        self.patch_log: list = []          # (res, namespace, name, strategic, patch) of every PATCH

    # ------------------------------------------------------------------ internals
    def _next_rv(self) -> str:
        self._last_rv = next(self._rv)
        return str(self._last_rv)

    def _emit(self, res: str, typ: str, obj: dict, old: Optional[dict] = None, rv: int = 0) -> None:
        if not rv:
            rv = int(obj["metadata"]["resourceVersion"])
        h = self._history[res]
        if len(h) == h.maxlen:
            self._oldest_rv[res] = h[0][0]
        h.append((rv, typ, obj, old))
        ws = self._watchers[res]
        # a push closes its watch (and leaves the set) only under drop_watch_every
        for w in (tuple(ws) if self.faults.drop_watch_every else ws):
            if w.selector is None:
                w.push((typ, obj))
            else:
                ev = filter_event(w.selector, typ, obj, old)
                if ev is not None:
                    w.push(ev)

    @staticmethod
    def _with_meta(obj: dict, **meta) -> dict:
        new = dict(obj)
        m = dict(obj.get("metadata") or {})
        m.update(meta)
        new["metadata"] = m
        return new

    # ------------------------------------------------------------------ CRUD
    def create(self, res: str, obj: dict, namespace: Optional[str] = None) -> dict:
        self.calls["create"] += 1
        r = resource(res)
        meta = dict(obj.get("metadata") or {})
        if r.namespaced:
            meta.setdefault("namespace", namespace or "default")
        if not meta.get("name"):
            if meta.get("generateName"):
                meta["name"] = meta["generateName"] + uuid.uuid4().hex[:5]
            else:
                raise ApiError(422, "Invalid", "metadata.name required")
        new = dict(obj)
        new.setdefault("apiVersion", r.api_version)
        new.setdefault("kind", r.kind)
        meta["uid"] = meta.get("uid") or f"{self._uid_prefix}-{next(self._uids):012x}"
        rv = self._last_rv = next(self._rv)
        meta["resourceVersion"] = str(rv)
        if "creationTimestamp" not in meta:
            meta["creationTimestamp"] = rfc3339(time.time())
        new["metadata"] = meta
        key = f"{meta['namespace'] or 'default'}/{meta['name']}" if r.namespaced else meta["name"]
        store = self._objs[res]
        if key in store:
            raise already_exists(f"{res} {key}")
        store[key] = new
        if res == "pods":
            self.create_log[key] = self.clock()
        self._emit(res, "ADDED", new, None, rv)
        return new

    def get(self, res: str, name: str, namespace: Optional[str] = None) -> dict:
        r = resource(res)
        key = f"{namespace or 'default'}/{name}" if r.namespaced else name
        try:
            return self._objs[res][key]
        except KeyError:
            raise not_found(f"{res} {key}") from None

    def update(self, res: str, obj: dict, namespace: Optional[str] = None, status_only: bool = False) -> dict:
        self.calls["update"] += 1
        r = resource(res)
        meta = obj.get("metadata") or {}
        ns = meta.get("namespace") or namespace
        cur = self.get(res, meta.get("name", ""), ns)
        rv = meta.get("resourceVersion")
        if rv and rv != cur["metadata"]["resourceVersion"]:
            raise conflict(f"{res} {obj_key(r, cur)}: the object has been modified")
        if status_only:
            new = dict(cur)
            new["status"] = obj.get("status")
        else:
            new = dict(obj)
            if "status" not in obj and "status" in cur:
                new["status"] = cur["status"]
        new["metadata"] = dict(cur["metadata"], **{k: v for k, v in meta.items()
                                                   if k not in ("uid", "creationTimestamp", "resourceVersion")})
        new["metadata"]["resourceVersion"] = self._next_rv()
        self._objs[res][obj_key(r, new)] = new
        self._emit(res, "MODIFIED", new, cur)
        return new

    def patch(self, res: str, name: str, patch: dict, namespace: Optional[str] = None,
              strategic: bool = False) -> dict:
        """JSON merge patch (RFC 7386), or a strategic merge patch (lists with a patch merge key —
        status.conditions by type, ... — merged element-wise, ``_strategic``)."""
        self.calls["patch"] += 1
        self.patch_log.append((res, namespace, name, strategic, patch))
        cur = self.get(res, name, namespace)
        new = _strategic(cur, patch) if strategic else _merge(cur, patch)
        new["metadata"] = dict(new.get("metadata") or {})
        new["metadata"]["resourceVersion"] = self._next_rv()
        for k in ("uid", "name", "namespace", "creationTimestamp"):
            if k in cur["metadata"]:
                new["metadata"][k] = cur["metadata"][k]
        self._objs[res][obj_key(resource(res), new)] = new
        self._emit(res, "MODIFIED", new, cur)
        return new

    def delete(self, res: str, name: str, namespace: Optional[str] = None) -> dict:
        self.calls["delete"] += 1
        r = resource(res)
        key = f"{namespace or 'default'}/{name}" if r.namespaced else name
        cur = self._objs[res].pop(key, None)
        if cur is None:
            raise not_found(f"{res} {key}")
        gone_obj = self._with_meta(cur, resourceVersion=self._next_rv())
        self._emit(res, "DELETED", gone_obj)
        return gone_obj

    def list(self, res: str, namespace: Optional[str] = None,
             field_selector: Optional[str] = None) -> tuple[list[dict], str]:
        self.calls["list"] += 1
        items = list(self._objs[res].values())
        if namespace and resource(res).namespaced:
            items = [o for o in items if o["metadata"].get("namespace") == namespace]
        sel = parse_fields(field_selector)
        if sel is not None:
            items = [o for o in items if sel.matches(o)]
        return items, str(self._last_rv)

    def list_page(self, res: str, namespace: Optional[str] = None, limit: int = 0,
                  cont: str = "", field_selector: Optional[str] = None) -> tuple[list[dict], str, str]:
        """Chunked list (``limit`` / ``continue``): items in key order; the continue token
        pins the list's resourceVersion and the last key served, like the apiserver's. A
        token older than the watch history window is expired (410)."""
        self.calls["list"] += 1
        if cont:
            try:
                tok = json.loads(base64.urlsafe_b64decode(cont.encode()).decode())
                rv, start = int(tok["rv"]), str(tok["start"])
            except (ValueError, KeyError, TypeError):
                raise ApiError(400, "BadRequest", "invalid continue token") from None
            if rv < self._oldest_rv[res]:
                raise ApiError(410, "Expired", "the provided continue parameter is too old")
        else:
            rv, start = self._last_rv, ""
        keys = sorted(k for k in self._objs[res] if k > start)
        if namespace and resource(res).namespaced:
            keys = [k for k in keys if self._objs[res][k]["metadata"].get("namespace") == namespace]
        sel = parse_fields(field_selector)
        if sel is not None:
            keys = [k for k in keys if sel.matches(self._objs[res][k])]
        nxt = ""
        if limit and len(keys) > limit:
            keys = keys[:limit]
            nxt = base64.urlsafe_b64encode(json.dumps({"rv": rv, "start": keys[-1]}).encode()).decode()
        return [self._objs[res][k] for k in keys], str(rv), nxt

    def bookmark(self, res: str) -> None:
        """Send a BOOKMARK (current resourceVersion, no object change) to every watcher."""
        obj = {"kind": resource(res).kind, "apiVersion": resource(res).api_version,
               "metadata": {"resourceVersion": str(self._last_rv)}}
        for w in tuple(self._watchers[res]):
            w.push(("BOOKMARK", obj))

    def watch(self, res: str, resource_version: str = "0", field_selector: Optional[str] = None) -> Watch:
        self.calls["watch"] += 1
        rv = int(resource_version or 0)
        if rv and rv < self._oldest_rv[res]:
            raise gone()
        sel = parse_fields(field_selector)
        w = Watch(self, res, sel)
        if rv:
            for erv, typ, obj, old in self._history[res]:
                if erv > rv:
                    ev = (typ, obj) if sel is None else filter_event(sel, typ, obj, old)
                    if ev is not None:
                        w._put(ev)
        self._watchers[res].add(w)
        return w

    def close_watches(self) -> None:
        for ws in self._watchers.values():
            for w in tuple(ws):
                w.close()

    # ------------------------------------------------------------------ subresources
    def bind(self, namespace: str, name: str, uid: str, node: str, annotations: Optional[dict] = None) -> dict:
        self.calls["bind"] += 1
        f = self.faults
        if f.bind_fail_ratio and f.rng.random() < f.bind_fail_ratio:
            raise ApiError(500, "InternalError", "injected bind failure")
        if f.bind_conflict_ratio and f.rng.random() < f.bind_conflict_ratio:
            raise conflict("injected bind conflict")
        key = f"{namespace}/{name}"
        cur = self._objs["pods"].get(key)
        if cur is None:
            raise not_found(f"pods {key}")
        if uid and cur["metadata"].get("uid") != uid:
            raise conflict(f"pod {key} uid mismatch")
        if (cur.get("spec") or {}).get("nodeName"):
            raise conflict(f"pod {key} is already assigned to node {cur['spec']['nodeName']}")
        spec = dict(cur.get("spec") or {})
        spec["nodeName"] = node
        status = dict(cur.get("status") or {})
        conds = [c for c in status.get("conditions") or [] if c.get("type") != "PodScheduled"]
        conds.append({"type": "PodScheduled", "status": "True", "lastTransitionTime": rfc3339(time.time())})
        status["conditions"] = conds
        meta = dict(cur["metadata"])
        if annotations:
            meta["annotations"] = dict(meta.get("annotations") or {}, **annotations)
        rv = self._last_rv = next(self._rv)
        meta["resourceVersion"] = str(rv)
        new = dict(cur)
        new["spec"], new["status"], new["metadata"] = spec, status, meta
        self._objs["pods"][key] = new
        self.bind_log[key] = self.clock()
        self.bind_node[key] = node
        self._emit("pods", "MODIFIED", new, cur, rv)
        return new

    # ------------------------------------------------------------------ bench helpers
    def latencies(self) -> list[float]:
        return [self.bind_log[k] - self.create_log[k] for k in self.bind_log if k in self.create_log]

    def reset_logs(self) -> None:
        self.create_log.clear()
        self.bind_log.clear()
        self.bind_node.clear()


def _merge(cur, patch):
    if not isinstance(patch, dict):
        return patch
    out = dict(cur) if isinstance(cur, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = _merge(out.get(k), v)
    return out


# patch merge keys of the core/v1 Pod lists (``native/kube/json.cpp::strategic_merge_patch``)
MERGE_KEYS = {"conditions": "type", "containers": "name", "initContainers": "name", "ephemeralContainers": "name",
              "volumes": "name", "env": "name", "ports": "containerPort", "ownerReferences": "uid",
              "volumeMounts": "mountPath", "imagePullSecrets": "name"}


def _strategic(cur, patch):
    """Kubernetes strategic merge patch, the subset a Pod needs: merge-keyed lists merge
    element-wise (``$patch: delete`` removes an element), other lists are replaced, ``$``
    directives ($setElementOrder, $retainKeys) are accepted and ignored."""
    if not isinstance(patch, dict):
        return patch
    out = dict(cur) if isinstance(cur, dict) else {}
    for k, v in patch.items():
        if k.startswith("$"):
            continue
        if v is None:
            out.pop(k, None)
            continue
        mk = MERGE_KEYS.get(k)
        old = out.get(k)
        if mk and isinstance(v, list) and isinstance(old, list):
            items = [dict(x) if isinstance(x, dict) else x for x in old]
            for item in v:
                if not isinstance(item, dict) or mk not in item:
                    items.append(item)
                    continue
                at = next((i for i, x in enumerate(items) if isinstance(x, dict) and x.get(mk) == item[mk]), None)
                if item.get("$patch") == "delete":
                    if at is not None:
                        items.pop(at)
                elif at is None:
                    items.append(_strategic({}, item))
                else:
                    items[at] = _strategic(items[at], item)
            out[k] = items
        elif isinstance(v, list):
            out[k] = [_strategic({}, x) if isinstance(x, dict) else x for x in v]
        else:
            out[k] = _strategic(old, v)
    return out
