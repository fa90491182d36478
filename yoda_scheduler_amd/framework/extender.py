"""HTTP scheduler extenders (``KubeSchedulerConfiguration.extenders``), the out-of-process
extension mechanism of the kube-scheduler the reference runs on.

Wire format (JSON over HTTP POST to ``urlPrefix/verb``), as upstream:

* filter:     ExtenderArgs ``{Pod, Nodes|NodeNames}`` → ExtenderFilterResult
  ``{Nodes|NodeNames, FailedNodes, Error}``
* prioritize: ExtenderArgs → HostPriorityList ``[{Host, Score}]`` with scores 0..10,
  scaled by ``weight × MaxNodeScore / 10`` and added to the node's total;
* bind:       ExtenderBindingArgs ``{PodName, PodNamespace, PodUID, Node}`` →
  ExtenderBindingResult ``{Error}``.

An extender with ``managedResources`` only sees pods that request one of them;
``ignorable`` extenders' failures are skipped instead of failing the cycle. Pods of a
scheduler with extenders take the (async) hybrid cycle.
"""
from __future__ import annotations

import asyncio
import json
from typing import Optional

import aiohttp

from .config import ExtenderConfig

MAX_EXTENDER_PRIORITY = 10
MAX_NODE_SCORE = 100


class ExtenderError(Exception):
    pass


class HTTPExtender:
    def __init__(self, cfg: ExtenderConfig) -> None:
        self.cfg = cfg
        self._session: Optional[aiohttp.ClientSession] = None

    @property
    def name(self) -> str:
        return self.cfg.url_prefix

    def is_interested(self, pod) -> bool:
        managed = self.cfg.managed_resources
        if not managed:
            return True
        names = {n for n, _ in managed}
        spec = pod.obj.get("spec") or {}
        for key in ("containers", "initContainers"):
            for c in spec.get(key) or ():
                res = c.get("resources") or {}
                if names & set(res.get("requests") or {}) or names & set(res.get("limits") or {}):
                    return True
        return False

    async def _post(self, verb: str, body: dict):
        if self._session is None or self._session.closed:
            self._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=self.cfg.http_timeout))
        async with self._session.post(f"{self.cfg.url_prefix}/{verb}", data=json.dumps(body),
                                      headers={"Content-Type": "application/json"}) as r:
            text = await r.text()
            if r.status >= 400:
                raise ExtenderError(f"{self.name}/{verb}: HTTP {r.status}: {text[:200]}")
            return json.loads(text) if text else {}

    def _args(self, pod, nodes: list[str], node_objs: dict) -> dict:
        if self.cfg.node_cache_capable:
            return {"Pod": pod.obj, "NodeNames": list(nodes)}
        return {"Pod": pod.obj, "Nodes": {"items": [node_objs[n] for n in nodes if n in node_objs]}}

    async def filter(self, pod, nodes: list[str], node_objs: dict) -> tuple[list[str], dict]:
        res = await self._post(self.cfg.filter_verb, self._args(pod, nodes, node_objs))
        if res.get("Error"):
            raise ExtenderError(f"{self.name}: {res['Error']}")
        if res.get("NodeNames") is not None:
            keep = list(res.get("NodeNames") or [])
        else:
            keep = [((n.get("metadata") or {}).get("name", "")) for n in ((res.get("Nodes") or {}).get("items") or [])]
        return keep, dict(res.get("FailedNodes") or {})

    async def prioritize(self, pod, nodes: list[str], node_objs: dict) -> dict[str, int]:
        res = await self._post(self.cfg.prioritize_verb, self._args(pod, nodes, node_objs))
        scale = self.cfg.weight * (MAX_NODE_SCORE // MAX_EXTENDER_PRIORITY)
        return {h.get("Host", ""): int(h.get("Score", 0)) * scale for h in res or []}

    async def bind(self, pod, node: str) -> None:
        res = await self._post(self.cfg.bind_verb, {"PodName": pod.name, "PodNamespace": pod.namespace,
                                                    "PodUID": pod.uid, "Node": node})
        if (res or {}).get("Error"):
            raise ExtenderError(f"{self.name}: bind: {res['Error']}")

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()


async def run_extenders(extenders: list, pod, nodes: list[str], node_objs: dict) -> tuple[list[str], dict, dict]:
    """Filter through every interested extender in order, then sum their priorities.
    Returns (feasible names, failed {node: reason}, extra scores {node: score})."""
    failed: dict = {}
    for e in extenders:
        if not e.cfg.filter_verb or not e.is_interested(pod) or not nodes:
            continue
        try:
            nodes, f = await e.filter(pod, nodes, node_objs)
            failed.update(f)
        except (ExtenderError, aiohttp.ClientError, asyncio.TimeoutError, ValueError) as err:
            if e.cfg.ignorable:
                continue
            raise ExtenderError(str(err)) from err
    scores: dict = {}
    if len(nodes) > 1:
        for e in extenders:
            if not e.cfg.prioritize_verb or not e.is_interested(pod):
                continue
            try:
                for h, s in (await e.prioritize(pod, nodes, node_objs)).items():
                    scores[h] = scores.get(h, 0) + s
            except (ExtenderError, aiohttp.ClientError, asyncio.TimeoutError, ValueError):
                continue   # upstream: a failing prioritizer is ignored
    return nodes, failed, scores
