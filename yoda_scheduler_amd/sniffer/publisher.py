"""Sniffer agent: sample the node's GPUs every ``interval`` and publish the ``Scv``
status (one cluster-scoped object per node, named after it — the contract the
reference reads at ``pkg/yoda/scheduler.go:80,118``).

Publishing is create-or-update with optimistic-concurrency retries; a failing sample
keeps the previous object, whose ``updateTime`` then ages until the scheduler treats
the node as stale (SURVEY §5 failure detection).
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import Optional

from ..kube.errors import ApiError
from .collector import samples_to_scv

log = logging.getLogger("yoda.sniffer")


class SnifferAgent:
    def __init__(self, client, node: str, backend, interval: float = 1.0, probe: bool = False,
                 probe_bytes: int = 1 << 30) -> None:
        self.client = client
        self.node = node
        self.backend = backend
        self.interval = interval
        self.probe = probe
        self.probe_bytes = probe_bytes
        self.measured_bw: dict[int, float] = {}
        self.probe_errors: dict[int, int] = {}
        self.published = 0
        self.failures = 0
        self._stop = asyncio.Event()

    def run_probes(self) -> dict:
        """HIP HBM bandwidth + pattern probes on every local GPU (hipcc gfx950 kernels)."""
        from ..ops import hip
        res = {}
        for d in range(hip.device_count()):
            bw = hip.hbm_bandwidth(d, self.probe_bytes, 5)
            pat = hip.hbm_pattern_check(d, self.probe_bytes)
            self.measured_bw[d] = round(bw["read_gbps"])
            self.probe_errors[d] = pat["errors"]
            res[d] = {"bandwidth": bw, "pattern": pat}
        return res

    def build(self):
        samples = self.backend.sample()
        return samples_to_scv(self.node, samples, int(self.interval * 1000), self.measured_bw or None,
                              self.probe_errors or None, sniffer=getattr(self.backend, "name", "amd-smi"))

    async def publish_once(self) -> dict:
        scv = self.build()
        obj = scv.to_json()
        for attempt in range(5):
            try:
                try:
                    cur = await self.client.get("scvs", self.node)
                except ApiError as e:
                    if e.code != 404:
                        raise
                    out = await self.client.create("scvs", obj)
                    # with the status subresource a real apiserver drops .status on create
                    obj["metadata"]["resourceVersion"] = out["metadata"]["resourceVersion"]
                    out = await self.client.update_status("scvs", obj)
                    self.published += 1
                    return out
                obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
                out = await self.client.update_status("scvs", obj)
                self.published += 1
                return out
            except ApiError as e:
                if e.code == 409 and attempt < 4:
                    continue
                raise
        raise RuntimeError("unreachable")

    async def run(self, count: Optional[int] = None) -> None:
        if self.probe:
            try:
                self.run_probes()
            except Exception as e:  # noqa: BLE001 - probes are optional
                log.warning("HIP probes failed: %r", e)
        n = 0
        while not self._stop.is_set() and (count is None or n < count):
            t0 = time.monotonic()
            try:
                await self.publish_once()
            except Exception as e:  # noqa: BLE001 - keep sampling
                self.failures += 1
                log.warning("publish failed: %r", e)
            n += 1
            if count is not None and n >= count:
                break
            try:
                await asyncio.wait_for(self._stop.wait(), max(0.0, self.interval - (time.monotonic() - t0)))
            except asyncio.TimeoutError:
                pass

    def stop(self) -> None:
        self._stop.set()
