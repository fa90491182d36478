"""Sniffer agent: sample the node's GPUs and publish the ``Scv`` status (one
cluster-scoped object per node, named after it — the contract the reference reads at
``pkg/yoda/scheduler.go:80,118``).

Change-driven publishing: the node is sampled every ``interval`` but the ``Scv`` is
written only when something the scheduler acts on moved — free HBM by ≥
``free_delta_mb`` on any GPU, health, the GPU count, xGMI link load by ≥ ``load_delta``,
CU occupancy by ≥ ``occupancy_delta`` points — or when ``heartbeat`` seconds passed. The
object's ``spec.updateInterval`` is the heartbeat, so the scheduler's staleness rule
(``staleFactor`` × interval) is driven by the heartbeat, not the sample rate. A write is
one ``PUT .../status`` with the resourceVersion of the previous write (a GET only after
a 409), so an idle 1000-node cluster costs ~1000/heartbeat writes/s instead of 2000/s.

HBM probes (gfx950 kernels, ``native/hip/probes.hip``) run only on idle GPUs (no tenant
process and little HBM in use), with a buffer sized from the free HBM, and are repeated
every ``probe_interval``; a GPU turns Unhealthy after ``fail_threshold`` consecutive
failed pattern checks and recovers after a clean one. Probe results are attributed to
amd-smi indices through the HIP ordinal ↔ amd-smi mapping (``hipId`` from
``amdsmi_get_gpu_enumeration_info``, else the PCI bus id), never by assuming the two
enumerations agree.
"""
from __future__ import annotations

import asyncio
import logging
import time
from typing import Optional

from ..kube.errors import ApiError
from .collector import UNHEALTHY, samples_to_scv

log = logging.getLogger("yoda.sniffer")


def hip_to_index(samples: list[dict], hip_count: int, bus_id=None) -> dict[int, int]:
    """HIP ordinal → amd-smi index. Uses the collector's ``hipId``; falls back to matching
    ``hipDeviceGetPCIBusId`` against the samples' BDFs (ambiguous BDFs — partitions of one
    GPU without a hipId — are left unmapped rather than guessed)."""
    by_hip = {int(s["hipId"]): int(s["index"]) for s in samples if int(s.get("hipId", -1)) >= 0}
    if by_hip and all(d in by_hip for d in range(hip_count)):
        return {d: by_hip[d] for d in range(hip_count)}
    counts: dict[str, int] = {}
    for s in samples:
        b = str(s.get("bdf", "")).lower()
        counts[b] = counts.get(b, 0) + 1
    by_bdf = {str(s.get("bdf", "")).lower(): int(s["index"]) for s in samples}
    out = dict(by_hip)
    if bus_id is None:
        return out
    for d in range(hip_count):
        if d in out:
            continue
        try:
            b = bus_id(d).lower()
        except Exception:  # noqa: BLE001
            continue
        if counts.get(b) == 1:
            out[d] = by_bdf[b]
    return out


class HipProber:
    """The gfx950 HBM probes of ``ops.hip`` behind the interface the agent uses."""

    def count(self) -> int:
        from ..ops import hip
        return hip.device_count()

    def bus_id(self, d: int) -> str:
        from ..ops import hip
        return hip.pci_bus_id(d)

    def bandwidth_gbps(self, d: int, nbytes: int) -> float:
        from ..ops import hip
        return float(hip.hbm_bandwidth(d, nbytes, 5)["read_gbps"])

    def pattern_errors(self, d: int, nbytes: int) -> int:
        from ..ops import hip
        return int(hip.hbm_pattern_check(d, nbytes)["errors"])


class SnifferAgent:
    def __init__(self, client, node: str, backend, interval: float = 1.0, probe: bool = False,
                 probe_bytes: int = 1 << 30, heartbeat: float = 10.0, free_delta_mb: int = 1024,
                 load_delta: float = 0.05, occupancy_delta: float = 5.0, probe_interval: float = 600.0,
                 probe_max_fraction: float = 0.25, busy_vram_mb: int = 2048, fail_threshold: int = 3,
                 prober=None, clock=time.monotonic) -> None:
        self.client = client
        self.node = node
        self.backend = backend
        self.interval = interval
        self.heartbeat = max(heartbeat, interval)
        self.free_delta_mb = free_delta_mb
        self.load_delta = load_delta
        self.occupancy_delta = occupancy_delta
        self.probe = probe
        self.probe_bytes = probe_bytes
        self.probe_interval = probe_interval
        self.probe_max_fraction = probe_max_fraction
        self.busy_vram_mb = busy_vram_mb
        self.fail_threshold = max(1, fail_threshold)
        self.prober = prober
        self.clock = clock
        # probe state per amd-smi index
        self.measured_bw: dict[int, float] = {}
        self.probe_fail_streak: dict[int, int] = {}
        self.probe_runs: dict[int, int] = {}
        self.probe_skipped: dict[int, str] = {}
        self._last_probe = -1e18
        # publishing state
        self.published = 0
        self.samples = 0
        self.failures = 0
        self.skipped = 0
        self._last_pub: Optional[tuple] = None     # (signature, monotonic time)
        self._rv = ""
        self._stop = asyncio.Event()

    # ------------------------------------------------------------------ probes
    def probe_unhealthy(self) -> dict[int, int]:
        return {i: 1 for i, n in self.probe_fail_streak.items() if n >= self.fail_threshold}

    def run_probes(self, samples: Optional[list[dict]] = None) -> dict:
        """Probe every idle GPU once (synchronous; the agent runs it in a worker thread).
        Returns {amd-smi index: result or skip reason}."""
        prober = self.prober or HipProber()
        if samples is None:
            samples = self.backend.sample()
        by_index = {int(s["index"]): s for s in samples}
        mapping = hip_to_index(samples, prober.count(), prober.bus_id)
        res: dict = {}
        for d, i in sorted(mapping.items()):
            s = by_index.get(i)
            if s is None:
                continue
            procs = int(s.get("processes", -1))
            used = int(s.get("vramUsedMB", 0))
            free_mb = max(0, int(s.get("vramTotalMB", 0)) - used)
            if procs > 0 or used > self.busy_vram_mb:
                why = f"busy ({procs} process(es), {used} MB in use)"
                self.probe_skipped[i] = why
                res[i] = {"skipped": why}
                continue
            nbytes = min(self.probe_bytes, int(free_mb * self.probe_max_fraction) << 20)
            nbytes -= nbytes % (1 << 20)
            if nbytes < (16 << 20):
                self.probe_skipped[i] = "too little free HBM"
                res[i] = {"skipped": "too little free HBM"}
                continue
            self.probe_skipped.pop(i, None)
            bw = prober.bandwidth_gbps(d, nbytes)
            errs = prober.pattern_errors(d, nbytes)
            self.measured_bw[i] = round(bw)
            self.probe_fail_streak[i] = self.probe_fail_streak.get(i, 0) + 1 if errs else 0
            self.probe_runs[i] = self.probe_runs.get(i, 0) + 1
            res[i] = {"hip": d, "bytes": nbytes, "read_gbps": bw, "pattern_errors": errs,
                      "fail_streak": self.probe_fail_streak[i]}
        return res

    async def maybe_probe(self, samples: list[dict]) -> Optional[dict]:
        now = self.clock()
        if not self.probe or now - self._last_probe < self.probe_interval:
            return None
        self._last_probe = now
        try:
            return await asyncio.get_event_loop().run_in_executor(None, self.run_probes, samples)
        except Exception as e:  # noqa: BLE001 - probes are optional
            log.warning("HIP probes failed: %r", e)
            return None

    # ------------------------------------------------------------------ publishing
    def build(self, samples: Optional[list[dict]] = None):
        samples = self.backend.sample() if samples is None else samples
        return samples_to_scv(self.node, samples, int(self.heartbeat * 1000), self.measured_bw or None,
                              self.probe_unhealthy() or None, sniffer=getattr(self.backend, "name", "amd-smi"))

    @staticmethod
    def signature(scv) -> tuple:
        return tuple((c.health, c.free_memory, c.total_memory, round(c.cu_occupancy, 1),
                      tuple(sorted((l.peer, round(l.load, 3)) for l in c.xgmi))) for c in scv.status.card_list)

    def changed(self, sig: tuple) -> bool:
        """Meaningful change since the last publish (or heartbeat due)."""
        if self._last_pub is None:
            return True
        old, t = self._last_pub
        if self.clock() - t >= self.heartbeat or len(old) != len(sig):
            return True
        for a, b in zip(old, sig):
            if a[0] != b[0] or a[2] != b[2]:
                return True                                   # health or capacity
            if abs(a[1] - b[1]) >= self.free_delta_mb or abs(a[3] - b[3]) >= self.occupancy_delta:
                return True
            la, lb = dict(a[4]), dict(b[4])
            if la.keys() != lb.keys() or any(abs(la[k] - lb[k]) >= self.load_delta for k in la):
                return True
        return False

    async def _write(self, obj: dict) -> dict:
        for attempt in range(5):
            try:
                if self._rv:
                    obj["metadata"]["resourceVersion"] = self._rv
                    out = await self.client.update_status("scvs", obj)
                else:
                    try:
                        cur = await self.client.get("scvs", self.node)
                        obj["metadata"]["resourceVersion"] = cur["metadata"]["resourceVersion"]
                    except ApiError as e:
                        if e.code != 404:
                            raise
                        created = await self.client.create("scvs", obj)
                        # with the status subresource a real apiserver drops .status on create
                        obj["metadata"]["resourceVersion"] = created["metadata"]["resourceVersion"]
                    out = await self.client.update_status("scvs", obj)
                self._rv = (out.get("metadata") or {}).get("resourceVersion", "")
                return out
            except ApiError as e:
                if e.code in (404, 409) and attempt < 4:
                    self._rv = ""             # someone else wrote (or deleted) it: re-read
                    continue
                raise
        raise RuntimeError("unreachable")

    async def publish_once(self, force: bool = True, samples: Optional[list[dict]] = None) -> Optional[dict]:
        scv = self.build(samples)
        self.samples += 1
        sig = self.signature(scv)
        if not force and not self.changed(sig):
            self.skipped += 1
            return None
        out = await self._write(scv.to_json())
        self._last_pub = (sig, self.clock())
        self.published += 1
        return out

    async def run(self, count: Optional[int] = None) -> None:
        n = 0
        while not self._stop.is_set() and (count is None or n < count):
            t0 = time.monotonic()
            try:
                samples = self.backend.sample()
                probed = await self.maybe_probe(samples)
                await self.publish_once(force=n == 0 or bool(probed), samples=samples)
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


__all__ = ["SnifferAgent", "HipProber", "hip_to_index", "UNHEALTHY"]
