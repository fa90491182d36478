"""Burst harness: pods created through the (fake) apiserver at t0, latency = pod
creation → binding acknowledged by the apiserver (BASELINE.md measurement protocol).

A :class:`Shard` is one scheduler process-worth of state: its own apiserver, cluster
(nodes + Scv telemetry) and scheduler instance. The fake apiserver runs in the same
process and event loop, so its CPU cost (create, watch fan-out, bind) is charged to the
measured throughput — a conservative setup compared with a real, separate apiserver.
"""
from __future__ import annotations

import asyncio
import time
from dataclasses import dataclass, field
from typing import Optional

from ..fakeapi.client import InProcessClient
from ..fakeapi.server import FakeApiServer
from ..framework.config import parse_config
from ..framework.scheduler import Scheduler
from ..utils.metrics import NullMetrics, SchedulerMetrics
from .workloads import Workload, pod_object, populate


def bench_config(scheduler_name: str, qps: float, burst: int, batch: int, compat: bool = False,
                 device: str = "auto") -> dict:
    """The shipped deploy profile (yoda at filter + score weight 300 on top of the
    upstream defaults) with the yoda QueueSort enabled (Q7) and the given client QPS."""
    prof = {"schedulerName": scheduler_name,
            "plugins": {"queueSort": {"enabled": [{"name": "yoda"}], "disabled": [{"name": "*"}]},
                        "filter": {"enabled": [{"name": "yoda", "weight": 0}]},
                        "score": {"enabled": [{"name": "yoda", "weight": 300}]}}}
    if compat:
        prof["pluginConfig"] = [{"name": "yoda", "args": {"compat": True}}]
    return {"apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration",
            "leaderElection": {"leaderElect": False},
            "clientConnection": {"qps": qps, "burst": burst},
            "percentageOfNodesToScore": 0, "podInitialBackoffSeconds": 1, "podMaxBackoffSeconds": 10,
            "yodaRuntime": {"batchSize": batch, "bindConcurrency": 256, "deviceScorer": {"enabled": device}},
            "profiles": [prof]}


@dataclass
class BurstResult:
    pods: int
    bound: int
    unschedulable: int
    elapsed_s: float
    latencies_s: list[float]
    e2e_s: list[float] = field(default_factory=list)   # scheduler-internal: cycle start → bind ack

    @property
    def pods_per_s(self) -> float:
        return self.bound / self.elapsed_s if self.elapsed_s > 0 else 0.0


def percentile(xs: list[float], q: float) -> float:
    if not xs:
        return float("nan")
    s = sorted(xs)
    k = min(len(s) - 1, max(0, int(round(q / 100.0 * (len(s) - 1)))))
    return s[k]


class Shard:
    def __init__(self, w: Workload, qps: float = 5000.0, burst: int = 10000, batch: int = 256,
                 template: Optional[dict] = None, metrics: bool = False, events: bool = True,
                 compat: bool = False, seed: int = 0, engine_threads: int = 1, device: str = "auto") -> None:
        self.w = w
        self.server = FakeApiServer()
        self.client = InProcessClient(self.server)
        populate(self.server, w, template, link_load=0.2 if w.id == 5 else 0.0, seed=seed)
        cfg = parse_config(bench_config(w.scheduler_name, qps, burst, batch, compat, device))
        self.sched = Scheduler(self.client, cfg, metrics=SchedulerMetrics() if metrics else NullMetrics(),
                               record_events=events, seed=seed, engine_threads=engine_threads)
        self.sched.e2e_samples = []
        self._loop_task: Optional[asyncio.Task] = None

    async def start(self) -> None:
        await self.sched.start()
        self._loop_task = asyncio.get_event_loop().create_task(self.sched.scheduling_loop())

    async def burst(self, tag: str = "b", timeout: float = 600.0) -> BurstResult:
        srv, w = self.server, self.w
        srv.reset_logs()
        self.sched.e2e_samples.clear()
        objs = [pod_object(i, lab, w.scheduler_name, prefix=tag) for i, lab in enumerate(w.pods)]
        t0 = time.perf_counter()
        for i, o in enumerate(objs):
            srv.create("pods", o)
            if i % 64 == 63:
                await asyncio.sleep(0)      # the apiserver accepts creates while the scheduler runs
        n = len(objs)
        q = self.sched.queue
        deadline = t0 + timeout
        while True:
            if len(srv.bind_log) >= n:
                break
            if not q._active_entries and self.sched.pending_binds == 0 and \
                    len(srv.bind_log) + len(q._unsched) + len(q._backoff_pods) >= n:
                break
            if time.perf_counter() > deadline:
                break
            await asyncio.sleep(0.0005)
        t_end = max(srv.bind_log.values()) if srv.bind_log else time.perf_counter()
        lat = srv.latencies()
        return BurstResult(n, len(srv.bind_log), n - len(srv.bind_log), t_end - t0, lat,
                           list(self.sched.e2e_samples))

    async def stop(self) -> None:
        await self.sched.shutdown()
        if self._loop_task:
            self._loop_task.cancel()
            await asyncio.gather(self._loop_task, return_exceptions=True)


async def run_bursts(w: Workload, steps: int, warmup: int, **kw) -> tuple[list[BurstResult], float]:
    """Warmup bursts, then ``steps`` timed bursts, each on a fresh pre-built shard."""
    shards = [Shard(w, seed=i, **kw) for i in range(warmup + steps)]
    for s in shards:
        await s.start()
    for i in range(warmup):
        await shards[i].burst(f"w{i}")
    t0 = time.perf_counter()
    res = [await shards[warmup + i].burst(f"s{i}") for i in range(steps)]
    total = time.perf_counter() - t0
    for s in shards:
        await s.stop()
    return res, total
