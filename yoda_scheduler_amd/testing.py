"""Test / demo helpers: an in-process cluster (fake apiserver + synthetic MI355X nodes +
scheduler) driven from asyncio code."""
from __future__ import annotations

import asyncio
import time
from typing import Optional

from .fakeapi.client import InProcessClient
from .fakeapi.server import FakeApiServer, Faults
from .framework.config import parse_config
from .framework.registry import Registry
from .framework.scheduler import Scheduler
from .models.device import MI355X, GpuSpec, make_node, make_scv
from .utils.metrics import SchedulerMetrics


def yoda_config(name: str = "yoda-scheduler", *, compat: bool = False, backoff: float = 0.05,
                max_backoff: float = 0.2, extra_filter: Optional[list] = None, extra_score: Optional[list] = None,
                yoda_args: Optional[dict] = None, qps: float = 0, batch: int = 64, pct: int = 0,
                leader_elect: bool = False) -> dict:
    args = dict(yoda_args or {})
    if compat:
        args["compat"] = True
    return {
        "apiVersion": "kubescheduler.config.k8s.io/v1beta1", "kind": "KubeSchedulerConfiguration",
        "leaderElection": {"leaderElect": leader_elect, "resourceName": "yoda-scheduler",
                           "leaseDuration": "1s", "renewDeadline": "0.6s", "retryPeriod": "0.1s"},
        "clientConnection": {"qps": qps, "burst": 100},
        "percentageOfNodesToScore": pct,
        "podInitialBackoffSeconds": backoff, "podMaxBackoffSeconds": max_backoff,
        "yodaRuntime": {"batchSize": batch, "bindConcurrency": 16, "unschedulableFlushSeconds": 5},
        "profiles": [{
            "schedulerName": name,
            "plugins": {"queueSort": {"enabled": [{"name": "yoda"}], "disabled": [{"name": "*"}]},
                        "filter": {"enabled": [{"name": "yoda"}] + [{"name": n} for n in (extra_filter or [])]},
                        "score": {"enabled": [{"name": "yoda", "weight": 300}] +
                                  [{"name": n, "weight": 1} for n in (extra_score or [])]}},
            "pluginConfig": [{"name": "yoda", "args": args}],
        }],
    }


class FakeCluster:
    def __init__(self, config: Optional[dict] = None, registry: Optional[Registry] = None,
                 faults: Optional[Faults] = None, server: Optional[FakeApiServer] = None, seed: int = 0) -> None:
        self.server = server or FakeApiServer(faults=faults)
        self.client = InProcessClient(self.server)
        self.config = parse_config(config or yoda_config())
        self.registry = registry
        self.seed = seed
        self.sched: Optional[Scheduler] = None
        self._loop_task: Optional[asyncio.Task] = None

    # ------------------------------------------------------------------ objects
    def add_node(self, name: str, gpus: int = 8, spec: GpuSpec = MI355X, used_mb: Optional[list] = None,
                 scv: bool = True, labels: Optional[dict] = None, taints: Optional[list] = None,
                 interval_ms: int = 60_000, **kw) -> None:
        self.server.create("nodes", make_node(name, labels=labels, taints=taints))
        if scv:
            s = make_scv(name, spec, gpus, update_time=time.time(), used_mb=used_mb, **kw)
            s.update_interval_ms = interval_ms
            self.server.create("scvs", s.to_json())

    def scv_obj(self, name: str) -> dict:
        return self.server.get("scvs", name)

    def add_pod(self, name: str, labels: Optional[dict] = None, scheduler: str = "yoda-scheduler",
                priority: int = 0, ns: str = "default", **spec_extra) -> dict:
        spec = {"schedulerName": scheduler, "containers": [{"name": "c", "image": "x"}], **spec_extra}
        if priority:
            spec["priority"] = priority
        return self.server.create("pods", {"metadata": {"name": name, "namespace": ns, "labels": dict(labels or {})},
                                           "spec": spec})

    def pod(self, name: str, ns: str = "default") -> dict:
        return self.server.get("pods", name, ns)

    def node_of(self, name: str) -> str:
        return (self.pod(name).get("spec") or {}).get("nodeName", "")

    def gpus_of(self, name: str) -> list[int]:
        v = ((self.pod(name).get("metadata") or {}).get("annotations") or {}).get("scv.amd.com/gpus", "")
        return [int(x) for x in v.split(",") if x]

    # ------------------------------------------------------------------ scheduler
    async def start(self, **kw) -> Scheduler:
        self.sched = Scheduler(self.client, self.config, self.registry, metrics=SchedulerMetrics(), seed=self.seed,
                               **kw)
        await self.sched.start()
        self._loop_task = asyncio.get_event_loop().create_task(self.sched.scheduling_loop())
        return self.sched

    async def wait(self, cond, timeout: float = 5.0, step: float = 0.002) -> bool:
        t = time.monotonic() + timeout
        while time.monotonic() < t:
            if cond():
                return True
            await asyncio.sleep(step)
        return bool(cond())

    async def wait_bound(self, n: int, timeout: float = 5.0) -> bool:
        return await self.wait(lambda: len(self.server.bind_log) >= n, timeout)

    async def stop(self) -> None:
        if self.sched is not None:
            await self.sched.shutdown()
        if self._loop_task is not None:
            self._loop_task.cancel()
            await asyncio.gather(self._loop_task, return_exceptions=True)


class NativeApiServerProcess:
    """The native C++ fake apiserver (``yoda-fake-apiserver-native``) as a child process
    for tests and tools; ``url`` once started, ``stop()`` terminates it."""

    def __init__(self, token: str = "", history: int = 0, extra: Optional[list] = None) -> None:
        import os
        import subprocess
        import tempfile

        from .bench.harness import native_apiserver_binary
        d = tempfile.mkdtemp(prefix="yoda-nfa-")
        pf = os.path.join(d, "port")
        cmd = [native_apiserver_binary(), "--port", "0", "--port-file", pf]
        if history:
            cmd += ["--history", str(history)]
        if token:
            cmd += ["--token", token]
        cmd += list(extra or [])
        self.proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL)
        t = time.time()
        while not os.path.exists(pf):
            if self.proc.poll() is not None or time.time() - t > 15:
                raise RuntimeError("native fake apiserver did not start")
            time.sleep(0.01)
        with open(pf) as f:
            self.port = int(f.read())
        self.url = f"http://127.0.0.1:{self.port}"

    def stop(self) -> None:
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(10)
            except Exception:  # noqa: BLE001
                self.proc.kill()
