"""Burst harness: pods created through the (fake) apiserver at t0, latency = pod
creation → binding acknowledged by the apiserver (BASELINE.md measurement protocol).

A :class:`Shard` is one scheduler process-worth of state: its own apiserver, cluster
(nodes + Scv telemetry) and scheduler instance. The fake apiserver runs in the same
process and event loop, so its CPU cost (create, watch fan-out, bind) is charged to the
measured throughput — a conservative setup compared with a real, separate apiserver.
"""
from __future__ import annotations

import asyncio
import json
import os
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
                 device: str = "auto", overlap: str = "auto", engine_threads: int = 1,
                 device_index: int = 0) -> dict:
    """The shipped deploy profile (yoda at filter + score weight 300 on top of the
    upstream defaults) with the yoda QueueSort enabled (Q7) and the given client QPS.
    ``device_index`` is the HIP ordinal the gfx950 device scorer runs on: a rank of a
    multi-GPU bench passes its LOCAL_RANK, so rank r scores on GPU r."""
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
            "yodaRuntime": {"batchSize": batch, "bindConcurrency": 256, "deviceScorer": {"enabled": device, "device": device_index},
                            "overlapEngine": overlap, "engineThreads": engine_threads},
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
                 compat: bool = False, seed: int = 0, engine_threads: int = 1, device: str = "auto",
                 overlap: str = "auto", device_index: int = 0) -> None:
        self.w = w
        self.server = FakeApiServer()
        self.client = InProcessClient(self.server)
        populate(self.server, w, template, link_load=0.2 if w.id == 5 else 0.0, seed=seed)
        cfg = parse_config(bench_config(w.scheduler_name, qps, burst, batch, compat, device, overlap,
                                        device_index=device_index))
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
        objs = [pod_object(i, lab, w.scheduler_name, prefix=tag, spec=w.specs.get(i), meta=w.metas.get(i))
                for i, lab in enumerate(w.pods)]
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
            if not w.wait_bound and not q._active_entries and self.sched.pending_binds == 0 and \
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


class _Recorder:
    """Collects ``create`` calls of :func:`populate` so they can be replayed over HTTP."""

    def __init__(self) -> None:
        self.objs: list[tuple[str, dict]] = []

    def create(self, res: str, obj: dict, namespace=None) -> dict:
        self.objs.append((res, obj))
        return obj


def native_apiserver_binary() -> str:
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    # YODA_FAKEAPI_BIN: another build of the native fake apiserver (same-box A/B)
    return os.environ.get("YODA_FAKEAPI_BIN") or os.path.join(root, "_native", "yoda-fake-apiserver-native")


class HttpShard:
    """The same burst over real HTTP/JSON: the fake apiserver runs in its own process and
    the scheduler talks to it through the production client
    (:class:`~yoda_scheduler_amd.kube.client.KubeClient`: list/watch streams, binding
    POSTs — on the native C++ transport when it is built). The apiserver creates the pods
    and measures latency on its own clock. Between bursts it deletes the previous burst's
    pods, which releases their reservations through the scheduler's informer.

    ``apiserver="native"`` (default) is the C++ epoll fake apiserver
    (``native/kube/fakeapi.cpp``): pre-encoded watch frames, ~µs per request, so the
    measurement is the scheduler's. ``"python"`` is the aiohttp fake apiserver
    (``yoda-fake-apiserver``), the semantic reference, whose own CPU caps the burst."""

    def __init__(self, w: Workload, qps: float = 5000.0, burst: int = 10000, batch: int = 256,
                 template: Optional[dict] = None, events: bool = True, compat: bool = False, seed: int = 0,
                 device: str = "auto", overlap: str = "auto", apiserver: str = "native",
                 client_native: str | bool = "auto", engine_threads: int = 1, device_index: int = 0) -> None:
        import json
        import os
        import subprocess
        import sys
        import tempfile
        self.w = w
        self.apiserver = apiserver
        self.client_native = client_native
        self._dir = tempfile.mkdtemp(prefix="yoda-bench-")
        self.port_file = f"{self._dir}/port"
        self.template = template
        if apiserver == "native":
            exe = native_apiserver_binary()
            if not os.path.exists(exe):
                raise RuntimeError(f"{exe} is not built (python -m yoda_scheduler_amd.ops.build)")
            cmd = [exe, "--port", "0", "--port-file", self.port_file]
            env = None
            if "YODA_BENCH_ORIG_GLIBC_TUNABLES" in os.environ:
                # bench.py set the scheduler's malloc tunable for its own process: the fake
                # apiserver (the test double of kube-apiserver) runs as it was started
                env = {k: v for k, v in os.environ.items() if k != "GLIBC_TUNABLES"}
                if os.environ["YODA_BENCH_ORIG_GLIBC_TUNABLES"]:
                    env["GLIBC_TUNABLES"] = os.environ["YODA_BENCH_ORIG_GLIBC_TUNABLES"]
        else:
            cmd = [sys.executable, "-m", "yoda_scheduler_amd.cmd.fakeapi", "--port", "0", "--bench-config",
                   str(w.id), "--seed", str(seed), "--port-file", self.port_file]
            if template:
                cmd += ["--template", json.dumps(template)]
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            env = dict(os.environ, PYTHONPATH=os.pathsep.join(p for p in (root, os.environ.get("PYTHONPATH")) if p))
        self.proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env)
        self.cfg = parse_config(bench_config(w.scheduler_name, qps, burst, batch, compat, device, overlap,
                                             engine_threads, device_index))
        self.events, self.seed = events, seed
        self.sched: Optional[Scheduler] = None
        self.client = None
        self._loop_task: Optional[asyncio.Task] = None
        self._bursts = 0

    async def _port(self, timeout: float = 120.0) -> int:
        import os
        t = time.monotonic() + timeout
        while time.monotonic() < t:
            if os.path.exists(self.port_file):
                with open(self.port_file) as f:
                    return int(f.read())
            if self.proc.poll() is not None:
                raise RuntimeError(f"fake apiserver exited: {self.proc.stderr.read().decode()[-2000:]}")
            await asyncio.sleep(0.05)
        raise TimeoutError("fake apiserver did not start")

    async def start(self) -> None:
        import aiohttp

        from ..kube.client import KubeClient, KubeConfig
        port = await self._port()
        self.base = f"http://127.0.0.1:{port}"
        self.client = KubeClient(KubeConfig(self.base), native=self.client_native)
        self._http = aiohttp.ClientSession()
        if self.apiserver == "native":
            # the cluster (nodes + Scv telemetry) and the burst's pod templates, over HTTP
            rec = _Recorder()
            populate(rec, self.w, self.template, link_load=0.2 if self.w.id == 5 else 0.0, seed=self.seed)
            for res, obj in rec.objs:
                await self.client.create(res, obj)
            pods = [pod_object(i, lab, self.w.scheduler_name, prefix="t", spec=self.w.specs.get(i),
                               meta=self.w.metas.get(i))
                    for i, lab in enumerate(self.w.pods)]
            await self._call("POST", "/debug/bench/load", {"pods": pods})
        self.sched = Scheduler(self.client, self.cfg, metrics=NullMetrics(), record_events=self.events,
                               seed=self.seed)
        self.sched.e2e_samples = []
        await self.sched.start()
        self._loop_task = asyncio.get_event_loop().create_task(self.sched.scheduling_loop())

    async def _call(self, method: str, path: str, body: Optional[dict] = None) -> dict:
        """A /debug/bench control request. Over the scheduler's own native transport when it
        has one (a C++ round trip, ≈ 50 µs, instead of ≈ 0.3 ms through aiohttp — three per
        timed step); YODA_BENCH_CTL=aiohttp forces the Python client."""
        nat = getattr(self.client, "native", None) if self.client is not None else None
        if nat is not None and os.environ.get("YODA_BENCH_CTL", "native") == "native":
            data = json.dumps(body).encode() if body is not None else b""
            status, out = await nat.request(method, path, data, "application/json" if data else "", limited=False)
            if status < 200 or status >= 300:
                raise RuntimeError(f"{method} {path}: HTTP {status} {out[:200]!r}")
            return json.loads(out)
        async with self._http.request(method, self.base + path, json=body) as r:
            r.raise_for_status()
            return await r.json()

    async def burst(self, tag: str = "b", timeout: float = 600.0) -> BurstResult:
        sched = self.sched
        q = sched.queue
        self.last_reset_s = 0.0
        hook = getattr(self, "phase_hook", None)   # profilers: hook("reset" | "burst", started)
        if self._bursts:
            tr = time.perf_counter()
            if hook:
                hook("reset", True)
            await self._call("POST", "/debug/bench/reset")
            self.last_reset_post_s = time.perf_counter() - tr
            trace = [] if os.environ.get("YODA_BENCH_RUNLOG") else None
            if os.environ.get("YODA_BENCH_LOOPDEBUG"):
                # name the event-loop callbacks that hold the loop during the reset
                import logging
                import sys
                lg = logging.getLogger("asyncio")
                lg.setLevel(logging.WARNING)
                if not lg.handlers:
                    lg.addHandler(logging.StreamHandler(sys.stderr))
                    lg.propagate = False
                lp = asyncio.get_event_loop()
                lp.slow_callback_duration = 0.0003
                lp.set_debug(True)
            if sched.lane is not None and trace is not None:
                # runlog: the drain curve (ms, lane-owned pods, watch events decoded) every 0.2 ms
                # (+ the I/O thread's watch-decode CPU ms and the watch bytes read since the POST)
                nat = getattr(self.client, "native", None)
                s0 = nat.stats() if nat is not None else {}
                drain = self.last_reset_drain = []
                while True:
                    owned = sched.lane_owned()
                    s1 = nat.stats() if nat is not None else {}
                    drain.append((round((time.perf_counter() - tr) * 1e3, 3), owned,
                                  s1.get("watch_events", 0) - s0.get("watch_events", 0),
                                  round((s1.get("watch_cpu_s", 0.0) - s0.get("watch_cpu_s", 0.0)) * 1e3, 3),
                                  s1.get("watch_bytes", 0) - s0.get("watch_bytes", 0)))
                    if not owned or time.perf_counter() - tr > 60.0:
                        break
                    await asyncio.sleep(0.0002)
            elif sched.lane is not None:
                # woken by the lane when its last pod is released (an asyncio sleep shorter than
                # a millisecond still waits for epoll's 1 ms tick when nothing else wakes the loop)
                await sched.lane.wait_unowned(60.0)
            # the pods the Python side owns (a mirror of lane pods does not count: the lane's own
            # count covers them, and syncing the mirror here would switch the lane's change log
            # on and charge a Python copy of every lane pod to each timed step)
            # (YODA_BENCH_RESET_SYNC=1 restores round 3's sync in this loop: same-box A/B only)
            old_sync = os.environ.get("YODA_BENCH_RESET_SYNC") == "1"
            # (a populated cluster's bound pods — `--prefill` — stay: they are not the burst's)
            keep = sum(1 for res, _o in self.w.objects if res == "pods")
            while ((old_sync and sched.cache.sync_lane() >= 0 and len(sched.cache.pods) > keep)
                   or sched.cache.python_pods() > keep
                   or q._active_entries or sched.pending_binds or sched.lane_owned()):
                if trace is not None:
                    trace.append((round((time.perf_counter() - tr) * 1e3, 3), sched.lane_owned(), len(sched.cache.pods),
                                  len(q._active_entries), sched.pending_binds))
                await asyncio.sleep(0.0002)     # the deletes reached the scheduler
                if trace is not None:
                    trace.append((round((time.perf_counter() - tr) * 1e3, 3),))
            self.last_reset_trace = trace
            if os.environ.get("YODA_BENCH_LOOPDEBUG"):
                asyncio.get_event_loop().set_debug(False)
            self.last_reset_s = time.perf_counter() - tr
            if hook:
                hook("reset", False)
        self._bursts += 1
        sched.take_lane_samples()
        sched.e2e_samples.clear()
        # every step is an independent burst: the client's token bucket starts full, as
        # in the in-process harness where each step is a fresh scheduler
        cc = self.cfg.client_connection
        self.client.set_rate(cc.qps, cc.burst)
        done0 = sched.scheduled
        if sched.lane is not None:
            sched.lane.lane.run_log()           # drop the reset's runs
        t_burst = time.monotonic()
        n = (await self._call("POST", "/debug/bench/burst", {"tag": tag}))["n"]
        deadline = time.monotonic() + timeout
        # completion is observed locally (every bind acknowledged, or every pod parked):
        # no polling requests charged to the scheduler process during the burst. With the
        # native lane the loop sleeps until the lane's acknowledged count reaches the burst
        # (an eventfd wake-up, not a poll); the poll below then only settles the remainder.
        def parked() -> bool:
            # every pod bound or parked (unschedulable: in the lane's own unschedulableQ /
            # backoffQ, or handed to the Python queue)
            bound = sched.scheduled - done0
            waiting = sched.lane.waiting() if sched.lane is not None else 0
            return not q._active_entries and sched.pending_binds == 0 and \
                bound + len(q._unsched) + len(q._backoff_pods) + waiting >= n
        if sched.lane is not None:
            # woken when the acknowledged count (lane + Python path) crosses the burst; a burst
            # with unschedulable pods never gets there, so the parked check runs between waits
            target = done0 + n
            while time.monotonic() < deadline:
                if await sched.lane.wait_scheduled(target, min(0.02, max(0.0, deadline - time.monotonic()))):
                    break
                if parked():
                    break
        while time.monotonic() < deadline:
            if sched.scheduled - done0 >= n or parked():
                break
            await asyncio.sleep(0.0005)
        t_seen = time.monotonic()
        st = await self._call("GET", "/debug/bench/status?full=" + ("2" if os.environ.get("YODA_BENCH_RUNLOG") else "1"))
        self.last_timeline = st.get("timeline")
        sched.take_lane_samples()
        # the lane's runs of this burst, ms from the burst request: (pick, worker start, worker
        # end, lane done, pods), and when the scheduler saw the last acknowledgement
        self.last_runs = ([tuple(round((x - t_burst) * 1e3, 3) if x else 0.0 for x in r[:4]) + (r[4],)
                           for r in sched.lane.lane.run_log()] if sched.lane is not None else [])
        self.last_seen_ms = round((t_seen - t_burst) * 1e3, 3)
        return BurstResult(n, st["bound"], n - st["bound"], st["elapsed"], st["latencies"],
                           list(sched.e2e_samples))

    async def api_prof(self) -> dict:
        """The fake apiserver's cumulative event-loop seconds and counts by request kind."""
        st = await self._call("GET", "/debug/bench/status")
        return st.get("prof_s", {})

    async def stop(self) -> None:
        import shutil
        if self.sched is not None:
            await self.sched.shutdown()
        if self._loop_task:
            self._loop_task.cancel()
            await asyncio.gather(self._loop_task, return_exceptions=True)
        if self.client is not None:
            await self.client.close()
            await self._http.close()
        self.proc.terminate()
        try:
            self.proc.wait(10)
        except Exception:  # noqa: BLE001
            self.proc.kill()
        shutil.rmtree(self._dir, ignore_errors=True)
