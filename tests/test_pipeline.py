"""Overlapped engine batches (yodaRuntime.overlapEngine): when the active queue is empty
while a batch is in flight, the scheduling loop waits for whichever comes first — a pod
reaching the queue or the batch's result (``Scheduler._await_pods_or_result``) — so pods
that arrive while the engine (the GPU, with the device scorer) works are submitted behind
the running batch instead of after its result has been applied."""
import asyncio
import threading
import time

from yoda_scheduler_amd.testing import FakeCluster, yoda_config


class SlowEngine:
    """The scheduler's engine with a slow ``schedule_batch`` (a stand-in for a device batch):
    not the native class, so batches go to the executor path."""

    def __init__(self, eng, delay: float) -> None:
        self._eng, self._delay = eng, delay
        self.calls: list = []
        self._mu = threading.Lock()

    def __getattr__(self, k):
        return getattr(self._eng, k)

    def schedule_batch(self, ids, reqs):
        t0 = time.perf_counter()
        time.sleep(self._delay)
        out = self._eng.schedule_batch(ids, reqs)
        with self._mu:
            self.calls.append((t0, time.perf_counter(), len(ids)))
        return out


def test_pods_arriving_during_a_batch_are_submitted_behind_it():
    async def go():
        cfg = yoda_config(batch=64)
        cfg["yodaRuntime"]["overlapEngine"] = "on"
        c = FakeCluster(cfg)
        for i in range(2):
            c.add_node(f"n{i}")
        await c.start()
        sched = c.sched
        sched.engine = SlowEngine(sched.engine, 0.15)
        submits: list = []
        orig = sched._submit_engine_batch

        def submit(loop, ids, reqs):
            fut = orig(loop, ids, reqs)
            submits.append((time.perf_counter(), len(ids), len(sched._inflight)))
            return fut
        sched._submit_engine_batch = submit
        for i in range(4):
            c.add_pod(f"a{i}", {"scv/memory": "1024"})
        await c.wait(lambda: len(submits) >= 1, 5.0, 0.002)
        await asyncio.sleep(0.02)                 # the first batch is on the engine now
        for i in range(20):
            c.add_pod(f"b{i}", {"scv/memory": "1024"})
        names = [f"a{i}" for i in range(4)] + [f"b{i}" for i in range(20)]
        ok = await c.wait(lambda: all(c.node_of(p) for p in names), 10.0, 0.005)
        calls = list(sched.engine.calls)
        await c.stop()
        return ok, submits, calls
    ok, submits, calls = asyncio.run(go())
    assert ok
    assert len(submits) >= 2
    first_done = calls[0][1]
    # the second batch was handed to the engine while the first one was still running
    assert submits[1][2] >= 1 and submits[1][0] < first_done, (submits, calls)


class FlakyEngine(SlowEngine):
    """``schedule_batch`` raises on its first call (after reserving nothing)."""

    def __init__(self, eng) -> None:
        super().__init__(eng, 0.0)
        self.failures = 0

    def schedule_batch(self, ids, reqs):
        if self.failures == 0:
            self.failures += 1
            raise RuntimeError("injected engine failure")
        return super().schedule_batch(ids, reqs)


def test_failed_engine_batch_requeues_its_pods_and_the_loop_keeps_going():
    async def go():
        cfg = yoda_config(batch=64, backoff=0.01, max_backoff=0.05)
        cfg["yodaRuntime"]["overlapEngine"] = "on"
        c = FakeCluster(cfg)
        c.add_node("n0")
        await c.start()
        sched = c.sched
        sched.engine = FlakyEngine(sched.engine)
        names = [f"p{i}" for i in range(12)]
        for n in names:
            c.add_pod(n, {"scv/memory": "1024"})
        ok = await c.wait(lambda: all(c.node_of(p) for p in names), 10.0, 0.005)
        errors, failures = sched.engine_batch_errors, sched.engine.failures
        ledger = sched.engine.ledger_size
        await c.stop()
        return ok, errors, failures, ledger
    ok, errors, failures, ledger = asyncio.run(go())
    assert ok and errors == 1 and failures == 1 and ledger == 12


def test_failed_inline_engine_batch_requeues_its_pods():
    async def go():
        cfg = yoda_config(batch=64, backoff=0.01, max_backoff=0.05)
        cfg["yodaRuntime"]["overlapEngine"] = "off"
        c = FakeCluster(cfg)
        c.add_node("n0")
        await c.start()
        sched = c.sched
        sched.engine = FlakyEngine(sched.engine)
        names = [f"q{i}" for i in range(12)]
        for n in names:
            c.add_pod(n, {"scv/memory": "1024"})
        ok = await c.wait(lambda: all(c.node_of(p) for p in names), 10.0, 0.005)
        errors = sched.engine_batch_errors
        await c.stop()
        return ok, errors
    ok, errors = asyncio.run(go())
    assert ok and errors == 1
