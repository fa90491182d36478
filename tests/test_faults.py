"""Failure detection / fault injection: apiserver faults (dropped watches,
latency, bind 409/500) and amd-smi faults (uncorrectable ECC, xGMI link down, HBM
consumed behind the scheduler's back) with end-state invariants: every pod bound exactly
once, no GPU over-reserved, the ledger equal to the annotations, unhealthy GPUs unused."""
import asyncio
import random

from yoda_scheduler_amd.fakeapi.server import Faults
from yoda_scheduler_amd.models.device import make_node
from yoda_scheduler_amd.sniffer.collector import FakeBackend
from yoda_scheduler_amd.sniffer.publisher import SnifferAgent
from yoda_scheduler_amd.testing import FakeCluster, yoda_config


def run(c):
    return asyncio.run(c)


def _ledger_invariants(c, pods):
    """Per GPU: reserved == Σ scv/memory of the pods annotated onto it, and ≤ total."""
    want: dict = {}
    for name, mem in pods.items():
        node = c.node_of(name)
        for g in c.gpus_of(name):
            want[(node, g)] = want.get((node, g), 0) + mem
    for node in {n for n, _ in want}:
        for g, st in enumerate(c.sched.cache.node_gpu_state(node)):
            assert st["reserved"] == want.get((node, g), 0), (node, g, st, want.get((node, g)))
            assert st["reserved"] <= st["total"]


def test_burst_survives_watch_drops_latency_and_bind_faults():
    faults = Faults(drop_watch_every=97, latency_s=0.0002, bind_conflict_ratio=0.08, bind_fail_ratio=0.05, seed=7)

    async def go():
        c = FakeCluster(yoda_config(backoff=0.01, max_backoff=0.05), faults=faults)
        for i in range(4):
            c.add_node(f"n{i}")
        await c.start()
        rng = random.Random(3)
        pods = {}
        for i in range(240):
            mem = rng.choice([2048, 8192, 16384])
            lab = {"scv/memory": str(mem)}
            if i % 7 == 0:
                lab["scv/number"] = "2"
            c.add_pod(f"p{i}", lab)
            pods[f"p{i}"] = mem
        ok = await c.wait(lambda: all(c.node_of(p) for p in pods), 30.0, 0.01)
        await asyncio.sleep(0.1)               # let the informer confirm the last binds
        relists = sum(inf.relists for inf in c.sched.informers.values())
        bind_errors = c.sched.bind_errors
        _ledger_invariants(c, pods)
        await c.stop()
        return ok, relists, bind_errors, c.server.calls["bind"]
    ok, relists, bind_errors, binds = run(go())
    assert ok
    assert relists > 0                      # watches really dropped and were re-established
    assert bind_errors > 0 and binds > 240  # injected failures were retried


def test_overlapped_engine_batches_keep_ledger_exact():
    """yodaRuntime.overlapEngine: native batches run on the engine's native worker thread while the
    event loop binds, retries failed binds (engine release) and ingests node updates (engine
    upserts) — the process-wide engine lock keeps every reservation exact."""
    faults = Faults(bind_conflict_ratio=0.05, bind_fail_ratio=0.05, seed=11)

    async def go():
        cfg = yoda_config(backoff=0.01, max_backoff=0.05, batch=32)
        cfg["yodaRuntime"]["overlapEngine"] = "on"
        c = FakeCluster(cfg, faults=faults)
        for i in range(4):
            c.add_node(f"n{i}")
        await c.start()
        rng = random.Random(5)
        pods = {}
        for i in range(400):
            mem = rng.choice([1024, 4096, 8192])
            lab = {"scv/memory": str(mem)}
            if i % 5 == 0:
                lab["scv/number"] = "2"
            c.add_pod(f"p{i}", lab)
            pods[f"p{i}"] = mem
            if i % 50 == 25:              # node churn while batches are in flight
                c.server.patch("nodes", f"n{i % 4}", {"metadata": {"labels": {"tick": str(i)}}})
                await asyncio.sleep(0)
        ok = await c.wait(lambda: all(c.node_of(p) for p in pods), 30.0, 0.01)
        await asyncio.sleep(0.1)
        # batches ran on the native engine worker thread (core.BatchWorker), not inline
        overlapped = c.sched._batch_worker is not None and c.sched._engine_exec is None
        _ledger_invariants(c, pods)
        await c.stop()
        return ok, overlapped, c.sched.bind_errors
    ok, overlapped, bind_errors = run(go())
    assert ok and overlapped and bind_errors > 0


def test_amdsmi_faults_steer_placement():
    """GPU 3 reports an uncorrectable ECC error, GPU 5 an xGMI link down, and something
    outside the scheduler filled GPU 0's HBM: none of them may receive pods."""
    async def go():
        c = FakeCluster(yoda_config(yoda_args={"sampleSettleSeconds": 0.0}))
        c.server.create("nodes", make_node("gpu-node"))
        be = FakeBackend(gpus=8, seed=1)
        be.state[3].ecc_uncorrectable = 2
        be.state[5].links_down = 1
        be.state[0].used_mb = be.spec.hbm_mb - 1000
        agent = SnifferAgent(c.client, "gpu-node", be, interval=60.0)
        await agent.publish_once()
        await c.start()
        for i in range(10):
            c.add_pod(f"w{i}", {"scv/memory": "20000"})
        await c.wait_bound(10)
        used = sorted({g for i in range(10) for g in c.gpus_of(f"w{i}")})
        # ECC clears, link recovers: the next sample makes those GPUs schedulable again
        be.state[3].ecc_uncorrectable = 0
        be.state[5].links_down = 0
        await agent.publish_once()
        await asyncio.sleep(0.05)
        health = [g["healthy"] for g in c.sched.cache.node_gpu_state("gpu-node")]
        await c.stop()
        return used, health
    used, health = run(go())
    assert used and not {0, 3, 5} & set(used)
    assert all(health)


def test_gpu_fault_mid_burst_moves_new_pods_off_the_card():
    async def go():
        c = FakeCluster(yoda_config(yoda_args={"sampleSettleSeconds": 0.0}))
        c.server.create("nodes", make_node("gpu-node"))
        be = FakeBackend(gpus=8, seed=2)
        agent = SnifferAgent(c.client, "gpu-node", be, interval=60.0)
        await agent.publish_once()
        await c.start()
        for i in range(16):
            c.add_pod(f"a{i}", {"scv/memory": "1000"})
        await c.wait_bound(16)
        be.state[2].ecc_uncorrectable = 1
        await agent.publish_once()
        await asyncio.sleep(0.05)
        for i in range(16):
            c.add_pod(f"b{i}", {"scv/memory": "1000"})
        await c.wait_bound(32)
        before = {g for i in range(16) for g in c.gpus_of(f"a{i}")}
        after = {g for i in range(16) for g in c.gpus_of(f"b{i}")}
        await c.stop()
        return before, after
    before, after = run(go())
    assert 2 in before and 2 not in after


def test_apiserver_outage_then_recovery():
    """Binds fail for a while (every call 500), then the apiserver recovers: pods back off
    and all get bound exactly once."""
    async def go():
        faults = Faults(bind_fail_ratio=1.0)
        c = FakeCluster(yoda_config(backoff=0.01, max_backoff=0.05), faults=faults)
        c.add_node("n0")
        await c.start()
        for i in range(20):
            c.add_pod(f"p{i}", {"scv/memory": "1000"})
        await asyncio.sleep(0.3)
        during = len(c.server.bind_log)
        faults.bind_fail_ratio = 0.0
        ok = await c.wait_bound(20, 10.0)
        _ledger_invariants(c, {f"p{i}": 1000 for i in range(20)})
        await c.stop()
        return during, ok, c.sched.bind_errors
    during, ok, errors = run(go())
    assert during == 0 and ok and errors >= 20
